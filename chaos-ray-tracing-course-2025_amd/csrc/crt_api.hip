/*
 * crt_api.hip — the extern "C" entry points of include/crt_hip.h: scene
 * upload / create / destroy, render (host and device buffers), shards and
 * their unpack, the trace hook, work counters and options.  Replaces
 * crt::render_image (src/core/crt_renderer.cpp:157-199) for the reference's
 * callers (src/standalone/main.cpp:38, src/python/py_crt_module.cpp:100).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <future>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "crt_lbvh.h"
#include "crt_scene_impl.h"
#include "crt_tree_build.h"

namespace {

constexpr int kStageChunks = 8;

bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

/* hipEventQuery until the event is reached (the copy's host threads poll:
 * a blocking wait may sleep past a ~10 us chunk). */
hipError_t spin_event(hipEvent_t e) {
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipErrorNotReady) return r;
        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
    }
}

/* The whole image through the pinned staging copy in chunks, each chunk copied
 * on to the caller's buffer by a pool thread as soon as its DMA is done (the
 * runtime would first page-lock a pageable caller buffer: ~10 ms for a
 * 1920x1080 image the first time, profiles/r03/cold).  Pinned caller memory:
 * one DMA. */
int image_to_host_full(crt_hip_scene *sc, float *dst, size_t nfl) {
    const size_t bytes = nfl * sizeof(float);
    if (!sc->h_stage || host_pinned(dst)) {
        HIP_TRY(hipMemcpyAsync(dst, sc->d_out, bytes, hipMemcpyDeviceToHost, sc->stream));
        HIP_TRY(hipStreamSynchronize(sc->stream));
        return CRT_OK;
    }
    const size_t step = ((bytes + kStageChunks - 1) / kStageChunks + 4095) & ~size_t(4095);
    int nc = 0;
    for (size_t off = 0; off < bytes; off += step, ++nc) {
        const size_t len = std::min(step, bytes - off);
        HIP_TRY(hipMemcpyAsync(reinterpret_cast<char *>(sc->h_stage) + off, reinterpret_cast<const char *>(sc->d_out) + off,
                               len, hipMemcpyDeviceToHost, sc->stream));
        HIP_TRY(hipEventRecord(sc->stage_ev[(size_t)nc], sc->stream));
    }
    struct Job {
        crt_hip_scene *sc;
        float *dst;
        size_t bytes, step;
        hipError_t err[kStageChunks];
    } job{sc, dst, bytes, step, {}};
    HostPool::get().run(nc, [](void *a, int i) {
        Job &j = *static_cast<Job *>(a);
        const size_t off = (size_t)i * j.step, len = std::min(j.step, j.bytes - off);
        j.err[i] = spin_event(j.sc->stage_ev[(size_t)i]);
        if (j.err[i] == hipSuccess)
            std::memcpy(reinterpret_cast<char *>(j.dst) + off, reinterpret_cast<const char *>(j.sc->h_stage) + off, len);
    }, &job);
    for (int i = 0; i < nc; ++i)
        if (job.err[i] != hipSuccess) return set_error(CRT_E_HIP, std::string("image copy: ") + hipGetErrorString(job.err[i]));
    return CRT_OK;
}

/* The compact copy's row records for the scene's frame height. */
int ensure_copy_rows(crt_hip_scene *sc) {
    const int H = sc->info.height;
    if (sc->h_rows && sc->copy_h == H) return CRT_OK;
    HIP_TRY(hipStreamSynchronize(sc->stream));
    if (sc->h_rows) (void)hipHostFree(sc->h_rows);
    if (sc->d_row_spans) (void)hipFree(sc->d_row_spans);
    sc->h_rows = nullptr;
    sc->d_row_spans = nullptr;
    sc->copy_h = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&sc->h_rows), (size_t)H * sizeof(HostRow), hipHostMallocDefault));
    HIP_TRY(hipMalloc(&sc->d_row_spans, (size_t)H * sizeof(int2)));
    if (!sc->spans_ev) HIP_TRY(hipEventCreateWithFlags(&sc->spans_ev, hipEventDisableTiming));
    if (!sc->copy_ev) HIP_TRY(hipEventCreateWithFlags(&sc->copy_ev, hipEventDisableTiming));
    for (hipEvent_t &e : sc->copy_band_ev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    sc->copy_h = H;
    return CRT_OK;
}

/* Device address of pinned (or registered) host memory, or null. */
void *device_view(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

/* A check for the copy's host threads to run while the frame renders
 * (render_checked): fn(arg, i, n) for i < n; any false sets `failed`. */
struct HostCheck {
    bool (*fn)(void *, int, int) = nullptr;
    void *arg = nullptr;
    std::atomic<bool> failed{false};
};

int image_to_host_full_checked(crt_hip_scene *sc, float *dst, size_t nfl, HostCheck *check) {
    if (check && check->fn) {   /* the check on the pool while the frame renders, then the copy */
        HostPool &pool = HostPool::get();
        pool.run(pool.threads(), [](void *a, int i) {
            HostCheck &c = *static_cast<HostCheck *>(a);
            if (!c.fn(c.arg, i, HostPool::get().threads())) c.failed = true;
        }, check);
    }
    return image_to_host_full(sc, dst, nfl);
}

/* The compact copy of the frame in d_out into host memory, queued behind the
 * frame on the scene's stream.  k_row_spans finds each row's span of
 * non-background pixels (into pinned row records); k_rows_to_host writes the
 * spans straight into host memory: into the caller's image when it is pinned,
 * else into the pinned staging image.  Meanwhile the host (HostPool, one band
 * of rows a thread) writes the background outside each span as soon as the
 * spans are known, and (staging) copies each span on once the spans are in
 * host memory.  Every pixel outside a row's span has the background's bits
 * (k_row_spans compares bits), so the caller's image equals d_out bit for
 * bit.  ~1/7 of C2's frame crosses PCIe. */
int image_to_host(crt_hip_scene *sc, float *dst, size_t nfl, HostCheck *check = nullptr) {
    const int W = sc->info.width, H = sc->info.height;
    if (!sc->compact_copy || !sc->h_stage || sc->grid_empty || W <= 0 || H <= 0 || (size_t)W * H * 3 != nfl)
        return image_to_host_full_checked(sc, dst, nfl, check);
    int rc = ensure_copy_rows(sc);
    if (rc != CRT_OK) return rc;
    float *dst_dev = static_cast<float *>(device_view(dst));
    float *target = dst_dev;
    if (!target && !(target = static_cast<float *>(device_view(sc->h_stage))))
        return image_to_host_full_checked(sc, dst, nfl, check);
    HostRow *rows_dev = static_cast<HostRow *>(device_view(sc->h_rows));
    if (!rows_dev) return image_to_host_full_checked(sc, dst, nfl, check);
    Rgb<uint32_t> bgb;
    std::memcpy(bgb.c, sc->ds.background, sizeof bgb.c);
    hipLaunchKernelGGL(k_row_spans, dim3((unsigned)H), dim3(256), 0, sc->stream, sc->d_out, W, bgb, sc->d_row_spans,
                       rows_dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(sc->spans_ev, sc->stream));
    /* into the staging image in bands of rows, so the host copies a band on
     * while the next ones cross PCIe; into the caller's pinned image at once */
    const bool staged = dst_dev == nullptr;
    const int G = staged ? std::min(4, H) : 1;
    for (int g = 0; g < G; ++g) {
        const int y0 = (int)((int64_t)H * g / G), y1 = (int)((int64_t)H * (g + 1) / G);
        hipLaunchKernelGGL(k_rows_to_host, dim3((unsigned)(y1 - y0)), dim3(256), 0, sc->stream, sc->d_out, W, H, y0,
                           sc->d_row_spans, target);
        HIP_TRY(hipGetLastError());
        if (g + 1 < G) HIP_TRY(hipEventRecord(sc->copy_band_ev[g], sc->stream));
    }
    HIP_TRY(hipEventRecord(sc->copy_ev, sc->stream));
    HostPool &pool = HostPool::get();
    const int nb = std::min(pool.threads(), H);
    struct Job {
        crt_hip_scene *sc;
        float *dst;
        bool staged;
        int W, H, nb, G;
        float bg[3];
        HostCheck *check;
        std::atomic<int> err{0};   /* a hipError_t of a copy kernel's event */
    } job;
    job.check = check && check->fn ? check : nullptr;
    job.sc = sc;
    job.dst = dst;
    job.staged = staged;
    job.G = G;
    job.W = W;
    job.H = H;
    job.nb = nb;
    std::memcpy(job.bg, sc->ds.background, sizeof job.bg);
    pool.run(nb, [](void *a, int b) {
        Job &j = *static_cast<Job *>(a);
        const int r0 = (int)((int64_t)j.H * b / j.nb), r1 = (int)((int64_t)j.H * (b + 1) / j.nb);
        const int64_t row = 3 * (int64_t)j.W;
        const HostRow *R = j.sc->h_rows;
        if (j.check && !j.check->fn(j.check->arg, b, j.nb)) j.check->failed = true;   /* while the GPU renders */
        auto wait = [&](hipEvent_t ev) -> bool {   /* poll: a blocking wait may sleep past the copy */
            for (;;) {
                const hipError_t e = hipEventQuery(ev);
                if (e == hipSuccess) return true;
                if (e != hipErrorNotReady) {
                    int z = 0;
                    j.err.compare_exchange_strong(z, (int)e);
                    return false;
                }
                if (j.err.load(std::memory_order_relaxed)) return false;
                for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
            }
        };
        if (!wait(j.sc->spans_ev)) return;
        for (int y = r0; y < r1; ++y) {   /* the background, while the spans cross PCIe */
            float *d = j.dst + y * row;
            const int x0 = R[y].x0, x1 = R[y].x1;
            fill_background(d, x0, j.bg);
            fill_background(d + 3 * (int64_t)x1, j.W - x1, j.bg);
        }
        if (j.staged) {
            /* the launches (bands of rows) that hold rows r0 .. r1 - 1 */
            for (int g = 0; g < j.G; ++g) {
                const int y0 = (int)((int64_t)j.H * g / j.G), y1 = (int)((int64_t)j.H * (g + 1) / j.G);
                if (y1 > r0 && y0 < r1 && !wait(g + 1 < j.G ? j.sc->copy_band_ev[g] : j.sc->copy_ev)) return;
            }
            for (int y = r0; y < r1; ++y)
                if (R[y].x1 > R[y].x0)
                    std::memcpy(j.dst + y * row + 3 * (int64_t)R[y].x0, j.sc->h_stage + y * row + 3 * (int64_t)R[y].x0,
                                (size_t)(R[y].x1 - R[y].x0) * 3 * sizeof(float));
        }
        store_fence();
    }, &job);
    const int err = job.err.load();
    const hipError_t e = err ? (hipError_t)err : spin_event(sc->copy_ev);
    if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("image copy: ") + hipGetErrorString(e));
    return CRT_OK;
}

}  // namespace

namespace crt_amd {

int UploadBatch::flush(crt_hip_scene *sc) {
    if (items_.empty()) return CRT_OK;
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, host_.size()));
    sc->allocs.push_back(p);
    HIP_TRY(hipMemcpy(p, host_.data(), host_.size(), hipMemcpyHostToDevice));
    for (const Item &it : items_) *it.dst = static_cast<const char *>(p) + it.off;
    sc->info.device_bytes += (int64_t)host_.size();
    items_.clear();
    host_.clear();
    return CRT_OK;
}

/* A prepared host scene into HBM of `device`.  primary = false: a further
 * replica of a multi-GPU handle (crt_multi.hip), which renders into the
 * gather buffers only — no output image, no pinned staging image. */
/* CRT_CREATE_TRACE builds (A/B): each step of scene_upload timed on stderr */
#ifdef CRT_CREATE_TRACE
#define CRT_CREATE_STAMP(what)                                                                                  \
    do {                                                                                                       \
        const auto t_ = std::chrono::steady_clock::now();                                                      \
        std::fprintf(stderr, "create %-10s %8.3f ms\n", what,                                                  \
                     std::chrono::duration<double, std::milli>(t_ - t_stamp).count());                         \
        t_stamp = t_;                                                                                          \
    } while (0)
#else
#define CRT_CREATE_STAMP(what) ((void)0)
#endif

int scene_upload(const HostScene &hs, int device, bool primary, crt_hip_scene **out) {
    *out = nullptr;
    const auto t_up = std::chrono::steady_clock::now();
#ifdef CRT_CREATE_TRACE
    auto t_stamp = t_up;
#endif
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_error(CRT_E_INVALID, "no such HIP device");
    HIP_TRY(hipSetDevice(device));
    /* the pinned staging image (copies into pageable memory, image_to_host):
     * page-locking 25 MB takes ~4 ms, so it runs beside the rest of the upload */
    const size_t out_bytes = (size_t)hs.width * hs.height * 3 * sizeof(float);
    const bool want_stage = primary && out_bytes > 0;
    std::future<std::pair<hipError_t, float *>> stage_f;
    if (want_stage)
        stage_f = std::async(std::launch::async, [device, out_bytes]() {
            float *p = nullptr;
            hipError_t e = hipSetDevice(device);
            if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&p), out_bytes, hipHostMallocDefault);
            return std::make_pair(e, p);
        });
    /* joined on every return path: a staging image not taken by the scene (an
     * error, an empty bucket grid) is freed here */
    struct StageJoin {
        std::future<std::pair<hipError_t, float *>> *f;
        ~StageJoin() {
            if (f->valid()) {
                const auto r = f->get();
                if (r.second) (void)hipHostFree(r.second);
            }
        }
    } stage_join{&stage_f};
    std::unique_ptr<crt_hip_scene> sc(new crt_hip_scene());
    sc->device = device;
#ifdef CRT_AB_OPTIONS
    /* A/B builds only (scripts/make_variant.sh RENDER_FLAGS=-DCRT_AB_OPTIONS): environment
     * overrides of the options (crt_hip_scene_set_option names) */
    static const char *const kEnv[][2] = {{"CRT_TRAVERSAL", "traversal"}, {"CRT_SECONDARY", "secondary"},
                                           {"CRT_WAVEFRONT", "wavefront"}, {"CRT_GI_REFILL", "gi_refill"},
                                           {"CRT_WF_RPW", "wf_rpw"},       {"CRT_TRACE_WALK", "trace_walk"},
                                           {"CRT_CALIBRATE", "calibrate"}, {"CRT_WINDOW", "window"},
                                           {"CRT_EVENTS", "events"}};
    for (const auto &kv : kEnv)
        if (const char *e = std::getenv(kv[0]))
            if (crt_hip_scene_set_option(sc.get(), kv[1], std::atoi(e)) != CRT_OK) return CRT_E_INVALID;
    if (const char *e = std::getenv("CRT_CALIB_K")) {   /* a fixed split threshold instead of the tuned one */
        sc->calib_k = (float)std::atof(e);
        if (sc->calibrate) sc->calibrate = 2;
    }
    if (const char *e = std::getenv("CRT_BINS_MEAN_CAP")) sc->bins_mean_cap = std::max<int64_t>(1, std::atoll(e));
#endif
    sc->bvh_device = hs.device_bvh;   /* create flag CRT_SCENE_NO_DEVICE_BVH: none */
    if (hs.tree_on_host) sc->tile_work = tile_work_estimate(hs, (hs.width + 7) / 8, (hs.height + 7) / 8);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) {
            sc->wave_slots = prop.multiProcessorCount * 4 * 6;
            sc->refill_waves = prop.multiProcessorCount * 4 * CRT_GI_WAVES;
            int per_cu = 0;   /* resident blocks of the GI machine (registers, LDS) */
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_render_gi<false>, 256, 0) == hipSuccess &&
                per_cu > 0)
                sc->gi_blocks = prop.multiProcessorCount * per_cu;
        }
    }
    crt_host_scene_info(reinterpret_cast<const crt_host_scene *>(&hs), &sc->info);
    sc->info.device_bytes = 0;
    for (const DMaterial &m : hs.materials) {
        if (m.type == CRT_MATERIAL_REFLECTIVE || m.type == CRT_MATERIAL_REFRACTIVE) sc->has_secondary = true;
        if (m.type == CRT_MATERIAL_REFRACTIVE) sc->has_refractive = true;
        if (m.type == CRT_MATERIAL_DIFFUSE) sc->has_diffuse = true;
    }
    const bool gi_tables = hs.gi_on && sc->has_diffuse, pow5_table = hs.refractions_on && sc->has_refractive;
    start_host_tables(gi_tables, pow5_table);   /* background, overlapping the upload below */
    DeviceScene &ds = sc->ds;
    int rc;
    UploadBatch ub;   /* every host array of the scene: one allocation, one copy */
    ds.prune_origin_max = hs.prune_origin_max;
    if (hs.tree_on_host) {
        ub.add(hs.nodes, &ds.nodes);
        ds.node_count = (int32_t)hs.nodes.size();
        ub.add(hs.pnodes, &ds.pnodes);
        auto ok = [](float x) {
            const float m = std::fabs(x);
            return x == 0.0f || (m >= 0x1p-40f && m <= 0x1p62f);
        };
        ds.planes_ok = 1;
        for (const DNode &n : hs.nodes)
            if (!(ok(n.lo_x) && ok(n.lo_y) && ok(n.lo_z) && ok(n.hi_x) && ok(n.hi_y) && ok(n.hi_z) &&
                  n.lo_x <= n.hi_x && n.lo_y <= n.hi_y && n.lo_z <= n.hi_z))   /* ordered: crt_device.h in_slab */
                ds.planes_ok = 0;
        ub.add(hs.slots, &ds.slots);
        ub.add(hs.slot_tri, &ds.slot_tri);
        ub.add(hs.slot_cull, &ds.slot_cull);
        std::vector<uint32_t> bits((hs.slot_cull.size() + 31) / 32 + 1, 0u);
        for (size_t k = 0; k < hs.slot_cull.size(); ++k)
            if (hs.slot_cull[k]) bits[k >> 5] |= 1u << (k & 31);
        ub.add(bits, &ds.slot_cull_bits);
        sc->ref_bounds = hs.ref_bounds;
        sc->ref_children = hs.ref_children;
        sc->ref_leaf_off = hs.ref_leaf_off;
        sc->ref_leaf_tris = hs.ref_leaf_tris;
    } else {
        /* exact tree build on the device (crt_tree_build.hip) */
        DeviceTree dt;
        rc = build_tree_device(hs, nullptr, dt);
        for (void *p : dt.allocs) sc->allocs.push_back(p);
        if (rc != CRT_OK) return rc;
        ds.nodes = dt.nodes;
        ds.node_count = dt.node_count;
        ds.pnodes = dt.pnodes;
        ds.planes_ok = dt.planes_ok;
        ds.slots = dt.slots;
        ds.slot_tri = dt.slot_tri;
        ds.slot_cull = dt.slot_cull;
        ds.slot_cull_bits = dt.slot_cull_bits;
        sc->dt_ref_bounds = dt.ref_bounds;
        sc->dt_ref_children = dt.ref_children;
        sc->dt_ref_leaf_off = dt.ref_leaf_off;
        sc->dt_ref_leaf_tris = dt.ref_leaf_tris;
        sc->info.node_count = dt.node_count;
        sc->info.leaf_count = dt.leaf_count;
        sc->info.leaf_ref_count = dt.slot_count;
        sc->info.max_depth = dt.max_depth;
        sc->info.max_leaf_size = dt.max_leaf_size;
        sc->info.tree_build_ms = dt.build_ms;
        sc->info.tree_on_device = 1;
        const int64_t n = dt.node_count, m = dt.slot_count;
        sc->info.device_bytes += n * (int64_t)sizeof(DNode) + 8 * (n + 1) * (int64_t)sizeof(PNode) +
                                 m * (int64_t)(sizeof(DTriGeo) + 4 + 1) + (m / 32 + 1) * 4;
    }
    if (hs.bnode_count > 0) {   /* secondary-ray BVH (crt_bvh.h) */
        ub.add(hs.bnodes, &ds.bnodes);
        ub.add(hs.btri, &ds.btri);
        ub.add(hs.btri_id, &ds.btri_id);
        ds.bnode_count = hs.bnode_count;
        ub.add(hs.ktopo, &ds.ktopo);
        ub.add(hs.ktopo2, &ds.ktopo2);
    } else if (hs.tri_attr.size() > kHostBvhMax && sc->bvh_device) {   /* too large for the host build: on the device */
        DeviceBvh db;
        rc = build_bvh_device(hs, nullptr, db);
        for (void *p : db.allocs) sc->allocs.push_back(p);
        if (rc != CRT_OK) return rc;
        ds.bnodes = db.bnodes;
        ds.btri = db.btri;
        ds.btri_id = db.btri_id;
        ds.bnode_count = db.node_count;
        ub.add(hs.ktopo, &ds.ktopo);   /* host-built trees only */
        ub.add(hs.ktopo2, &ds.ktopo2);
        sc->info.bvh_on_device = 1;
        sc->info.bvh_depth = db.max_depth;
        sc->info.bvh_ms += db.build_ms;
        const int64_t n = db.node_count, nt = (int64_t)hs.tri_attr.size();
        sc->info.device_bytes += 8 * (n + 1) * (int64_t)sizeof(BNode) + nt * (int64_t)(sizeof(DTriGeo) + 4);
    }
    ds.cam = host_camera(hs);
    sc->fov_radians = hs.fov_radians;
    sc->prune_origin_max = hs.prune_origin_max;
    sc->camera_fast = camera_rays_fast(ds.cam, ds.planes_ok != 0);
    /* camera rays through the BVH too — not through a device-built
     * one: C5's camera rays take the pruned kd packet walk faster (4.49 against
     * 4.80 ms at 4K); that BVH serves the scattered rays */
    if (ds.bnodes && !sc->info.bvh_on_device) sc->traversal = 14;
    ub.add(hs.tri_attr, &ds.tri_attr);
    ub.add(hs.vnormal, &ds.vnormal);
    ub.add(hs.vuv, &ds.vuv);
    ub.add(hs.materials, &ds.materials);
    ub.add(hs.textures, &ds.textures);
    ub.add(hs.texels, &ds.texels);
    ub.add(hs.lights, &ds.lights);
    if ((rc = ub.flush(sc.get())) != CRT_OK) return rc;
    CRT_CREATE_STAMP("flush");
    ds.light_count = (int32_t)hs.lights.size();
    std::memcpy(ds.background, hs.background, sizeof ds.background);
    ds.gi_on = hs.gi_on;
    ds.reflections_on = hs.reflections_on;
    ds.refractions_on = hs.refractions_on;

    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    CRT_CREATE_STAMP("stream");
    if (sc->has_secondary && !(hs.gi_on && sc->has_diffuse))   /* the wavefront path's frame sets (render_wavefront) */
        if ((rc = wf_streams(sc->wf, sc->stream)) != CRT_OK) return rc;
    warm_code_objects(sc->device, sc->stream);
    CRT_CREATE_STAMP("warm");
    /* camera bins (crt_bins.hip), rebuilt on the device by every camera frame
     * of scenes whose camera rays the tile kernels trace without recursion
     * (no reflective / refractive material, no GI with a diffuse one); on a
     * scene without the BVH (> 2^18 triangles) only when no cell's list is
     * over the cap (those cells walk the BVH) */
    if (!sc->has_secondary && !(hs.gi_on && sc->has_diffuse)) {
        if ((rc = bins_setup(sc.get(), hs)) != CRT_OK) return rc;
        CRT_CREATE_STAMP("bins");
        if (ds.bins) sc->traversal = 14;   /* bins off: the BVH walk, or the kd walk without a BVH */
    }
    HIP_TRY(hipEventCreate(&sc->ev_start));
    HIP_TRY(hipEventCreate(&sc->ev_stop));
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, 16 * sizeof(unsigned long long)));
    sc->allocs.push_back(p);
    sc->d_counters = static_cast<unsigned long long *>(p);
    p = nullptr;
    HIP_TRY(hipMalloc(&p, 64));
    sc->allocs.push_back(p);
    sc->d_next_px = static_cast<int32_t *>(p);

    int64_t px = 0;
    const std::vector<DBucket> all = shard_buckets(hs.width, hs.height, hs.bucket_size, 0, 1, &px);
    sc->grid_empty = all.empty();
    if ((rc = make_tile_plan(sc.get(), all, true, sc->full)) != CRT_OK) return rc;
    CRT_CREATE_STAMP("plan");
    /* one-time costs of a first render that belong to the upload, like the
     * runtime's own initialisation (profiles/r03/cold): the device record, the
     * output image of crt_hip_render, and the runtime's staging for copies into
     * pageable host memory (allocated by the first such copy) */
    /* the scene's libm tables on this device (GI angles, Fresnel pow5): a
     * process-lifetime precompute of the host libm's values, kept out of the
     * first frame (main.cpp:37-43 times that frame) */
    if (gi_tables && (rc = ensure_gi_tables(sc.get())) != CRT_OK) return rc;
    CRT_CREATE_STAMP("tables");
    if (pow5_table && (rc = ensure_pow5_table(sc.get())) != CRT_OK) return rc;
    {
        const DeviceScene *d = nullptr;
        if ((rc = sync_device_record(sc.get(), &d, sc->stream)) != CRT_OK) return rc;
        if (!sc->grid_empty && primary) {
            const size_t bytes = (size_t)hs.width * hs.height * 3 * sizeof(float);
            HIP_TRY(hipMalloc(&sc->d_out, bytes));
            CRT_CREATE_STAMP("d_out");
            /* the staging image of copies into pageable memory (image_to_host), allocated beside the upload */
            if (want_stage) {
                const auto r = stage_f.get();
                if (r.first != hipSuccess) return set_error(CRT_E_HIP, std::string("staging image: ") + hipGetErrorString(r.first));
                sc->h_stage = r.second;
            } else {
                HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&sc->h_stage), bytes, hipHostMallocDefault));
            }
            CRT_CREATE_STAMP("h_stage");
            sc->stage_ev.assign(kStageChunks, nullptr);
            for (auto &e : sc->stage_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            (void)HostPool::get();
            /* the first DMA into a fresh pinned buffer, and the stream's first
             * asynchronous copy, pay one-time setup (~7 ms: profiles/r03/cold) */
            HIP_TRY(hipMemcpyAsync(sc->h_stage, sc->d_out, bytes, hipMemcpyDeviceToHost, sc->stream));
            HIP_TRY(hipStreamSynchronize(sc->stream));
            if ((rc = ensure_copy_rows(sc.get())) != CRT_OK) return rc;   /* the compact copy's row records */
            {   /* the copy's host threads started here, not inside the first render call */
                HostPool &pool = HostPool::get();
                pool.run(pool.threads(), [](void *, int) {}, nullptr);
            }
            CRT_CREATE_STAMP("first_dma");
        }
        unsigned long long probe[16];
        HIP_TRY(hipMemcpy(probe, sc->d_counters, sizeof probe, hipMemcpyDeviceToHost));
    }
    sc->info.bins_ms = sc->bins.setup_ms;
    sc->info.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_up).count();
    CRT_CREATE_STAMP("end");
    *out = sc.release();
    return CRT_OK;
}

}  // namespace crt_amd

extern "C" {

int crt_hip_scene_upload(const crt_host_scene *h, int device, crt_hip_scene **out) {
    if (!h || !out) return set_error(CRT_E_INVALID, "null argument");
    return scene_upload(*reinterpret_cast<const HostScene *>(h), device, true, out);
}

int crt_hip_scene_create_ex(const crt_scene_desc *desc, int device, int flags, crt_hip_scene **out) {
    const int32_t dev = device;
    return crt_hip_scene_create_on(desc, &dev, 1, flags, out);
}

int crt_hip_scene_from_tree(const crt_tree_scene_desc *desc, int device, crt_hip_scene **out) {
    const int32_t dev = device;
    return crt_hip_scene_from_tree_on(desc, &dev, 1, out);
}

int crt_hip_scene_create(const crt_scene_desc *desc, int device, crt_hip_scene **out) {
    return crt_hip_scene_create_ex(desc, device, CRT_SCENE_TREE_AUTO, out);
}

int64_t crt_hip_scene_bvh(const crt_hip_scene *sc, void *nodes_out, int32_t *tri_ids_out) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    const int64_t n = sc->ds.bnodes ? sc->ds.bnode_count : 0;
    if (n == 0) return 0;
    HIP_TRY(hipSetDevice(sc->device));
    if (nodes_out)
        HIP_TRY(hipMemcpy(nodes_out, sc->ds.bnodes, (size_t)8 * (n + 1) * sizeof(BNode), hipMemcpyDeviceToHost));
    if (tri_ids_out)
        HIP_TRY(hipMemcpy(tri_ids_out, sc->ds.btri_id, (size_t)sc->info.triangle_count * sizeof(int32_t),
                          hipMemcpyDeviceToHost));
    return n;
}

int crt_hip_scene_tree(const crt_hip_scene *sc, float *bounds, int32_t *children, int64_t *leaf_offsets,
                       int32_t *leaf_tris) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    const int64_t n = sc->info.node_count, m = sc->info.leaf_ref_count;
    if (sc->info.tree_on_device) {
        HIP_TRY(hipSetDevice(sc->device));
        if (bounds) HIP_TRY(hipMemcpy(bounds, sc->dt_ref_bounds, (size_t)n * 6 * sizeof(float), hipMemcpyDeviceToHost));
        if (children) HIP_TRY(hipMemcpy(children, sc->dt_ref_children, (size_t)n * 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
        if (leaf_offsets)
            HIP_TRY(hipMemcpy(leaf_offsets, sc->dt_ref_leaf_off, (size_t)(n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
        if (leaf_tris && m > 0)
            HIP_TRY(hipMemcpy(leaf_tris, sc->dt_ref_leaf_tris, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost));
        return CRT_OK;
    }
    if (bounds) std::memcpy(bounds, sc->ref_bounds.data(), sc->ref_bounds.size() * sizeof(float));
    if (children) std::memcpy(children, sc->ref_children.data(), sc->ref_children.size() * sizeof(int32_t));
    if (leaf_offsets) std::memcpy(leaf_offsets, sc->ref_leaf_off.data(), sc->ref_leaf_off.size() * sizeof(int64_t));
    if (leaf_tris) std::memcpy(leaf_tris, sc->ref_leaf_tris.data(), sc->ref_leaf_tris.size() * sizeof(int32_t));
    return CRT_OK;
}

int crt_hip_scene_info(const crt_hip_scene *sc, crt_scene_info *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = sc->info;
    out->wf_sets = 0;
    for (const WfSet &w : sc->wf.set) out->wf_sets += w.nodes ? 1 : 0;
    out->camera_moves = sc->camera_moves;
    out->view_rebuilds = sc->view_rebuilds;
    out->records_written = sc->records_written;
    out->bins_binnings = sc->bins.binnings;
    out->bins_reuses = sc->bins.reuses;
    out->light_bin_records = sc->lbins_records;
    out->light_bins_ms = sc->lbins_ms;
    return CRT_OK;
}

void crt_hip_scene_destroy(crt_hip_scene *sc) {
    if (!sc) return;
    multi_free(sc);
    (void)hipSetDevice(sc->device);
    if (sc->stream) (void)hipStreamSynchronize(sc->stream);
    for (void *p : sc->allocs) (void)hipFree(p);
    for (void *p : sc->plan_allocs) (void)hipFree(p);
    bins_free(sc);
    if (sc->d_out) (void)hipFree(sc->d_out);
    if (sc->h_rows) (void)hipHostFree(sc->h_rows);
    if (sc->d_row_spans) (void)hipFree(sc->d_row_spans);
    if (sc->spans_ev) (void)hipEventDestroy(sc->spans_ev);
    if (sc->copy_ev) (void)hipEventDestroy(sc->copy_ev);
    for (hipEvent_t e : sc->copy_band_ev)
        if (e) (void)hipEventDestroy(e);
    if (sc->gi_frames) (void)hipFree(sc->gi_frames);
    if (sc->sh_buf) (void)hipFree(sc->sh_buf);
    if (sc->sh_done) (void)hipEventDestroy(sc->sh_done);
    wf_free(sc->wf);
    for (auto &kv : sc->unpack_plans) (void)hipFree(kv.second.first);
    for (auto &kv : sc->compact_unpack) (void)hipFree(kv.second.first);
    if (sc->probe_buf) (void)hipFree(sc->probe_buf);
    if (sc->h_stage) (void)hipHostFree(sc->h_stage);
    for (hipEvent_t e : sc->stage_ev)
        if (e) (void)hipEventDestroy(e);
    for (int j = 0; j < kRecRing; ++j) {
        if (sc->rec_up[j]) (void)hipEventDestroy(sc->rec_up[j]);
        if (sc->rec_use[j]) (void)hipEventDestroy(sc->rec_use[j]);
    }
    if (sc->ev_start) (void)hipEventDestroy(sc->ev_start);
    if (sc->ev_stop) (void)hipEventDestroy(sc->ev_stop);
    if (sc->stream) (void)hipStreamDestroy(sc->stream);
    delete sc;
}

int crt_hip_render_device(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, void *stream) {
    if (!sc || !d_rgb) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    if (!sc->replicas.empty()) {   /* multi-GPU scene (crt_multi.hip) */
        if (multi_overflowed(sc))
            return set_error(CRT_E_STATE, "a wavefront level outgrew its recorded size in the previous frame; "
                                             "that frame is wrong (sizes are now read back again)");
        return render_multi_into(sc, st, d_rgb, s);
    }
    return render_into(sc, st, d_rgb, s, false);
}


}  // extern "C"

namespace crt_amd {

int render_checked(crt_hip_scene *sc, const crt_renderer_settings *st, float *rgb_out, crt_render_stats *stats,
                   bool (*check)(void *, int, int), void *check_arg, bool *mismatch) {
    if (mismatch) *mismatch = false;
    if (!sc || !rgb_out) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(sc->device));
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    const bool multi = !sc->replicas.empty();
    auto frame = [&]() -> int {
        return multi ? render_multi_into(sc, st, sc->d_out, sc->stream) : render_into(sc, st, sc->d_out, sc->stream, false);
    };
    rc = frame();
    if (rc != CRT_OK) return rc;
    HostCheck hc;
    hc.fn = check;
    hc.arg = check_arg;
    if ((rc = image_to_host(sc, rgb_out, nfl, check ? &hc : nullptr)) != CRT_OK) return rc;
    const bool overflow = multi ? multi_overflowed(sc) : wf_overflowed(sc->wf, true);
    if (check && hc.failed) {   /* the caller's scene is not this one: the frame is for nobody */
        if (mismatch) *mismatch = true;
        return CRT_OK;
    }
    if (overflow) {   /* recorded level sizes did not hold: render again with read-backs */
        if ((rc = frame()) != CRT_OK) return rc;
        if ((rc = image_to_host(sc, rgb_out, nfl)) != CRT_OK) return rc;
    }
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        float ms = 0.f;
        if (multi) {   /* the slowest replica's shard */
            std::vector<double> rm(1 + sc->replicas.size(), 0.0);
            if ((rc = crt_hip_last_replica_ms(sc, rm.data(), (int32_t)rm.size())) < 0) return rc;
            for (double r : rm) ms = std::max(ms, (float)r);
        } else if (!sc->grid_empty && sc->full.ntiles > 0 && sc->events_valid) {
            HIP_TRY(hipEventElapsedTime(&ms, sc->ev_start, sc->ev_stop));
        }
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->width = sc->info.width;
        stats->height = sc->info.height;
    }
    return CRT_OK;
}


}  // namespace crt_amd

extern "C" {

int crt_hip_render(crt_hip_scene *sc, const crt_renderer_settings *st, float *rgb_out, crt_render_stats *stats) {
    return render_checked(sc, st, rgb_out, stats, nullptr, nullptr, nullptr);
}

int crt_hip_plan_info(const crt_hip_scene *sc, crt_plan_info *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    std::memset(out, 0, sizeof *out);
    out->calib_k = (sc->calib_walk >= 0 && !sc->calib.empty()) ? (double)sc->calib_k : 0.0;
    out->tiles = sc->full.ntiles;
    for (const Tile &t : sc->full.tiles) out->small_tiles += t.w * t.h <= 16 ? 1 : 0;
    return CRT_OK;
}

int crt_hip_last_kernel_ms(crt_hip_scene *sc, double *ms) {
    if (!sc || !ms) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    if (!sc->events_valid) return set_error(CRT_E_INVALID, "no timed render (option \"events\" is off)");
    HIP_TRY(hipEventSynchronize(sc->ev_stop));
    float f = 0.f;
    HIP_TRY(hipEventElapsedTime(&f, sc->ev_start, sc->ev_stop));
    *ms = f;
    return CRT_OK;
}

int64_t crt_hip_shard_floats(const crt_hip_scene *sc, int shard, int shard_count) {
    if (!sc || shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    int64_t px = 0;
    shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, shard, shard_count, &px);
    return 3 * px;
}

int64_t crt_hip_shard_stride(const crt_hip_scene *sc, int shard_count) {
    if (!sc || shard_count <= 0) return set_error(CRT_E_INVALID, "bad shard count");
    int64_t m = 0;
    for (int s = 0; s < shard_count; ++s) m = std::max(m, crt_hip_shard_floats(sc, s, shard_count));
    return (m + 63) / 64 * 64;
}

}  // extern "C"

extern "C" {

int crt_hip_render_shard(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count,
                         float *d_packed, void *stream) {
    return render_shard_t(sc, st, shard, shard_count, d_packed, stream, false);
}

int crt_hip_unpack_shards(crt_hip_scene *sc, int shard_count, const float *d_gathered, float *d_rgb, void *stream) {
    return unpack_shards_t<float>(sc, shard_count, d_gathered, d_rgb, stream, false);
}

int crt_hip_unpack_shards_rgb8(crt_hip_scene *sc, int shard_count, const uint8_t *d_gathered, uint8_t *d_rgb8,
                               void *stream) {
    return unpack_shards_t<uint8_t>(sc, shard_count, d_gathered, d_rgb8, stream, false);
}

int crt_hip_live_mask(crt_hip_scene *sc, uint8_t *out) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_live_mask(sc);
    if (rc != CRT_OK) return rc;
    if (out && !sc->live_mask.empty()) std::memcpy(out, sc->live_mask.data(), sc->live_mask.size());
    else if (out) std::memset(out, 0, (size_t)sc->info.width * sc->info.height);
    return CRT_OK;
}

int64_t crt_hip_compact_floats(crt_hip_scene *sc, int shard, int shard_count) {
    if (!sc || shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_live_mask(sc);
    if (rc != CRT_OK) return rc;
    int64_t px = 0;
    compact_tiles(sc, shard, shard_count, &px);
    return 3 * px;
}

int64_t crt_hip_compact_stride(crt_hip_scene *sc, int shard_count) {
    if (!sc || shard_count <= 0) return set_error(CRT_E_INVALID, "bad shard count");
    int64_t m = 0;
    for (int s = 0; s < shard_count; ++s) {
        const int64_t f = crt_hip_compact_floats(sc, s, shard_count);
        if (f < 0) return f;
        m = std::max(m, f);
    }
    return std::max<int64_t>(64, (m + 63) / 64 * 64);
}

int crt_hip_render_shard_compact(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count,
                                 float *d_packed, void *stream) {
    return render_shard_t(sc, st, shard, shard_count, d_packed, stream, true);
}

int crt_hip_unpack_compact(crt_hip_scene *sc, int shard_count, const float *d_gathered, float *d_rgb, void *stream) {
    return unpack_shards_t<float>(sc, shard_count, d_gathered, d_rgb, stream, true);
}

int crt_hip_unpack_compact_rgb8(crt_hip_scene *sc, int shard_count, const uint8_t *d_gathered, uint8_t *d_rgb8,
                                void *stream) {
    return unpack_shards_t<uint8_t>(sc, shard_count, d_gathered, d_rgb8, stream, true);
}

int crt_hip_quantize_rgb8(const float *d_rgb, int64_t n, int32_t max_color_component, uint8_t *d_out, void *stream) {
    if ((n > 0 && (!d_rgb || !d_out)) || n < 0) return set_error(CRT_E_INVALID, "bad argument");
    if (max_color_component < 0 || max_color_component > 255)
        return set_error(CRT_E_UNSUPPORTED, "8-bit output needs max_color_component in 0..255");
    if (n == 0) return CRT_OK;
    const int64_t threads = (n + 3) / 4;
    hipLaunchKernelGGL(k_quantize, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_rgb, d_out, n, (float)max_color_component,
                       max_color_component);
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

int crt_hip_trace_batch(crt_hip_scene *sc, const float *rays, int64_t n, crt_hit *hits_out) {
    if (!sc || (n > 0 && (!rays || !hits_out)) || n < 0) return set_error(CRT_E_INVALID, "bad argument");
    if (n == 0) return CRT_OK;
    HIP_TRY(hipSetDevice(sc->device));
    float *d_rays = nullptr;
    crt_hit *d_hits = nullptr;
    HIP_TRY(hipMalloc(&d_rays, (size_t)n * 6 * sizeof(float)));
    hipError_t e = hipMalloc(&d_hits, (size_t)n * sizeof(crt_hit));
    if (e != hipSuccess) { (void)hipFree(d_rays); return set_error(CRT_E_HIP, hipGetErrorString(e)); }
    e = hipMemcpy(d_rays, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_trace_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, sc->stream, sc->ds, d_rays,
                           n, d_hits, sc->trace_walk);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
    if (e == hipSuccess) e = hipMemcpy(hits_out, d_hits, (size_t)n * sizeof(crt_hit), hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    (void)hipFree(d_hits);
    if (e != hipSuccess) return set_error(CRT_E_HIP, hipGetErrorString(e));
    return CRT_OK;
}

int crt_hip_profile_waves(crt_hip_scene *sc, const crt_renderer_settings *st, uint64_t *stamps, int64_t cap,
                          int32_t *tile_xy) {
    if (!sc || !st) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    {
        const int rc = ensure_plans(sc, st, sc->stream);
        if (rc != CRT_OK) return rc;
    }
    const int nt = sc->full.waves;
    if (!stamps || !tile_xy) return nt;      /* query the size */
    if (cap < nt) return set_error(CRT_E_INVALID, "stamp buffer too small");
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)nt * 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(d, 0, (size_t)nt * 2 * sizeof(unsigned long long)));
    int rc = launch_render(sc, st, sc->full, sc->d_out, sc->stream, false, d);
    hipError_t e = rc == CRT_OK ? hipStreamSynchronize(sc->stream) : hipSuccess;
    if (rc == CRT_OK && e == hipSuccess)
        e = hipMemcpy(stamps, d, (size_t)nt * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    /* each wave's tile: the plan's tiles in order, or (camera bins) the
     * frame's work lists, then the rest tiles */
    const ShardPlan &p = sc->full;
    const BinsPlan &bp = p.bp;
    std::vector<BinsWork> work;
    std::vector<int32_t> ph_all, rest;
    int par = 0;
    if (rc == CRT_OK && e == hipSuccess && bp.cell_tile) {
        par = (int)((sc->bins.frame - 1) % kBinSets);   /* the set the frame just used */
        int64_t slots = 0;
        slots = (int64_t)kBinKinds * kBinShards * bp.ecap;
        work.resize((size_t)std::max<int64_t>(1, slots));
        ph_all.resize((size_t)kBinsPhdrInts);
        rest.resize((size_t)std::max(1, bp.nrest));
        e = hipMemcpy(work.data(), bp.work + (size_t)par * bp.wslots, work.size() * sizeof(BinsWork),
                      hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(ph_all.data(), bp.phdr, ph_all.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(rest.data(), bp.rest, rest.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    if (rc != CRT_OK) return rc;
    if (e != hipSuccess) return set_error(CRT_E_HIP, hipGetErrorString(e));
    for (int k = 0; k < nt; ++k) {
        int x = -1, y = -1;
        if (!bp.cell_tile) {
            x = p.tiles[(size_t)k].x;
            y = p.tiles[(size_t)k].y;
        } else {
            int kind = 0, slot = k >> 2, q = k & 3;
            if (k >= 4 * kBinShards * bp.gcap[0]) {
                slot = k - 4 * kBinShards * bp.gcap[0];
                q = -1;
                kind = 1;
                while (kind < kBinKinds && slot >= kBinShards * bp.gcap[kind]) slot -= kBinShards * bp.gcap[kind++];
            }
            if (kind == kBinKinds) {
                if (slot < bp.nrest) {
                    x = p.tiles[(size_t)rest[(size_t)slot]].x;
                    y = p.tiles[(size_t)rest[(size_t)slot]].y;
                }
            } else {
                const int sh = slot % kBinShards, i2 = slot / kBinShards;
                if (i2 < std::min(ph_all[(size_t)bins_phdr_at(par, kind, sh)], bp.ecap)) {
                    const Tile &t = work[(size_t)(bp.wbase[kind] + sh * bp.ecap + i2)].t;
                    x = t.x + (q >= 0 ? (q & 1) * 4 : 0);
                    y = t.y + (q >= 0 ? (q >> 1) * 4 : 0);
                }
            }
        }
        tile_xy[2 * k] = x;
        tile_xy[2 * k + 1] = y;
    }
    return nt;
}

int crt_hip_plan_tiles(crt_hip_scene *sc, const crt_renderer_settings *st, int32_t *xywh, float *cost, int64_t cap) {
    if (!sc || !st) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_plans(sc, st, sc->stream);
    if (rc != CRT_OK) return rc;
    const ShardPlan &p = sc->full;
    if (!xywh) return p.ntiles;
    if (cap < p.ntiles) return set_error(CRT_E_INVALID, "tile buffer too small");
    for (int k = 0; k < p.ntiles; ++k) {
        xywh[4 * k] = p.tiles[k].x;
        xywh[4 * k + 1] = p.tiles[k].y;
        xywh[4 * k + 2] = p.tiles[k].w;
        xywh[4 * k + 3] = p.tiles[k].h;
        if (cost) cost[k] = p.cost.empty() ? 0.f : p.cost[k];
    }
    return p.ntiles;
}

int crt_hip_count_work(crt_hip_scene *sc, const crt_renderer_settings *st, crt_work_counts *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    std::memset(out, 0, sizeof *out);
    if (sc->grid_empty) return CRT_OK;
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    if ((rc = ensure_plans(sc, st, sc->stream)) != CRT_OK) return rc;
    HIP_TRY(hipMemsetAsync(sc->d_counters, 0, 16 * sizeof(unsigned long long), sc->stream));
    rc = launch_render(sc, st, sc->full, sc->d_out, sc->stream, true);
    if (rc != CRT_OK) return rc;
    unsigned long long c[16];
    HIP_TRY(hipMemcpyAsync(c, sc->d_counters, sizeof c, hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    out->traversals = c[0];
    out->node_tests = c[1];
    out->triangle_tests = c[2];
    out->hits = c[3];
    sc->wave_counts.node_steps = c[4];
    sc->wave_counts.triangle_steps = c[5];
    sc->wave_counts.edge_steps = c[6];
    sc->wave_counts.waves = c[7];
    sc->wave_counts.box_steps = c[8];
    sc->wave_counts.pass_steps = c[9];
    sc->wave_counts.window_waves = c[10];
    sc->wave_counts.window_steps = c[11];
    sc->wave_counts.window_slots = c[12];
    sc->wave_counts.window_reached = c[13];
    sc->wave_counts.window_tri_rounds = c[14];
    return CRT_OK;
}

/* One replica's option (on its device). */
static int set_option_one(crt_hip_scene *sc, const char *name, int value) {
    const std::string k(name);
    if (k == "traversal") {
        if (value != 7 && value != 8 && value != 14)
            return set_error(CRT_E_INVALID, "traversal must be 7 (reference order), 8 (pruned) or 14 (BVH)");
        sc->traversal = value;
        wf_graphs_clear(sc->wf);   /* captured wavefront frames bake in the level-0 walk */
    } else if (k == "secondary") {
        if (value != 0 && value != 4 && value != 10 && value != 14)
            return set_error(CRT_E_INVALID, "secondary must be 0, 4, 10 or 14");
        sc->secondary = value;
        wf_graphs_clear(sc->wf);   /* ... the levels' walk */
    } else if (k == "wavefront") {
        sc->wavefront = value != 0;
    } else if (k == "window") {
        sc->window_walk = value != 0;
    } else if (k == "gi_refill") {
        sc->gi_refill = value != 0;
    } else if (k == "gi_machine") {
        sc->gi_machine = value != 0;
    } else if (k == "rec_machine") {
        sc->rec_machine = value != 0;
        sc->calib_walk = -1;
    } else if (k == "wf_record") {   /* the next frames' choice between recorded sizes and device-sized levels */
        sc->wf_record = value != 0;
        return CRT_OK;
    } else if (k == "wf_dynamic" || k == "wf_dyn_ids" || k == "wf_dyn_waves") {   /* device-sized frames (render_wavefront) */
        if (k == "wf_dyn_ids" && (value < 1 || value > 64)) return set_error(CRT_E_INVALID, "wf_dyn_ids must be 1..64");
        if (k == "wf_dyn_waves" && (value < 64 || value > (1 << 20)))
            return set_error(CRT_E_INVALID, "wf_dyn_waves must be 64..2^20");
        HIP_TRY(hipDeviceSynchronize());
        (k == "wf_dynamic" ? sc->wf_dynamic : k == "wf_dyn_ids" ? sc->wf_dyn_ids : sc->wf_dyn_waves) =
            k == "wf_dynamic" ? (value != 0) : (int)value;
        return CRT_OK;
    } else if (k == "compact_copy") {   /* crt_hip_render's image copy: 1 compact (default), 0 the whole image */
        sc->compact_copy = value != 0;
        return CRT_OK;
    } else if (k == "bins_qmax") {   /* test hook: groups k_bins_pairs takes (a kernel argument of the binning) */
        if (value < 1) return set_error(CRT_E_INVALID, "bins_qmax must be >= 1");
        sc->bins.qmax = std::min((int)value, 8192);   /* kMaxGroups (crt_bins.hip) */
        return CRT_OK;
    } else if (k == "bins_reuse") {   /* no plan depends on it */
        sc->bins_reuse = value != 0;
        return CRT_OK;
    } else if (k == "bins" || k == "bins_split" || k == "bins_quad" || k == "bins_slack") {   /* camera bins: the full-frame plan depends on them */
        if (k == "bins_split" && value < 1) return set_error(CRT_E_INVALID, "bins_split must be >= 1");
        if (k == "bins_slack" && (value < 0 || value > 1000)) return set_error(CRT_E_INVALID, "bins_slack must be 0..1000");
        int &field = k == "bins" ? sc->bins_on : k == "bins_quad" ? sc->bins_quad : k == "bins_slack" ? sc->bins_slack : sc->bins_split;
        const int v = k == "bins" || k == "bins_quad" ? (value != 0) : (int)value;
        if (v != field) {
            HIP_TRY(hipDeviceSynchronize());
            field = v;
            sc->calib_walk = -1;
            free_plans(sc);
            int64_t px = 0;
            const int rc = make_tile_plan(sc, shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, 0, 1, &px),
                                          true, sc->full);
            if (rc != CRT_OK) return rc;
        }

    } else if (k == "calib_k_milli") {   /* a fixed split threshold k = value / 1000 (calibrate 2) */
        if (value <= 0) return set_error(CRT_E_INVALID, "calib_k_milli must be > 0");
        sc->calib_defer = false;   /* an explicit plan request: calibrate on the first frame */
        sc->calib_k = (float)value / 1000.0f;
        sc->calibrate = 2;
        sc->calib_walk = -1;
    } else if (k == "wf_graph") {
        sc->wf_graph = value != 0;
        wf_graphs_clear(sc->wf);
    } else if (k == "wf_replay") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "wf_replay must be 0, 1 or 2");
        sc->wf_replay = value;
        { sc->wf.recs.clear(); ++sc->wf.epoch; }
        wf_graphs_clear(sc->wf);
    } else if (k == "wf_rpw") {
        if (value < 1 || value > 64) return set_error(CRT_E_INVALID, "wf_rpw must be 1..64");
        sc->wf_rays_per_wave = value;
        wf_graphs_clear(sc->wf);   /* ... and each level's rays per wave */
    } else if (k == "events") {
        sc->record_events = value != 0;
    } else if (k == "calibrate") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "calibrate must be 0 (estimate plan), 1 (tuned) or 2 (fixed k)");
        sc->calib_defer = false;   /* an explicit plan request: calibrate on the first frame */
        if (value != sc->calibrate) sc->calib_walk = sc->calibrate ? -1 : sc->calib_walk;   /* re-plan on next use */
        sc->calib_tuned = false;   /* calibrate 1: tune k again */
        sc->calibrate = value;
        if (!sc->calibrate && !sc->calib.empty()) {   /* back to the estimate plan */
            HIP_TRY(hipDeviceSynchronize());
            sc->calib.clear();
            sc->calib_walk = -1;
            free_plans(sc);
            int64_t px = 0;
            const int rc = make_tile_plan(sc, shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, 0, 1, &px),
                                          true, sc->full);
            if (rc != CRT_OK) return rc;
        }
    } else if (k == "calib_min") {   /* smallest side the calibrated plan splits tiles down to */
        if (value != 1 && value != 2 && value != 4 && value != 8) return set_error(CRT_E_INVALID, "calib_min must be 1, 2, 4 or 8");
        sc->calib_defer = false;   /* an explicit plan request: calibrate on the first frame */
        sc->calib_min = value;
        sc->calib_walk = -1;
        sc->calib_tuned = false;
    } else if (k == "shadows") {
        sc->shadows = value != 0;
    } else if (k == "shadow_defer") {
        sc->shadow_defer = value != 0;
    } else if (k == "light_bins") {
        sc->light_bins = value != 0;
        if (sc->lbins_tried) sc->ds.lbin_n = sc->light_bins ? sc->lbins_n : 0;
    } else if (k == "trace_walk") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "trace_walk must be 0, 1 or 2 (BVH)");
        sc->trace_walk = value;
    } else {
        return set_error(CRT_E_INVALID, "unknown option: " + k);
    }
    /* tile plans depend on the walk (tile splitting): rebuild on next use */
    return CRT_OK;
}

/* ---- the camera (crt_hip_scene_set_camera) ---- */

namespace {

/* Device buffers and plans derived from the view, rebuilt with the device
 * drained: the resolution changed, the camera bins must be built or dropped
 * for the new camera, or the compact shards' live mask (a function of the
 * camera) is in use. */
int rebuild_view(crt_hip_scene *sc, const DCamera &c, bool resized, bool bins_ok, bool primary) {
    HIP_TRY(hipDeviceSynchronize());
    sc->ds.cam = c;
    if (resized) {
        sc->info.width = c.width;
        sc->info.height = c.height;
        sc->calib.clear();   /* per 8x8 tile of the old frame */
        sc->calib_walk = -1;
        sc->calib_deferred_walk = -1;
        sc->calib_tuned = false;
        if (!sc->ref_children.empty())
            sc->tile_work = tile_work_estimate_of(c, sc->ref_bounds, sc->ref_children, sc->ref_leaf_off,
                                                  (c.width + 7) / 8, (c.height + 7) / 8);
        else
            sc->tile_work.clear();
    }
    sc->live_mask.clear();
    for (auto &kv : sc->compact_unpack) (void)hipFree(kv.second.first);
    sc->compact_unpack.clear();
    if (resized) {
        for (auto &kv : sc->unpack_plans) (void)hipFree(kv.second.first);
        sc->unpack_plans.clear();
    }
    free_plans(sc);   /* full frame, shards, compact shards; wavefront sizes and graphs */
    if (sc->bins.tpl && (resized || (sc->ds.bins != nullptr) != bins_ok)) {
        bins_free_view(sc);
        int rc;
        if (bins_ok && (rc = bins_view(sc)) != CRT_OK) return rc;
    } else if (sc->ds.bins) {
        (void)bin_camera_of(c, sc->prune_origin_max, sc->bins.cam);
    }
    int64_t px = 0;
    const std::vector<DBucket> all = shard_buckets(c.width, c.height, sc->info.bucket_size, 0, 1, &px);
    sc->grid_empty = all.empty();
    if (resized && primary) {
        const size_t bytes = (size_t)c.width * c.height * 3 * sizeof(float);
        if (sc->d_out) (void)hipFree(sc->d_out);
        sc->d_out = nullptr;
        HIP_TRY(hipMalloc(&sc->d_out, bytes));
        if (sc->h_stage) (void)hipHostFree(sc->h_stage);
        sc->h_stage = nullptr;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&sc->h_stage), bytes, hipHostMallocDefault));
    }
    return make_tile_plan(sc, all, true, sc->full);
}

/* One replica (primary: the handle's first, which owns the output image). */
int set_camera_one(crt_hip_scene *sc, const DCamera &c, float fov_radians, bool primary) {
    HIP_TRY(hipSetDevice(sc->device));
    if (std::memcmp(&sc->ds.cam, &c, sizeof c) == 0 && sc->fov_radians == fov_radians) return CRT_OK;
    const bool resized = c.width != sc->ds.cam.width || c.height != sc->ds.cam.height;
    BinCamera bc;
    const bool bins_ok = sc->bins.tpl && bin_camera_of(c, sc->prune_origin_max, bc);
    sc->fov_radians = fov_radians;
    sc->camera_fast = camera_rays_fast(c, sc->ds.planes_ok != 0);
    ++sc->camera_moves;
    if (resized || (sc->bins.tpl && (sc->ds.bins != nullptr) != bins_ok) || !sc->live_mask.empty() ||
        !sc->compact_unpack.empty()) {
        ++sc->view_rebuilds;
        return rebuild_view(sc, c, resized, bins_ok, primary);
    }
    /* the camera alone: frames in flight keep their device record and their
     * binning's camera (both taken by value when a frame is issued); the next
     * frames take these */
    sc->ds.cam = c;
    if (sc->ds.bins) sc->bins.cam = bc;
    if (!sc->wf.recs.empty() || !sc->wf.graphs.empty()) {   /* level sizes are the old camera's rays */
        wf_graphs_clear(sc->wf);
        sc->wf.recs.clear();
    }
    ++sc->wf.epoch;   /* nor may a device-sized frame of the old camera record its sizes (wf_harvest) */
    return CRT_OK;
}

int set_camera_all(crt_hip_scene *sc, const crt_vec3 *location, const float *rotation, float fov_radians,
                   int32_t width, int32_t height) {
    if (!sc || !location || !rotation) return set_error(CRT_E_INVALID, "null argument");
    if (width <= 0 || height <= 0) return set_error(CRT_E_INVALID, "image width/height must be positive");
    const float loc[3] = {location->x, location->y, location->z};
    DCamera c{};
    if (!make_camera(loc, rotation, fov_radians, width, height, c))
        return set_error(CRT_E_INVALID, "bad camera");
    int rc = set_camera_one(sc, c, fov_radians, true);
    for (size_t i = 0; rc == CRT_OK && i < sc->replicas.size(); ++i) rc = set_camera_one(sc->replicas[i], c, fov_radians, false);
    HIP_TRY(hipSetDevice(sc->device));
    return rc;
}

}  // namespace

int crt_hip_scene_set_camera(crt_hip_scene *sc, const crt_camera_desc *camera) {
    if (!sc || !camera) return set_error(CRT_E_INVALID, "null argument");
    return set_camera_all(sc, &camera->location, camera->rotation, fov_degrees_to_radians(camera->fov_degrees),
                          camera->width, camera->height);
}

int crt_hip_scene_set_camera_rad(crt_hip_scene *sc, const crt_vec3 *location, const float *rotation,
                                 float fov_radians, int32_t width, int32_t height) {
    return set_camera_all(sc, location, rotation, fov_radians, width, height);
}

int crt_hip_scene_camera(const crt_hip_scene *sc, crt_camera_desc *camera, float *fov_radians) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    if (camera) {
        camera->location = crt_vec3{sc->ds.cam.loc[0], sc->ds.cam.loc[1], sc->ds.cam.loc[2]};
        std::memcpy(camera->rotation, sc->ds.cam.rot, sizeof camera->rotation);
        camera->width = sc->ds.cam.width;
        camera->height = sc->ds.cam.height;
        camera->fov_degrees = sc->fov_radians * 180.0f / 3.14159265358979323846f;
    }
    if (fov_radians) *fov_radians = sc->fov_radians;
    return CRT_OK;
}

/* Every replica of a multi-GPU handle takes the option (each renders its own
 * shard with its own settings: an option set on the first alone would mix two
 * renderers in one image). */
int crt_hip_scene_set_option(crt_hip_scene *sc, const char *name, int value) {
    if (!sc || !name) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    int rc = set_option_one(sc, name, value);
    for (size_t i = 0; rc == CRT_OK && i < sc->replicas.size(); ++i) {
        HIP_TRY(hipSetDevice(sc->replicas[i]->device));
        rc = set_option_one(sc->replicas[i], name, value);
    }
    HIP_TRY(hipSetDevice(sc->device));
    return rc;
}

int crt_hip_wave_counts(crt_hip_scene *sc, crt_wave_counts *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = sc->wave_counts;
    return CRT_OK;
}

}  // extern "C"

