/*
 * crt_multi.hip — several GPUs behind one scene handle (include/crt_hip.h
 * crt_hip_scene_create_on / _mask, SURVEY §8(b) gpu_mask).
 *
 * The reference's render_image spans every hardware thread of the host
 * (crt_renderer.cpp:176-196: a bucket queue drained by
 * hardware_concurrency() threads); this spans every GPU the handle holds.
 * The scene is prepared once on the host and uploaded to each device; a
 * frame deals the reference's bucket grid to the replicas (bucket k ->
 * replica k % G, compact shards: only tiles with a live pixel), each replica
 * renders its shard on its own stream, copies it peer-to-peer (xGMI) into the
 * first device's gather buffer, and the first device unpacks the frame
 * (background into dead tiles).  Pixels are independent (per-pixel PCG seed,
 * read-only scene), so the image is bit-identical for any replica count.
 *
 * A device may be listed more than once: it then holds several replicas —
 * how a one-GPU host runs the whole split (tests/test_gpu_multi.py).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "crt_scene_impl.h"

namespace crt_amd {

namespace {

/* Peer access both ways between the gathering device and a replica's
 * (already enabled / not supported: the copy still works, staged by the
 * runtime). */
void enable_peers(int a, int b) {
    if (a == b) return;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        (void)hipSetDevice(a);
        (void)hipDeviceEnablePeerAccess(b, 0);
    }
    if (hipDeviceCanAccessPeer(&can, b, a) == hipSuccess && can) {
        (void)hipSetDevice(b);
        (void)hipDeviceEnablePeerAccess(a, 0);
    }
    (void)hipGetLastError();   /* hipErrorPeerAccessAlreadyEnabled is not an error here */
}

/* The multi-device probe's verdict (crt_multi_probe_verdict). */
int probe_verdict(const float *multi, const float *single, int64_t n, int render_status) {
    if (render_status != CRT_OK) return 2;
    if (n > 0 && std::memcmp(multi, single, (size_t)n * sizeof(float)) != 0) return 1;
    return 0;
}

/* A handle over >= 2 distinct devices renders a 64x36 probe frame of its
 * scene through every replica (shards dealt over the devices, peer copies
 * into device 0, cross-device event waits: the path no single-GPU test
 * exercises) and through device 0 alone, before its first real frame; on any
 * error or a differing bit the replicas go and the handle renders on one GPU
 * (crt_scene_info.multi_probe = -1 / -2, the reason in crt_hip_last_error()).
 * CRT_MULTI_PROBE=0 skips it, =force runs it also over repeated devices;
 * CRT_MULTI_PROBE_INJECT=1 flips one bit of the multi-device image (tests). */
int multi_probe(crt_hip_scene *sc) {
    const auto t0 = std::chrono::steady_clock::now();
    const DCamera full = sc->ds.cam;
    const float fov = sc->fov_radians;
    const crt_vec3 loc{full.loc[0], full.loc[1], full.loc[2]};
    const int pw = std::min(64, full.width), ph = std::min(36, full.height);
    crt_renderer_settings st;
    crt_renderer_settings_default(&st);
    std::vector<float> multi((size_t)pw * ph * 3, 0.f), single((size_t)pw * ph * 3, 0.f);
    int rc = crt_hip_scene_set_camera_rad(sc, &loc, full.rot, fov, pw, ph);
    if (rc == CRT_OK) rc = crt_hip_render(sc, &st, multi.data(), nullptr);
    if (rc == CRT_OK) {
        std::vector<crt_hip_scene *> reps;
        reps.swap(sc->replicas);   /* device 0 alone */
        rc = crt_hip_render(sc, &st, single.data(), nullptr);
        sc->replicas.swap(reps);
    }
    std::string why = rc != CRT_OK ? std::string(crt_hip_last_error()) : std::string();
    if (rc == CRT_OK) {
        if ((sc->create_flags & CRT_SCENE_PROBE_TEST_MISMATCH) && !multi.empty())   /* test hook: a differing bit */
            reinterpret_cast<uint32_t *>(multi.data())[0] ^= 1u;
    }
    const int verdict = probe_verdict(multi.data(), single.data(), (int64_t)multi.size(), rc);
    /* back to the scene's own camera, then drop the replicas if the probe failed */
    (void)hipGetLastError();
    const int rc2 = crt_hip_scene_set_camera_rad(sc, &loc, full.rot, fov, full.width, full.height);
    sc->info.multi_probe_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (verdict == 0 && rc2 == CRT_OK) {
        sc->info.multi_probe = 1;
        return CRT_OK;
    }
    multi_free(sc);
    HIP_TRY(hipSetDevice(sc->device));
    if (rc2 != CRT_OK) {   /* one GPU: its camera back, plans and buffers of its size */
        const int rc3 = crt_hip_scene_set_camera_rad(sc, &loc, full.rot, fov, full.width, full.height);
        if (rc3 != CRT_OK) return rc3;
    }
    sc->info.multi_probe = verdict == 1 ? -1 : -2;
    set_error(CRT_E_STATE, verdict == 1 ? "multi-GPU probe: the replicas' 64x36 frame differs from device 0's; "
                                          "rendering on one GPU"
                                        : "multi-GPU probe failed (" + why + "); rendering on one GPU");
    return CRT_OK;
}

/* One prepared host scene uploaded to every listed device. */
int upload_on(const HostScene &hs, const int32_t *devices, int32_t count, crt_hip_scene **out, int flags = 0) {
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if (!devices || count < 1) return set_error(CRT_E_INVALID, "no devices");
    crt_hip_scene *first = nullptr;
    int rc = scene_upload(hs, devices[0], true, &first);
    if (rc != CRT_OK) return rc;
    std::unique_ptr<crt_hip_scene, void (*)(crt_hip_scene *)> sc(first, crt_hip_scene_destroy);
    sc->create_flags = flags;
    for (int32_t i = 1; i < count; ++i) {
        crt_hip_scene *r = nullptr;
        if ((rc = scene_upload(hs, devices[i], false, &r)) != CRT_OK) return rc;
        sc->replicas.push_back(r);
        enable_peers(devices[0], devices[i]);
        HIP_TRY(hipSetDevice(devices[i]));
        HIP_TRY(hipEventCreateWithFlags(&r->mg_done, hipEventDisableTiming));
    }
    if (count > 1) {
        HIP_TRY(hipSetDevice(devices[0]));
        HIP_TRY(hipEventCreateWithFlags(&sc->mg_done, hipEventDisableTiming));   /* "gather unpacked" */
        bool distinct = false;
        for (int32_t i = 1; i < count; ++i) distinct = distinct || devices[i] != devices[0];
        const bool force = (flags & CRT_SCENE_PROBE_FORCE) != 0, off = (flags & CRT_SCENE_PROBE_OFF) != 0;
        if (!off && (distinct || force) && !sc->grid_empty) {
            const int rc2 = multi_probe(sc.get());
            if (rc2 != CRT_OK) return rc2;
        }
    }
    sc->info.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *out = sc.release();
    return CRT_OK;
}

/* gpu_mask -> device list (0: env CRT_HIP_GPUS = a count, else every device) */
int mask_devices(uint64_t mask, std::vector<int32_t> &devs) {
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (n <= 0) return set_error(CRT_E_HIP, "no HIP device");
    devs.clear();
    if (mask == 0) {
        int want = n;
        if (const char *e = std::getenv("CRT_HIP_GPUS")) want = std::max(1, std::min(n, std::atoi(e)));
        for (int d = 0; d < want; ++d) devs.push_back(d);
        return CRT_OK;
    }
    for (int d = 0; d < 64; ++d)
        if ((mask >> d) & 1ull) {
            if (d >= n) return set_error(CRT_E_INVALID, "gpu_mask names a device that is not visible");
            devs.push_back(d);
        }
    return CRT_OK;
}

int tree_mode(const crt_scene_desc *desc, int flags) {
    int mode = flags & 3;
#ifdef CRT_AB_OPTIONS
    if (mode == CRT_SCENE_TREE_AUTO) {   /* A/B builds: the build site from the environment */
        if (const char *e = std::getenv("CRT_TREE_BUILD")) {
            if (std::strcmp(e, "host") == 0) mode = CRT_SCENE_TREE_HOST;
            if (std::strcmp(e, "device") == 0) mode = CRT_SCENE_TREE_DEVICE;
        }
    }
#endif
    if (mode == CRT_SCENE_TREE_AUTO) {
        int64_t nt = 0;
        for (int i = 0; i < desc->mesh_count && desc->meshes; ++i) nt += desc->meshes[i].index_count / 3;
        mode = nt >= CRT_SCENE_DEVICE_BUILD_MIN ? CRT_SCENE_TREE_DEVICE : CRT_SCENE_TREE_HOST;
    }
    return mode;
}

/* Estimated single-GPU frame (ms) of a scene, from what bounds it on one
 * MI355X (build f9abbdcba9f8bfe1 / round 4 frames): camera rays of
 * a frame without recursion ~0.05 ns each (C2: 2.07 M rays in ~0.1 ms),
 * scattered rays (GI fan-out, reflect / refract chains) ~0.3 ns (C4: 345 M in
 * 87 ms, C3: 3.2 M in 1.7 ms), both growing with the mesh once it leaves the
 * caches (C5: 1 M triangles, 0.5 ns per camera ray). */
double est_frame_ms(int64_t px, int64_t tris, bool gi, bool secondary, const crt_renderer_settings *st) {
    double rays = 1.0;
    if (gi && st->diffuse_reflection_ray_count > 0) {   /* the GI tree: sum of count^d over the traced depths */
        double level = 1.0;
        for (uint32_t d = 1; d <= std::min<uint32_t>(st->max_ray_depth, 8); ++d) {
            level *= (double)st->diffuse_reflection_ray_count;
            rays += level;
        }
    } else if (secondary) {
        rays = 1.6;
    }
    const double ns = ((gi || secondary) ? 0.30 : 0.05) * (1.0 + (double)tris / 1e5);
    return (double)px * rays * ns * 1e-6;
}

/* GPUs a frame is spread over when the caller leaves the choice: one unless
 * the estimated frame is >= 2 ms (a shard then saves more than the copies and
 * the unpack cost), else about one per 0.6 ms of it, at most `visible`.
 * C2 / C3 stay on one GPU (8 shards: 1.04x / 1.12x), C4 / C5 spread (6.1x /
 * 7.5x). */
int auto_gpus(double est_ms, int visible) {
    if (visible <= 1 || est_ms < 2.0) return 1;
    return (int)std::max(1.0, std::min((double)visible, std::ceil(est_ms / 0.6)));
}

/* The replicas follow replica 0's measured plan (tuned once, there) and its
 * live mask. */
int share_plan(crt_hip_scene *sc, crt_hip_scene *r) {
    if (r->calib_walk != sc->calib_walk || r->calib_k != sc->calib_k || r->calib.size() != sc->calib.size() ||
        r->calibrate != sc->calibrate) {
        HIP_TRY(hipSetDevice(r->device));
        HIP_TRY(hipStreamSynchronize(r->stream));   /* its tile lists may still be read */
        r->calib = sc->calib;
        r->calib_k = sc->calib_k;
        r->calib_walk = sc->calib_walk;
        r->calibrate = sc->calibrate;
        free_plans(r);
        int64_t px = 0;
        const int rc = make_tile_plan(r, shard_buckets(r->info.width, r->info.height, r->info.bucket_size, 0, 1, &px),
                                      true, r->full);
        if (rc != CRT_OK) return rc;
    }
    if (r->live_mask.empty()) r->live_mask = sc->live_mask;
    return CRT_OK;
}

}  // namespace

int render_multi_into(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, hipStream_t stream) {
    std::vector<crt_hip_scene *> all{sc};
    all.insert(all.end(), sc->replicas.begin(), sc->replicas.end());
    const int G = (int)all.size();
    HIP_TRY(hipSetDevice(sc->device));
    if (sc->grid_empty) {
        HIP_TRY(hipMemsetAsync(d_rgb, 0, (size_t)sc->info.width * sc->info.height * 3 * sizeof(float), stream));
        return CRT_OK;
    }
    int rc = ensure_plans(sc, st, stream, true);
    if (rc != CRT_OK) return rc;
    if ((rc = ensure_live_mask(sc)) != CRT_OK) return rc;
    for (crt_hip_scene *r : sc->replicas)
        if ((rc = share_plan(sc, r)) != CRT_OK) return rc;
    const int64_t stride = crt_hip_compact_stride(sc, G);
    if (stride < 0) return (int)stride;
    HIP_TRY(hipSetDevice(sc->device));
    if (sc->mg_gather_floats < G * stride) {
        HIP_TRY(hipStreamSynchronize(stream));
        if (sc->mg_gather) (void)hipFree(sc->mg_gather);
        sc->mg_gather = nullptr;
        sc->mg_gather_floats = 0;
        HIP_TRY(hipMalloc(&sc->mg_gather, (size_t)(G * stride) * sizeof(float)));
        sc->mg_gather_floats = G * stride;
    }
    for (int i = 0; i < G; ++i) {
        crt_hip_scene *rep = all[i];
        HIP_TRY(hipSetDevice(rep->device));
        hipStream_t rs = i == 0 ? stream : rep->stream;
        float *dst = sc->mg_gather;
        if (i > 0) {
            if (rep->mg_packed_floats < stride) {
                HIP_TRY(hipStreamSynchronize(rs));
                if (rep->mg_packed) (void)hipFree(rep->mg_packed);
                rep->mg_packed = nullptr;
                rep->mg_packed_floats = 0;
                HIP_TRY(hipMalloc(&rep->mg_packed, (size_t)stride * sizeof(float)));
                rep->mg_packed_floats = stride;
            }
            dst = rep->mg_packed;
            /* the previous frame's unpack may still read this replica's slot */
            HIP_TRY(hipStreamWaitEvent(rs, sc->mg_done, 0));
        }
        if ((rc = render_shard_t(rep, st, i, G, dst, rs, true)) != CRT_OK) return rc;
        if (i > 0) {
            const int64_t n = crt_hip_compact_floats(rep, i, G);
            if (n < 0) return (int)n;
            if (n > 0)
                HIP_TRY(hipMemcpyPeerAsync(sc->mg_gather + (int64_t)i * stride, sc->device, rep->mg_packed,
                                           rep->device, (size_t)n * sizeof(float), rs));
            HIP_TRY(hipEventRecord(rep->mg_done, rs));
        }
    }
    HIP_TRY(hipSetDevice(sc->device));
    for (crt_hip_scene *r : sc->replicas) HIP_TRY(hipStreamWaitEvent(stream, r->mg_done, 0));
    if ((rc = unpack_shards_t<float>(sc, G, sc->mg_gather, d_rgb, stream, true)) != CRT_OK) return rc;
    HIP_TRY(hipEventRecord(sc->mg_done, stream));
    return CRT_OK;
}

bool multi_overflowed(crt_hip_scene *sc) {
    bool any = wf_overflowed(sc->wf, true);
    for (crt_hip_scene *r : sc->replicas) {
        (void)hipSetDevice(r->device);
        any = wf_overflowed(r->wf, true) || any;
    }
    (void)hipSetDevice(sc->device);
    return any;
}

void multi_free(crt_hip_scene *sc) {
    for (crt_hip_scene *r : sc->replicas) {
        (void)hipSetDevice(r->device);
        if (r->stream) (void)hipStreamSynchronize(r->stream);
        if (r->mg_packed) (void)hipFree(r->mg_packed);
        if (r->mg_done) (void)hipEventDestroy(r->mg_done);
        r->mg_packed = nullptr;
        r->mg_done = nullptr;
        crt_hip_scene_destroy(r);
    }
    sc->replicas.clear();
    (void)hipSetDevice(sc->device);
    if (sc->stream) (void)hipStreamSynchronize(sc->stream);
    if (sc->mg_gather) (void)hipFree(sc->mg_gather);
    if (sc->mg_done) (void)hipEventDestroy(sc->mg_done);
    sc->mg_gather = nullptr;
    sc->mg_done = nullptr;
}

}  // namespace crt_amd

extern "C" {

int crt_multi_probe_verdict(const float *multi, const float *single, int64_t n, int render_status) {
    if (n < 0 || (n > 0 && (!multi || !single))) return set_error(CRT_E_INVALID, "bad argument");
    return probe_verdict(multi, single, n, render_status);
}

int crt_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int crt_hip_scene_create_on(const crt_scene_desc *desc, const int32_t *devices, int32_t count, int flags,
                            crt_hip_scene **out) {
    if (!desc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = nullptr;
    const int mode = tree_mode(desc, flags);
    if (mode != CRT_SCENE_TREE_HOST && mode != CRT_SCENE_TREE_DEVICE) return set_error(CRT_E_INVALID, "bad tree build flag");
    const auto t0 = std::chrono::steady_clock::now();
    {   /* the libm tables this scene's frames read: built in the background from here on (crt_host_render.hip) */
        bool diffuse = false, refractive = false;
        for (int i = 0; i < desc->material_count && desc->materials; ++i) {
            diffuse = diffuse || desc->materials[i].type == CRT_MATERIAL_DIFFUSE;
            refractive = refractive || desc->materials[i].type == CRT_MATERIAL_REFRACTIVE;
        }
        start_host_tables(desc->gi_on && diffuse, desc->refractions_on && refractive);
    }
    std::unique_ptr<HostScene> hs(new HostScene());
    int rc = prepare_scene(desc, *hs, mode == CRT_SCENE_TREE_HOST);
    if (rc != CRT_OK) return rc;
    hs->device_bvh = (flags & CRT_SCENE_NO_DEVICE_BVH) == 0;
    if ((rc = upload_on(*hs, devices, count, out, flags)) != CRT_OK) return rc;
    (*out)->info.create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

int crt_auto_gpus(const crt_scene_desc *desc, const crt_renderer_settings *st, int visible) {
    if (!desc || !st) return set_error(CRT_E_INVALID, "null argument");
    if (const char *e = std::getenv("CRT_HIP_GPUS")) return std::max(1, std::min(visible, std::atoi(e)));
    int64_t tris = 0;
    for (int i = 0; i < desc->mesh_count && desc->meshes; ++i) tris += desc->meshes[i].index_count / 3;
    bool diffuse = false, secondary = false;
    for (int i = 0; i < desc->material_count && desc->materials; ++i) {
        const int t = desc->materials[i].type;
        diffuse = diffuse || t == CRT_MATERIAL_DIFFUSE;
        secondary = secondary || t == CRT_MATERIAL_REFLECTIVE || t == CRT_MATERIAL_REFRACTIVE;
    }
    const int64_t px = (int64_t)std::max(0, desc->camera.width) * std::max(0, desc->camera.height);
    return auto_gpus(est_frame_ms(px, tris, desc->gi_on && diffuse, secondary, st), visible);
}

int crt_auto_gpus_tree(const crt_tree_scene_desc *desc, const crt_renderer_settings *st, int visible) {
    if (!desc || !st) return set_error(CRT_E_INVALID, "null argument");
    if (const char *e = std::getenv("CRT_HIP_GPUS")) return std::max(1, std::min(visible, std::atoi(e)));
    /* unique triangles ~ leaf copies / 4 (the reference tree duplicates straddling triangles) */
    const int64_t copies = desc->leaf_offsets && desc->node_count > 0 ? desc->leaf_offsets[desc->node_count] : 0;
    bool diffuse = false, secondary = false;
    for (int i = 0; i < desc->material_count && desc->materials; ++i) {
        const int t = desc->materials[i].type;
        diffuse = diffuse || t == CRT_MATERIAL_DIFFUSE;
        secondary = secondary || t == CRT_MATERIAL_REFLECTIVE || t == CRT_MATERIAL_REFRACTIVE;
    }
    const int64_t px = (int64_t)std::max(0, desc->width) * std::max(0, desc->height);
    return auto_gpus(est_frame_ms(px, copies / 4, desc->gi_on && diffuse, secondary, st), visible);
}

static uint64_t first_n(int n) { return n >= 64 ? ~0ull : (1ull << n) - 1ull; }

int crt_hip_scene_create_auto(const crt_scene_desc *desc, const crt_renderer_settings *st, int flags,
                              crt_hip_scene **out) {
    const int n = crt_auto_gpus(desc, st, std::max(1, crt_hip_device_count()));
    if (n < 0) return n;
    return crt_hip_scene_create_mask(desc, first_n(n), flags, out);
}

int crt_hip_scene_from_tree_auto(const crt_tree_scene_desc *desc, const crt_renderer_settings *st,
                                 crt_hip_scene **out) {
    const int n = crt_auto_gpus_tree(desc, st, std::max(1, crt_hip_device_count()));
    if (n < 0) return n;
    return crt_hip_scene_from_tree_mask(desc, first_n(n), out);
}

int crt_hip_scene_create_mask(const crt_scene_desc *desc, uint64_t gpu_mask, int flags, crt_hip_scene **out) {
    std::vector<int32_t> devs;
    const int rc = mask_devices(gpu_mask, devs);
    if (rc != CRT_OK) return rc;
    return crt_hip_scene_create_on(desc, devs.data(), (int32_t)devs.size(), flags, out);
}

int crt_hip_scene_from_tree_on(const crt_tree_scene_desc *desc, const int32_t *devices, int32_t count,
                               crt_hip_scene **out) {
    if (!desc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_ptr<HostScene> hs(new HostScene());
    int rc = prepare_scene_from_tree(desc, *hs);
    if (rc != CRT_OK) return rc;
    const double prep = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((rc = upload_on(*hs, devices, count, out)) != CRT_OK) return rc;
    (*out)->info.prep_ms = prep;
    (*out)->info.create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

int crt_hip_scene_from_tree_mask(const crt_tree_scene_desc *desc, uint64_t gpu_mask, crt_hip_scene **out) {
    std::vector<int32_t> devs;
    const int rc = mask_devices(gpu_mask, devs);
    if (rc != CRT_OK) return rc;
    return crt_hip_scene_from_tree_on(desc, devs.data(), (int32_t)devs.size(), out);
}

int crt_hip_scene_devices(const crt_hip_scene *sc, int32_t *devices, int32_t cap) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    const int32_t n = 1 + (int32_t)sc->replicas.size();
    if (devices) {
        if (cap < n) return set_error(CRT_E_INVALID, "device buffer too small");
        devices[0] = sc->device;
        for (int32_t i = 1; i < n; ++i) devices[i] = sc->replicas[i - 1]->device;
    }
    return n;
}

int crt_hip_last_replica_ms(crt_hip_scene *sc, double *ms, int32_t cap) {
    if (!sc || !ms) return set_error(CRT_E_INVALID, "null argument");
    std::vector<crt_hip_scene *> all{sc};
    all.insert(all.end(), sc->replicas.begin(), sc->replicas.end());
    if (cap < (int32_t)all.size()) return set_error(CRT_E_INVALID, "buffer too small");
    for (size_t i = 0; i < all.size(); ++i) {
        crt_hip_scene *r = all[i];
        ms[i] = 0.0;
        if (!r->events_valid) continue;
        HIP_TRY(hipSetDevice(r->device));
        HIP_TRY(hipEventSynchronize(r->ev_stop));
        float f = 0.f;
        HIP_TRY(hipEventElapsedTime(&f, r->ev_start, r->ev_stop));
        ms[i] = f;
    }
    (void)hipSetDevice(sc->device);
    return (int)all.size();
}

}  // extern "C"
