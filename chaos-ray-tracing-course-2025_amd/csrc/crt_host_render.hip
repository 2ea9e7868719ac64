/*
 * crt_host_render.hip — host layer of the render path: GI / Fresnel tables,
 * measured tile plans and their tuning, the device record, the wavefront
 * orchestration (recorded level sizes, HIP graphs), kernel selection and
 * launch, live masks and shard plans.  Entry points: crt_api.hip.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crt_scene_impl.h"

namespace crt_amd {

struct GiTables { float *d = nullptr; };   /* 4 * 2^23 floats on one device */

std::mutex g_gi_mu;
std::map<int, GiTables> g_gi;              /* per device, process lifetime */
std::vector<float> g_gi_host;

constexpr int64_t kGiN = int64_t(1) << 23;

/* Host threads for the table builds: the process's CPU quota (the cgroup's
 * cpu.max, as on the GPU boxes: 16 CPUs of 256), else the hardware threads,
 * at most 64. */
unsigned table_threads() {
    unsigned n = std::thread::hardware_concurrency();
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long per = 0;
        if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
            const long long quota = std::atoll(q);
            if (quota > 0) n = std::min(n, (unsigned)std::max(1ll, quota / per));
        }
        std::fclose(f);
    }
    return std::max(1u, std::min(64u, n));
}

void build_gi_host_tables() {
    if (!g_gi_host.empty()) return;
    g_gi_host.resize((size_t)(4 * kGiN));
    /* (cos, sin) pairs: one 8-B read per angle (the tables are 64 MB each and
     * read at random: one cache line per angle instead of two) */
    float *pi2 = g_gi_host.data(), *tau2 = pi2 + 2 * kGiN;
    const unsigned nt = table_threads();
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < nt; ++w) {
        pool.emplace_back([=]() {
            for (int64_t m = w; m < kGiN; m += nt) {
                const float u = (float)m * (1.0f / 8388608.0f);          /* = uniform() exactly */
                const float a = kPi * u;                                  /* crt_renderer.cpp:68 */
                const float b = 2.0f * kPi * u;                           /* crt_renderer.cpp:71 */
                pi2[2 * m] = std::cos(a);
                pi2[2 * m + 1] = std::sin(a);
                tau2[2 * m] = std::cos(b);
                tau2[2 * m + 1] = std::sin(b);
            }
        });
    }
    for (auto &t : pool) t.join();
}


/* HIP loads a TU's code object at the first launch of one of its kernels:
 * launching an empty kernel of every render TU when a device first receives a
 * scene keeps that one-time load (~1.5 ms for all of them) out of the first
 * render, like the runtime's own initialisation at the scene upload. */
void warm_code_objects(int device, hipStream_t stream) {
    static std::mutex mu;
    static std::vector<int> done;
    std::lock_guard<std::mutex> g(mu);
    if (std::find(done.begin(), done.end(), device) != done.end()) return;
    done.push_back(device);
    hipLaunchKernelGGL(k_warm_render, dim3(1), dim3(64), 0, stream);
    hipLaunchKernelGGL(k_warm_gi, dim3(1), dim3(64), 0, stream);
    hipLaunchKernelGGL(k_warm_wf, dim3(1), dim3(64), 0, stream);
    hipLaunchKernelGGL(k_warm_side, dim3(1), dim3(64), 0, stream);
    hipLaunchKernelGGL(k_warm_bins, dim3(1), dim3(64), 0, stream);
    (void)hipGetLastError();
}

void wf_graphs_clear(WfBuffers &w) {
    if (w.graphs.empty()) return;
    /* a graph may still run on its set's stream: let the sets' streams drain */
    for (hipStream_t st : w.streams)
        if (st) (void)hipStreamSynchronize(st);
    for (auto &g : w.graphs) (void)hipGraphExecDestroy(g.exec);
    w.graphs.clear();
}

/* Set si is about to regrow its buffers: its last frame (levels and pixels)
 * must be done with them, and the graphs captured on them go. */
int wf_set_release(WfBuffers &wb, int si) {
    WfSet &w = wb.set[si];
    if (w.free_ev) HIP_TRY(hipEventSynchronize(w.free_ev));
    for (size_t i = 0; i < wb.graphs.size();) {
        if (wb.graphs[i].set == si) {
            (void)hipGraphExecDestroy(wb.graphs[i].exec);
            wb.graphs.erase(wb.graphs.begin() + (std::ptrdiff_t)i);
        } else {
            ++i;
        }
    }
    return CRT_OK;
}



/* Every camera ray of the frame takes the fast box path of make_ray_rcp:
 * node planes and the camera origin inside the exact-division window, and
 * d = normalize(v R) with |d_i| <= 2^20 for every pixel.  v = (dx, dy, -1),
 * |dx| <= aspect tan(fov/2), |dy| <= tan(fov/2) (crt_camera.cpp:7-35): with R
 * finite and bounded, w = v R is finite; with sigma_min(R) >= |det R| /
 * |R|_F^2 far above the rounding of v R (and above 2^-50, so |w|^2 stays
 * normal), w cannot round to 0 — then each |d_i| = |w_i| / |w| <= 1. */
bool camera_rays_fast(const DCamera &c, bool planes_ok) {
    if (!planes_ok) return false;
    for (int k = 0; k < 3; ++k)
        if (!coord_ok(c.loc[k])) return false;
    const double ta = std::fabs((double)c.tan_half_fov), aa = std::fabs((double)c.aspect) * ta;
    if (!std::isfinite(ta) || !std::isfinite(aa) || ta > 0x1p40 || aa > 0x1p40) return false;
    double R[9], fro = 0.0, mx = 0.0;
    for (int k = 0; k < 9; ++k) {
        R[k] = c.rot[k];
        if (!std::isfinite(R[k]) || std::fabs(R[k]) > 0x1p40) return false;
        fro += R[k] * R[k];
        mx = std::max(mx, std::fabs(R[k]));
    }
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (!(fro > 0.0)) return false;
    const double smin = std::fabs(det) / fro;
    return smin > 0x1p-50 && smin > 1e-4 * (2.0 + aa + ta) * mx;
}

int make_tile_plan(crt_hip_scene *sc, const std::vector<DBucket> &buckets, bool full_frame, ShardPlan &plan) {
    std::vector<Tile> tiles;
    const int W = sc->info.width;
    if (full_frame) {
        for (int y = 0; y < sc->info.height; y += 8)
            for (int x = 0; x < W; x += 8)
                tiles.push_back(Tile{x, y, std::min(8, W - x), std::min(8, sc->info.height - y),
                                     (int64_t)y * W + x, W, 0});
        plan.packed_pixels = (int64_t)W * sc->info.height;
    } else {
        int64_t total = 0;
        for (const DBucket &b : buckets) {
            for (int ty = 0; ty < b.h; ty += 8)
                for (int tx = 0; tx < b.w; tx += 8)
                    tiles.push_back(Tile{b.x + tx, b.y + ty, std::min(8, b.w - tx), std::min(8, b.h - ty),
                                         b.packed_offset + (int64_t)ty * b.w + tx, b.w, 0});
            total += (int64_t)b.w * b.h;
        }
        plan.packed_pixels = total;
    }
    if (bins_active(sc) && !tiles.empty()) {
        /* camera bins: each frame's binning lists the cells by list length
         * for the render grid, heaviest first (crt_bins.hip bins_plan) */
        plan.cost.clear();
    } else if (!sc->calib.empty() && !tiles.empty()) {
        /* measured costs: split as calibrated, heaviest first */
        const int tx = (W + 7) / 8;
        std::vector<std::pair<float, Tile>> out;
        out.reserve(tiles.size() * 2);
        for (const Tile &t : tiles) {
            const size_t k = (size_t)(t.y / 8) * tx + t.x / 8;
            const auto &cal = sc->calib[k];
            const bool aligned = t.x % 8 == 0 && t.y % 8 == 0 && t.w == std::min(8, W - t.x) &&
                                 t.h == std::min(8, sc->info.height - t.y);
            if (aligned) {
                for (const auto &st : cal)
                    out.push_back({st.cost, Tile{t.x + st.dx, t.y + st.dy, st.w, st.h,
                                                 t.out_base + (int64_t)st.dy * t.out_stride + st.dx, t.out_stride, 0}});
            } else {   /* bucket grid not on the 8x8 grid: keep the tile, cost of its 8x8 cell */
                float c = 0.f;
                for (const auto &st : cal) c += st.cost;
                out.push_back({c, t});
            }
        }
        std::stable_sort(out.begin(), out.end(),
                         [](const std::pair<float, Tile> &a, const std::pair<float, Tile> &b) { return a.first > b.first; });
        tiles.clear();
        plan.cost.clear();
        for (const auto &e : out) {
            tiles.push_back(e.second);
            plan.cost.push_back(e.first);
        }
        /* issue priority for the heaviest waves, at most prio_tiles of them and
         * only those costing more than prio_min x the mean per wave slot */
        double csum = 0.0;
        for (float c : plan.cost) csum += c;
        const double slot_cost = csum / std::max(1, sc->wave_slots);
        for (size_t k = 0; k < tiles.size() && (int)k < sc->prio_tiles; ++k)
            tiles[k].prio = plan.cost[k] > sc->prio_min * slot_cost ? 1 : 0;
    } else if (!tiles.empty() && !sc->tile_work.empty()) {
        /* dispatch the expensive tiles first so the longest waves start at t=0;
         * with a sharing walk, split the heaviest tiles so each of their waves
         * carries fewer rays and the rest of its lanes help (4x4 or 2x2 pixels) */
        const int tx = (W + 7) / 8;
        auto work = [&](const Tile &t) { return sc->tile_work[(size_t)(t.y / 8) * tx + t.x / 8]; };
        double wsum = 0.0;
        for (const Tile &t : tiles) wsum += work(t);
        const float slot_work = (float)(wsum / sc->wave_slots);
        std::vector<Tile> split;
        if (slot_work > 0.f && (sc->split4 > 0.f || sc->split16 > 0.f)) {
            for (const Tile &t : tiles) {
                const float w = work(t) / slot_work;
                const int sub = (sc->split16 > 0.f && w >= sc->split16) ? 2 : (sc->split4 > 0.f && w >= sc->split4) ? 4 : 8;
                for (int yy = 0; yy < t.h; yy += sub)
                    for (int xx = 0; xx < t.w; xx += sub)
                        split.push_back(Tile{t.x + xx, t.y + yy, std::min(sub, t.w - xx), std::min(sub, t.h - yy),
                                             t.out_base + (int64_t)yy * t.out_stride + xx, t.out_stride, 0});
            }
            tiles.swap(split);
        }
        std::vector<std::pair<float, int>> key(tiles.size());
        for (size_t k = 0; k < tiles.size(); ++k) key[k] = {-work(tiles[k]), (int)k};
        std::stable_sort(key.begin(), key.end());
        std::vector<Tile> sorted(tiles.size());
        for (size_t k = 0; k < tiles.size(); ++k) sorted[k] = tiles[key[k].second];
        tiles.swap(sorted);
    }
    plan.ntiles = (int)tiles.size();
    plan.waves = plan.ntiles;
    plan.bp = BinsPlan{};
    plan.has_small = false;
    for (const Tile &t : tiles) plan.has_small = plan.has_small || t.w * t.h <= 16;
    plan.tiles = tiles;
    if (!tiles.empty()) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, tiles.size() * sizeof(Tile)));
        HIP_TRY(hipMemcpy(p, tiles.data(), tiles.size() * sizeof(Tile), hipMemcpyHostToDevice));
        sc->plan_allocs.push_back(p);
        plan.d_tiles = static_cast<Tile *>(p);
        if (bins_active(sc)) return bins_plan(sc, plan);
    }
    return CRT_OK;
}

/* Probe costs of a tile list (k_probe_tiles) with walk `walk`, synchronously. */
int probe_tiles(crt_hip_scene *sc, const DeviceScene *d_scene, int walk, const std::vector<Tile> &tiles,
                std::vector<uint32_t> &cost, hipStream_t stream) {
    cost.assign(tiles.size(), 0u);
    if (tiles.empty()) return CRT_OK;
    /* one per-scene buffer for every round (a hipFree would drain the device) */
    const size_t cbytes = (tiles.size() * sizeof(uint32_t) + 255) & ~size_t(255);
    const size_t need = cbytes + tiles.size() * sizeof(Tile);
    if (need > sc->probe_cap) {
        if (sc->probe_buf) HIP_TRY(hipFree(sc->probe_buf));
        sc->probe_buf = nullptr;
        sc->probe_cap = 0;
        HIP_TRY(hipMalloc(&sc->probe_buf, need));
        sc->probe_cap = need;
    }
    void *dc = sc->probe_buf, *dt = static_cast<char *>(sc->probe_buf) + cbytes;
    hipError_t e = hipMemcpyAsync(dt, tiles.data(), tiles.size() * sizeof(Tile), hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) {
        const int n = (int)tiles.size();
        const dim3 grid((unsigned)((n + 3) / 4));
        const Tile *t = static_cast<const Tile *>(dt);
        uint32_t *c = static_cast<uint32_t *>(dc);
        switch (walk) {
        case 7: hipLaunchKernelGGL(k_probe_tiles<7>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        case 12: hipLaunchKernelGGL(k_probe_tiles<12>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        case 13: hipLaunchKernelGGL(k_probe_tiles<13>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        case 14: hipLaunchKernelGGL(k_probe_tiles<14>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        default: hipLaunchKernelGGL(k_probe_tiles<8>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        }
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(cost.data(), dc, tiles.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("tile probe: ") + hipGetErrorString(e));
    return CRT_OK;
}

/* Measured-cost tile plan.  The frame's 8x8 tiles are probed with the primary
 * walk; a tile whose wave cost exceeds k x (total cost / resident wave slots)
 * would run past the ideal makespan, so it is split into quadrants, which are
 * probed in turn, down to calib_min pixels.  The leaves and their costs give
 * every later plan (full frame and shards): split as measured, dispatched
 * heaviest first.  Results do not depend on the plan. */
int calibrate_plan(crt_hip_scene *sc, const DeviceScene *d_scene, int walk, hipStream_t stream) {
    const int W = sc->info.width, H = sc->info.height;
    const int tx = (W + 7) / 8, ty = (H + 7) / 8;
    struct Item { int k; int32_t dx, dy, w, h; };
    std::vector<Item> cur;
    cur.reserve((size_t)tx * ty);
    for (int y = 0; y < ty; ++y)
        for (int x = 0; x < tx; ++x)
            cur.push_back(Item{y * tx + x, 0, 0, std::min(8, W - 8 * x), std::min(8, H - 8 * y)});
    std::vector<std::vector<crt_hip_scene::SubTile>> cal((size_t)tx * ty);
    double thresh = -1.0;
    int side = 8;
    while (!cur.empty()) {
        std::vector<Tile> tl(cur.size());
        for (size_t i = 0; i < cur.size(); ++i) {
            const int x0 = 8 * (cur[i].k % tx) + cur[i].dx, y0 = 8 * (cur[i].k / tx) + cur[i].dy;
            tl[i] = Tile{x0, y0, cur[i].w, cur[i].h, (int64_t)y0 * W + x0, W, 0};
        }
        std::vector<uint32_t> cost;
        const int rc = probe_tiles(sc, d_scene, walk, tl, cost, stream);
        if (rc != CRT_OK) return rc;
        if (thresh < 0.0) {
            double sum = 0.0;
            for (uint32_t c : cost) sum += c;
            thresh = sc->calib_k * sum / std::max(1, sc->wave_slots);
        }
        std::vector<Item> next;
        const int half = side / 2;
        for (size_t i = 0; i < cur.size(); ++i) {
            const Item &it = cur[i];
            if ((double)cost[i] > thresh && half >= sc->calib_min && (it.w > half || it.h > half)) {
                for (int yy = 0; yy < it.h; yy += half)
                    for (int xx = 0; xx < it.w; xx += half)
                        next.push_back(Item{it.k, it.dx + xx, it.dy + yy, std::min(half, it.w - xx), std::min(half, it.h - yy)});
            } else {
                cal[it.k].push_back(crt_hip_scene::SubTile{it.dx, it.dy, it.w, it.h, (float)cost[i]});
            }
        }
        cur.swap(next);
        side = half;
    }
    sc->calib.swap(cal);
    sc->calib_walk = walk;
    return CRT_OK;
}

void free_plans(crt_hip_scene *sc) {
    for (void *p : sc->plan_allocs) (void)hipFree(p);
    sc->plan_allocs.clear();
    { sc->wf.recs.clear(); ++sc->wf.epoch; }   /* keyed by the tile lists' device pointers */
    wf_graphs_clear(sc->wf);
    sc->full = ShardPlan{};
    sc->shard_plans.clear();
    sc->bins.last = -1;   /* the work lists were the freed plans' */
#ifdef CRT_BINS_TRACE   /* diagnostic builds: the binning's decisions on stderr */
    std::fprintf(stderr, "free_plans\n");
#endif
    sc->compact_plans.clear();
}

/* powf(x, 5.0f) for x = k * 2^-24, k = -2^24 .. 2^24 (fresnel_of), computed
 * by this process's libm — the one the reference's std::pow resolves to on
 * this host.  Called through a volatile pointer so the compiler cannot
 * replace the libm call by its own expansion. */
constexpr int64_t kPow5N = (int64_t(1) << 25) + 1;
std::mutex g_pow5_mu;
std::map<int, float *> g_pow5;             /* per device, process lifetime */
std::vector<float> g_pow5_host;

void build_pow5_host_table() {
    if (!g_pow5_host.empty()) return;
    g_pow5_host.resize((size_t)kPow5N);
    float *t = g_pow5_host.data();
    const unsigned nt = table_threads();
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < nt; ++w) {
        pool.emplace_back([=]() {
            float (*volatile pw)(float, float) = ::powf;
            for (int64_t k = w; k < kPow5N; k += nt) {
                const float x = (float)(k - (int64_t(1) << 24)) * (1.0f / 16777216.0f);   /* exact */
                t[k] = pw(x, 5.0f);
            }
        });
    }
    for (auto &th : pool) th.join();
}

/* The host tables are built once per process, in the background from the
 * first scene create that needs them (start_host_tables), overlapping the
 * rest of the create; the device copy waits for them (ensure_*). */
std::mutex g_fut_mu;
std::shared_future<void> g_gi_fut, g_pow5_fut;

void start_host_tables(bool gi, bool pow5) {
    std::lock_guard<std::mutex> g(g_fut_mu);
    if (gi && !g_gi_fut.valid()) g_gi_fut = std::async(std::launch::async, build_gi_host_tables).share();
    if (pow5 && !g_pow5_fut.valid()) g_pow5_fut = std::async(std::launch::async, build_pow5_host_table).share();
}

int ensure_pow5_table(crt_hip_scene *sc) {
    if (sc->ds.pow5) return CRT_OK;
    start_host_tables(false, true);
    std::lock_guard<std::mutex> g(g_pow5_mu);
    float *&d = g_pow5[sc->device];
    if (!d) {
        g_pow5_fut.wait();
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)kPow5N * sizeof(float)));
        HIP_TRY(hipMemcpy(p, g_pow5_host.data(), (size_t)kPow5N * sizeof(float), hipMemcpyHostToDevice));
        d = static_cast<float *>(p);
    }
    sc->ds.pow5 = d;
    return CRT_OK;
}

int ensure_gi_tables(crt_hip_scene *sc) {
    if (sc->ds.gi_pi) return CRT_OK;
    start_host_tables(true, false);
    std::lock_guard<std::mutex> g(g_gi_mu);
    GiTables &t = g_gi[sc->device];
    if (!t.d) {
        g_gi_fut.wait();
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)(4 * kGiN) * sizeof(float)));
        HIP_TRY(hipMemcpy(p, g_gi_host.data(), (size_t)(4 * kGiN) * sizeof(float), hipMemcpyHostToDevice));
        t.d = static_cast<float *>(p);
    }
    sc->ds.gi_pi = t.d;
    sc->ds.gi_2pi = t.d + 2 * kGiN;
    return CRT_OK;
}

/* Light bins (crt_light_bins.cpp; option "light_bins": on C2 the deferred
 * shadow rays over them take 0.396 ms a frame, against 0.469 over the BVH
 * wave walk; traced inline, 0.427 against 0.416) for the shadow rays, built
 * at the first shadow-ray frame with them on, from the camera bins' per-triangle templates (on the
 * device since the create) and the lights: once per scene, the camera does
 * not enter them.  Rays passing their light within e_max = max(0.02,
 * 1.25 |shadow_bias|) of the first frame are decided by them (larger biases
 * later: the BVH decides).  No templates (no camera bins) or no light taking
 * bins: the BVH walks as before. */
#ifndef CRT_LBINS_N
#define CRT_LBINS_N 128   /* light bins: cells a cube-face side (C2 with shadows: 64 0.400, 128 0.366-0.377 ms) */
#endif
int ensure_light_bins(crt_hip_scene *sc, const crt_renderer_settings *st) {
    if (!sc->light_bins || sc->lbins_tried) {
        sc->ds.lbin_n = sc->light_bins ? sc->lbins_n : 0;
        return CRT_OK;
    }
    sc->lbins_tried = true;
    const int nt = sc->bins.nt, nl = sc->ds.light_count;
    if (!sc->bins.tpl || nt <= 0 || nl <= 0 || !sc->ds.bnodes) return CRT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<CamCand> tpl((size_t)nt);
    std::vector<DLight> lights((size_t)nl);
    HIP_TRY(hipMemcpy(tpl.data(), sc->bins.tpl, tpl.size() * sizeof(CamCand), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(lights.data(), sc->ds.lights, lights.size() * sizeof(DLight), hipMemcpyDeviceToHost));
    const double bias = std::isfinite(st->shadow_bias) ? std::fabs((double)st->shadow_bias) : 0.0;
    LightBinsHost L;
    if (!build_light_bins(tpl.data(), nt, lights.data(), nl, std::max(0.02, 1.25 * bias), CRT_LBINS_N, L)) return CRT_OK;
    UploadBatch ub;
    ub.add(L.par, &sc->ds.lbin_par);
    ub.add(L.off, &sc->ds.lbin_off);
    ub.add(L.recs, &sc->ds.lbins, 1);   /* + a zero record: the wave walk loads one past a list */
    const int rc = ub.flush(sc);
    if (rc != CRT_OK) return rc;
    sc->lbins_n = L.n;
    sc->lbins_records = (int64_t)L.recs.size();
    sc->ds.lbin_n = sc->light_bins ? L.n : 0;
    sc->lbins_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

/* Deferred shadow rays of a frame without recursion (option "shadow_defer"):
 * the render kernel writes a group of records per diffuse hit (crt_shade.h
 * shade_hit_shadowed), k_shadow_vis traces one ray a lane over the whole
 * chip, k_shadow_compose writes the diffuse pixels.  Inline, a wave traced its
 * tile's rays light after light and the frame ended with its slowest waves
 * (C2: ~90 % of the SIMD slots idle).  The buffers hold a group per pixel;
 * frames on another stream wait for the previous deferred frame's compose. */
int shadow_defer_begin(crt_hip_scene *sc, DSettings &ds, hipStream_t stream) {
    const int nl = sc->ds.light_count;
    const int64_t cap = ((int64_t)sc->info.width * sc->info.height + 63) & ~int64_t(63);   /* whole chunks of 64 groups */
    const int64_t bytes = cap * nl * (int64_t)(sizeof(ShRay) + sizeof(ShCon));
    if (nl <= 0 || cap <= 0 || cap > INT32_MAX || bytes > (int64_t(4) << 30)) return CRT_OK;   /* inline */
    if (!sc->sh_count) {
        HIP_TRY(hipMalloc(&sc->sh_count, 256));
        HIP_TRY(hipEventCreateWithFlags(&sc->sh_done, hipEventDisableTiming));
    }
    if (bytes > sc->sh_bytes) {
        HIP_TRY(hipDeviceSynchronize());
        if (sc->sh_buf) (void)hipFree(sc->sh_buf);
        sc->sh_buf = nullptr;
        sc->sh_bytes = 0;
        HIP_TRY(hipMalloc(&sc->sh_buf, (size_t)bytes));
        sc->sh_bytes = bytes;
        sc->sh_stream = nullptr;
    }
    if (sc->sh_stream && sc->sh_stream != stream) HIP_TRY(hipStreamWaitEvent(stream, sc->sh_done, 0));
    HIP_TRY(hipMemsetAsync(sc->sh_count, 0, sizeof(int32_t), stream));
    ds.sh_rays = static_cast<ShRay *>(sc->sh_buf);
    ds.sh_con = reinterpret_cast<ShCon *>(static_cast<char *>(sc->sh_buf) + cap * nl * (int64_t)sizeof(ShRay));
    ds.sh_count = sc->sh_count;
    ds.sh_cap = (int32_t)cap;
    return CRT_OK;
}

int shadow_defer_end(crt_hip_scene *sc, const DeviceScene *d_scene, const DSettings &ds, float *d_out,
                     hipStream_t stream) {
    if (!ds.sh_rays) return CRT_OK;
    hipLaunchKernelGGL(k_shadow_vis, dim3(2048), dim3(256), 0, stream, d_scene, ds.sh_rays, ds.sh_con, ds.sh_count,
                       ds.sh_cap);
    HIP_TRY(hipGetLastError());
    const unsigned cb = (unsigned)std::min<int64_t>(4096, ((int64_t)ds.sh_cap + 255) / 256);
    hipLaunchKernelGGL(k_shadow_compose, dim3(cb), dim3(256), 0, stream, d_scene, ds, ds.sh_rays, ds.sh_con,
                       ds.sh_count, ds.sh_cap, d_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(sc->sh_done, stream));
    sc->sh_stream = stream;
    return CRT_OK;
}

/* Device copy of sc->ds for the render kernels.  When the host record
 * changed (a new camera, the first GI frame's tables) the next slot of a ring
 * of kRecRing records takes it, written on `stream` by a one-thread kernel
 * (the record travels as its by-value argument: no host sync, no staging);
 * frames issued before keep reading their own slot.  Ordering costs nothing
 * on one stream: a slot is rewritten after its last frame when both were
 * issued on the same stream, and read after its write by frames on the
 * writing stream.  Only across streams an event is recorded — on the stream
 * of the slot's last frame, or of its write, at the time another stream needs
 * it (later on that stream than strictly needed, never earlier). */
int sync_device_record(crt_hip_scene *sc, const DeviceScene **out, hipStream_t stream) {
    if (!sc->d_ring) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, kRecRing * sizeof(DeviceScene)));
        sc->allocs.push_back(p);
        sc->d_ring = static_cast<DeviceScene *>(p);
        for (int j = 0; j < kRecRing; ++j) {
            HIP_TRY(hipEventCreateWithFlags(&sc->rec_up[j], CRT_PIPE_EV_FLAGS));
            HIP_TRY(hipEventCreateWithFlags(&sc->rec_use[j], CRT_PIPE_EV_FLAGS));
        }
    }
    if (sc->ring_cur < 0 || std::memcmp(&sc->ds_uploaded, &sc->ds, sizeof(DeviceScene)) != 0) {
        if (sc->ring_cur >= 0) sc->rec_use_stream[sc->ring_cur] = sc->rec_last_stream;
        sc->rec_last_stream = nullptr;
        const int j = (sc->ring_cur + 1) % kRecRing;
        /* slot j's last frame: implied on this stream, else an event behind it */
        if (sc->rec_use_stream[j] && sc->rec_use_stream[j] != stream) {
            HIP_TRY(hipEventRecord(sc->rec_use[j], sc->rec_use_stream[j]));
            HIP_TRY(hipStreamWaitEvent(stream, sc->rec_use[j], 0));
        }
        /* ... and wavefront levels that read it on their sets' streams */
        for (WfSet &w : sc->wf.set)   /* (a set's done_ev is its latest frame's: it covers the set's earlier ones) */
            if ((w.rec_slots >> j) & 1u) {
                if (w.done_ev) HIP_TRY(hipStreamWaitEvent(stream, w.done_ev, 0));
                w.rec_slots &= ~(1u << j);
            }
        sc->rec_use_stream[j] = nullptr;
        hipLaunchKernelGGL(k_put_record, dim3(1), dim3(64), 0, stream, sc->d_ring + j, sc->ds);
        HIP_TRY(hipGetLastError());
        sc->ring_cur = j;
        sc->rec_up_stream = stream;
        sc->rec_up_done = false;
        sc->rec_up_recorded = false;
        sc->d_ds = sc->d_ring + j;
        std::memcpy(&sc->ds_uploaded, &sc->ds, sizeof(DeviceScene));
        ++sc->records_written;
    } else {
        const int rc = wait_device_record(sc, stream);
        if (rc != CRT_OK) return rc;
    }
    *out = sc->d_ds;
    return CRT_OK;
}

/* `stream` will read the current record: after its write (nothing to wait
 * for on the stream that wrote it, or once the write is done). */
int wait_device_record(crt_hip_scene *sc, hipStream_t stream) {
    if (sc->ring_cur < 0 || sc->rec_up_done || stream == sc->rec_up_stream) return CRT_OK;
    if (!sc->rec_up_recorded) {
        HIP_TRY(hipEventRecord(sc->rec_up[sc->ring_cur], sc->rec_up_stream));
        sc->rec_up_recorded = true;
    }
    if (hipEventQuery(sc->rec_up[sc->ring_cur]) == hipSuccess) {
        sc->rec_up_done = true;   /* written: every stream may read it */
        return CRT_OK;
    }
    HIP_TRY(hipStreamWaitEvent(stream, sc->rec_up[sc->ring_cur], 0));
    return CRT_OK;
}

/* The frame issued on `stream` is the current record's last reader so far
 * (frames of one record on several streams: the API asks callers to order
 * them, include/crt_hip.h crt_hip_render_device). */
int used_device_record(crt_hip_scene *sc, hipStream_t stream) {
    if (!sc->rec_read_by_set) sc->rec_last_stream = stream;
    sc->rec_read_by_set = false;
    return CRT_OK;
}

int check_settings(const crt_renderer_settings *st) {
    if (!st) return set_error(CRT_E_INVALID, "null settings");
    return CRT_OK;
}

/* Frames with reflective / refractive recursion and no GI taken by the GI
 * kernel's per-lane state machine (k_render_gi; option "rec_machine"): needs
 * the BVH and the pixel-refill head, at most 63 levels. */
bool rec_machine_on(const crt_hip_scene *sc, const crt_renderer_settings *st) {
    return sc->rec_machine && sc->ds.bnodes && sc->d_next_px && sc->secondary != 4 && sc->secondary != 10 &&
           st->max_ray_depth <= 63 && (int64_t)sc->info.width * sc->info.height < INT32_MAX;
}

/* The packet walk camera rays take: walk 8 becomes its fast-only build 12
 * when the host has proven every camera ray fast. */
int camera_walk(const crt_hip_scene *sc, int trav) {
    if (trav == 14 && !sc->ds.bnodes) trav = 8;   /* no BVH built for this scene */
    return (trav == 8 && sc->camera_fast) ? (sc->window_walk ? 13 : 12) : trav;
}

/* The primary walk a tile plan is measured with (-1: keep the estimate plan):
 * camera rays of diffuse frames and level 0 of the wavefront recursion. */
int plan_walk(const crt_hip_scene *sc, const crt_renderer_settings *st) {
    const bool gi = sc->info.gi_on && sc->has_diffuse && st->diffuse_reflection_ray_count > 0;
    const bool full = gi || sc->has_secondary;
    if (gi) return -1;
    if (bins_active(sc)) return -1;   /* camera bins: no plan to measure */
    if (full && rec_machine_on(sc, st)) return -1;   /* per-lane state machine: pixels pulled in order */
    if (full) return sc->wavefront ? camera_walk(sc, sc->traversal == 8 ? 8 : 7) : -1;
    return camera_walk(sc, sc->traversal);
}

/* Calibrate the tile plan for this frame's primary walk once (see
 * calibrate_plan), then rebuild the full-frame plan; shard plans are rebuilt
 * on their next use. */
/* Split threshold of the calibrated plan (calibrate_plan: a tile whose
 * measured cost exceeds k x mean cost per wave slot is split).  The best k
 * depends on the scene and on how the walks' step counts relate to time (a
 * split tile's window waves cost more per step than a packet wave), so by
 * default it is tuned: each candidate's plan renders the frame (one untimed,
 * five timed launches, median taken) and the fastest plan is kept.  Only the
 * tiling changes with k; every plan produces the same image bits.
 * calibrate = 2 (or env CRT_CALIB_K) keeps the given k instead.  The grid
 * is fine around 2-3: C2's frame moves by 5-10 % between neighbouring k. */
static const float kCalibK[] = {1.5f, 1.75f, 2.0f, 2.25f, 2.5f, 2.75f, 3.0f, 3.5f, 4.0f, 6.0f};


int ensure_plans(crt_hip_scene *sc, const crt_renderer_settings *st, hipStream_t stream, bool render) {
    if (!sc->calibrate || sc->grid_empty) return CRT_OK;
    const int walk = plan_walk(sc, st);
    /* the packet walk's camera-fast forms (12, 13: chosen per camera pose) share
     * one plan with it: a moving camera does not calibrate again */
    auto family = [](int w) { return w == 12 || w == 13 ? 8 : w; };
    if (walk < 0 || family(walk) == family(sc->calib_walk)) return CRT_OK;
    /* a one-shot caller's frame (calibrate 2, render entry points): the first
     * frame of this walk renders with the plan at hand (the scene's estimate
     * plan: C2 0.135 vs 0.108 ms) instead of paying the probes (~2.5 ms,
     * profiles/r03/cold); the second frame calibrates */
    if (render && sc->calibrate == 2 && sc->calib_defer && sc->calib_deferred_walk != walk) {
        sc->calib_deferred_walk = walk;
        return CRT_OK;
    }
    const DeviceScene *d_scene = nullptr;
    int rc = sync_device_record(sc, &d_scene, stream);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());   /* earlier frames may still read the old tile lists */
    int64_t px = 0;
    const std::vector<DBucket> all = shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, 0, 1, &px);
    if (sc->calibrate == 2 || sc->calib_tuned) {
        if ((rc = calibrate_plan(sc, d_scene, walk, stream)) != CRT_OK) return rc;
        free_plans(sc);
        return make_tile_plan(sc, all, true, sc->full);
    }
    float *scratch = nullptr;
    HIP_TRY(hipMalloc(&scratch, (size_t)sc->info.width * sc->info.height * 3 * sizeof(float)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float best_ms = INFINITY, best_k = kCalibK[0];
    std::vector<std::vector<crt_hip_scene::SubTile>> best_cal;
    auto tune = [&]() -> int {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        for (const float k : kCalibK) {
            sc->calib_k = k;
            int r = calibrate_plan(sc, d_scene, walk, stream);
            if (r != CRT_OK) return r;
            free_plans(sc);
            if ((r = make_tile_plan(sc, all, true, sc->full)) != CRT_OK) return r;
            std::vector<float> reps;
            for (int rep = 0; rep < 6; ++rep) {
                HIP_TRY(hipEventRecord(e0, stream));
                if ((r = launch_render(sc, st, sc->full, scratch, stream, false)) != CRT_OK) return r;
                HIP_TRY(hipEventRecord(e1, stream));
                HIP_TRY(hipEventSynchronize(e1));
                (void)wf_overflowed(sc->wf, true);   /* a wrong trial frame only drops the recorded level sizes */
                float t = 0.f;
                HIP_TRY(hipEventElapsedTime(&t, e0, e1));
                if (rep > 0) reps.push_back(t);
            }
            std::sort(reps.begin(), reps.end());
            const float ms = reps[reps.size() / 2];   /* median of 5 timed frames */
            if (ms < best_ms) {
                best_ms = ms;
                best_k = k;
                best_cal = sc->calib;
            }
        }
        return CRT_OK;
    };
    rc = tune();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(scratch);
    if (rc != CRT_OK) return rc;
    sc->calib_k = best_k;
    sc->calib_tuned = true;
    sc->calib.swap(best_cal);
    sc->calib_walk = walk;
    free_plans(sc);
    return make_tile_plan(sc, all, true, sc->full);
}

DSettings to_dsettings(const crt_renderer_settings *st) {
    DSettings d;
    d.max_ray_depth = st->max_ray_depth;
    d.diffuse_reflection_ray_count = st->diffuse_reflection_ray_count;
    d.shadow_bias = st->shadow_bias;
    d.reflection_bias = st->reflection_bias;
    d.diffuse_reflection_bias = st->diffuse_reflection_bias;
    d.refraction_bias = st->refraction_bias;
    d.sh_rays = nullptr;   /* shadow rays inline unless a frame defers them (shadow_defer_begin) */
    d.sh_con = nullptr;
    d.sh_count = nullptr;
    d.sh_cap = 0;
    return d;
}

int wf_grow_ids(WfBuffers &wb, int si, int64_t need, int64_t used, hipStream_t stream) {
    WfSet &w = wb.set[si];
    if (need <= w.cap) return CRT_OK;
    {   /* (mid-frame regrowth of a read-back frame: its stream waited for free_ev and was synchronised) */
        const int rc = wf_set_release(wb, si);
        if (rc != CRT_OK) return rc;
    }
    const int64_t cap = std::max<int64_t>(need, 2 * w.cap);
    void *pn = nullptr, *pc = nullptr;
    HIP_TRY(hipMalloc(&pn, (size_t)cap * sizeof(WNode)));
    HIP_TRY(hipMalloc(&pc, (size_t)cap * sizeof(DVec4)));
    if (used > 0) {
        HIP_TRY(hipMemcpyAsync(pn, w.nodes, (size_t)used * sizeof(WNode), hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipMemcpyAsync(pc, w.cols, (size_t)used * sizeof(DVec4), hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));
    }
    if (w.nodes) (void)hipFree(w.nodes);
    if (w.cols) (void)hipFree(w.cols);
    w.nodes = static_cast<WNode *>(pn);
    w.cols = static_cast<DVec4 *>(pc);
    w.cap = cap;
    return CRT_OK;
}

int wf_grow_queue(WfBuffers &wb, int si, int k, int64_t need) {
    WfSet &w = wb.set[si];
    if (need <= w.qcap[k]) return CRT_OK;
    {
        const int rc = wf_set_release(wb, si);
        if (rc != CRT_OK) return rc;
    }
    const int64_t cap = std::max<int64_t>(need, 2 * w.qcap[k]);
    if (w.q[k]) (void)hipFree(w.q[k]);
    w.q[k] = nullptr;
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)cap * sizeof(WRay)));
    w.q[k] = static_cast<WRay *>(p);
    w.qcap[k] = cap;
    return CRT_OK;
}

void wf_free(WfBuffers &wb) {
    wf_graphs_clear(wb);
    for (hipStream_t st : wb.streams)
        if (st) (void)hipStreamSynchronize(st);
    for (WfSet &w : wb.set) {
        for (void *p : {(void *)w.nodes, (void *)w.cols, (void *)w.q[0], (void *)w.q[1], (void *)w.counts, (void *)w.d_flag})
            if (p) (void)hipFree(p);
        if (w.h_flag) (void)hipHostFree(w.h_flag);
        if (w.h_counts) (void)hipHostFree(w.h_counts);
        for (hipEvent_t e : {w.flag_ev, w.free_ev, w.done_ev, w.counts_ev})
            if (e) (void)hipEventDestroy(e);
    }
    for (hipStream_t st : wb.streams)
        if (st) (void)hipStreamDestroy(st);
    wb = WfBuffers{};
}

/* The last recorded-size frames' overflow flags, if their copies have landed
 * (wait: block until they have).  Returns true when one of them overflowed;
 * the recorded sizes are then dropped, so the next frame reads its sizes back. */
bool wf_overflowed(WfBuffers &wb, bool wait) {
    bool any = false;
    for (WfSet &w : wb.set) {
        if (!w.flag_pending) continue;
        if (wait) {
            if (hipEventSynchronize(w.flag_ev) != hipSuccess) continue;
        } else if (hipEventQuery(w.flag_ev) != hipSuccess) {
            continue;
        }
        w.flag_pending = false;
        any = any || *w.h_flag != 0;
    }
    if (!any) return false;
    /* consumed: frames still in flight were queued with the same stale sizes
     * and are covered by this report; re-arm the device flags behind them */
    (void)hipDeviceSynchronize();
    for (WfSet &w : wb.set) {
        if (w.d_flag) (void)hipMemset(w.d_flag, 0, sizeof(int32_t));
        if (w.h_flag) *w.h_flag = 0;
        w.flag_pending = false;
    }
    wb.recs.clear();
    ++wb.epoch;
    wb.force_readback = true;   /* the next frame reads its sizes back (a device-sized frame may have overflowed) */
    wf_graphs_clear(wb);
    return true;
}

/* The sets' streams and events, created together (the runtime deals a
 * process's streams round robin over the device's hardware queues: streams
 * created back to back land on distinct queues, so the sets' levels can run
 * side by side — created at different times, two landed on one queue and ran
 * one after the other); free_ev recorded once on `stream`.  Called at scene
 * upload for scenes that take the wavefront path, so the first frame does
 * not pay for it. */
int wf_streams(WfBuffers &wb, hipStream_t stream) {
    if (wb.streams[0]) return CRT_OK;
    for (hipStream_t &st : wb.streams) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (WfSet &w : wb.set) {
        HIP_TRY(hipEventCreateWithFlags(&w.free_ev, CRT_PIPE_EV_FLAGS));
        HIP_TRY(hipEventCreateWithFlags(&w.done_ev, CRT_PIPE_EV_FLAGS));
        HIP_TRY(hipEventRecord(w.free_ev, stream));
    }
    return CRT_OK;
}

/* One frame of the wavefront path (see k_wf_level).  A level's size is
 * known only once the level before it has run, so the first frame of a
 * (settings, tile list) reads each level's queue length back before launching
 * the next level (one host sync per level) and records the sizes.  The sizes
 * are a function of the frame's rays alone, so every later frame with the same
 * key launches all levels back to back with the recorded sizes, no host sync:
 * each level may queue exactly the recorded size of the next, and a level
 * that would queue more sets an overflow flag instead (checked behind the
 * frame: crt_hip_render re-renders that frame with read-backs, the device-side
 * entry points report it on the next call).
 *
 * Recorded-size frames take up to kWfSets buffer sets in turn, set i's levels
 * and compose on stream i % kWfStreams (after the set's previous frame wrote
 * its pixels), the pixels on the caller's stream (after the set's levels):
 * consecutive frames' levels overlap — a level's few, long walks leave most
 * of the GPU idle — while the frame's only write the caller sees stays in
 * the caller's stream order.  More frames in flight kept paying: C3 back to
 * back 1.20 ms with 2 sets/2 streams, 1.07 with 4/4, 0.93 with 8/8, 0.89
 * with 12/12, 0.90 with 16/16; sets sharing streams were slower
 * (profiles/r04/ab_wf_sets.txt). */
/* Record the level sizes of device-sized frames whose copies have landed
 * (WfSet::counts_*): for their tile list and settings, unless a record was
 * dropped since the frame was issued (camera moved, plans freed, overflow)
 * or a level outgrew its queue. */
void wf_harvest(WfBuffers &wb) {
    for (WfSet &w : wb.set) {
        if (!w.counts_pending || hipEventQuery(w.counts_ev) != hipSuccess) continue;
        w.counts_pending = false;
        if (w.counts_epoch != wb.epoch || wb.recs.count(w.counts_tiles)) continue;
        if (w.h_counts[kWfDynMaxLevels] != 0) continue;   /* the frame overflowed: its counts are not its rays */
        std::vector<int32_t> sizes;
        bool ok = true;
        int64_t ids = 0;
        for (int L = 1; L < w.counts_levels; ++L) {
            const int32_t n = w.h_counts[L - 1];
            if (n == 0) break;
            ok = ok && n > 0 && n <= w.counts_qcap;
            ids += n;
            sizes.push_back(n);
        }
        if (!ok || ids > w.counts_idcap) continue;
        WfBuffers::Rec &r = wb.recs[w.counts_tiles];
        if (wb.shrink_records)
            for (int32_t &n : sizes) n = n > 1 ? n - 1 : n;
        r.sizes.swap(sizes);
        r.st = w.counts_st;
        r.ntiles = w.counts_ntiles;
    }
}

#ifdef CRT_WF_STAMPS
int wf_stamps_dump(const char *fn, int levels);
#endif
int render_wavefront(crt_hip_scene *sc, const DSettings &ds, const crt_renderer_settings *st, const ShardPlan &plan,
                     float *d_out, hipStream_t stream, bool count, const DeviceScene *d_scene, int sec, int primary) {
    WfBuffers &wb = sc->wf;
    /* levels 0..max_ray_depth are traced (a child deeper than max_ray_depth is
     * never queued, crt_renderer.cpp:47-48), so the loop below always drains
     * the queue: counts[max_ray_depth] is written by nobody and stays 0 */
    if (ds.max_ray_depth > (uint32_t)kWfMaxDepth)
        return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > " + std::to_string(kWfMaxDepth) +
                                                " with reflective/refractive materials is not supported");
    if (wf_overflowed(wb, false))
        return set_error(CRT_E_STATE, "a wavefront level outgrew its recorded size in the previous frame; "
                                         "that frame is wrong (sizes are now read back again)");
    const int64_t n0 = (int64_t)plan.ntiles * 64;
    wb.shrink_records = sc->wf_replay == 2;
    wf_harvest(wb);
    const auto rit = wb.recs.find((const void *)plan.d_tiles);
    const bool replay = !count && sc->wf_replay && sc->wf_record && rit != wb.recs.end() &&
                        rit->second.ntiles == plan.ntiles && std::memcmp(&rit->second.st, st, sizeof *st) == 0;
    /* no recorded sizes (a new camera, tile list or settings): device-sized
     * levels instead of read-backs — queues of 2 x n0 rays, wf_dyn_ids x n0
     * ray ids, each level's size read by its kernels from the counts the
     * levels before wrote; the same overflow flag as recorded-size frames.
     * Its level sizes are copied back behind it and recorded (wf_harvest)
     * if no record was dropped meanwhile, so the next frames replay. */
    const bool dyn_ok = sc->wf_replay && sc->wf_dynamic && ds.max_ray_depth + 2 <= (uint32_t)kWfDynMaxLevels;
    const bool dyn = !replay && !count && dyn_ok && !wb.force_readback;
    const bool async_frame = replay || dyn;
    const int64_t dyn_q = std::max<int64_t>(2 * n0, 4096), dyn_ids = std::max<int64_t>(1, sc->wf_dyn_ids) * n0;
    /* sets in use: as many as CRT_WF_SET_BUDGET holds of this frame size
     * (rays x (node + colour) + two queues), 2 <= sets <= kWfSets; each set
     * waits for its own previous frame, so the count may change between frames */
    {
        const int rc0 = wf_streams(wb, stream);
        if (rc0 != CRT_OK) return rc0;
    }
    int si = 0;
    if (async_frame) {
        int64_t tot = n0, mx = 1;
        if (replay) {
            for (int32_t n : rit->second.sizes) {
                tot += n;
                mx = std::max<int64_t>(mx, n);
            }
            if (dyn_ok) {
                tot = std::max(tot, dyn_ids);
                mx = std::max(mx, dyn_q);
            }
        } else {
            tot = dyn_ids;
            mx = dyn_q;
        }
        const int64_t set_bytes = tot * (int64_t)(sizeof(WNode) + sizeof(DVec4)) + 2 * mx * (int64_t)sizeof(WRay);
        const int64_t fit = CRT_WF_SET_BUDGET / std::max<int64_t>(set_bytes, 1);
        const int nsets = (int)std::min<int64_t>(kWfSets, std::max<int64_t>(1, fit));
        /* the first set whose last frame is done (a caller that waits for each
         * frame stays on set 0: one set's buffers and one graph); with every
         * set busy (frames back to back), the one issued longest ago */
        si = -1;
        for (int k = 0; k < nsets && si < 0; ++k)
            if (hipEventQuery(wb.set[k].free_ev) == hipSuccess) si = k;
        if (si < 0) {
            si = 0;
            for (int k = 1; k < nsets; ++k)
                if (wb.set[k].seq < wb.set[si].seq) si = k;
        }
        wb.set[si].seq = ++wb.frame;
    }
    WfSet &w = wb.set[si];
    /* where the levels run: a recorded-size frame on its set's stream, after
     * the set's previous frame; a frame with read-backs on the caller's */
    const hipStream_t ls = async_frame ? wb.streams[si % kWfStreams] : stream;
    HIP_TRY(hipStreamWaitEvent(ls, w.free_ev, 0));
    if (!d_scene) {   /* the scene record: written on ls if it changed, else waited for there */
        const int rc0 = sync_device_record(sc, &d_scene, ls);
        if (rc0 != CRT_OK) return rc0;
        if (async_frame) {   /* its readers: this set's levels (done_ev), not the caller's stream */
            w.rec_slots |= 1u << sc->ring_cur;
            sc->rec_read_by_set = true;
        }
    } else if (async_frame) {   /* the scene record this frame reads was written on another stream */
        const int rc0 = wait_device_record(sc, ls);
        if (rc0 != CRT_OK) return rc0;
    }
    const int kMaxLevels = (int)ds.max_ray_depth + 2;
    if (!w.counts || w.count_cap < kMaxLevels) {
        int rc0 = wf_set_release(wb, si);
        if (rc0 != CRT_OK) return rc0;
        if (w.counts) (void)hipFree(w.counts);
        w.counts = nullptr;
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)kMaxLevels * sizeof(int32_t)));
        w.counts = static_cast<int32_t *>(p);
        w.count_cap = kMaxLevels;
    }
    if (!w.d_flag) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, sizeof(int32_t)));
        w.d_flag = static_cast<int32_t *>(p);
        HIP_TRY(hipMemsetAsync(w.d_flag, 0, sizeof(int32_t), ls));
        HIP_TRY(hipHostMalloc(&p, sizeof(int32_t), hipHostMallocDefault));
        w.h_flag = static_cast<int32_t *>(p);
        *w.h_flag = 0;
        HIP_TRY(hipEventCreateWithFlags(&w.flag_ev, hipEventDisableTiming));
    }
    static const std::vector<int32_t> kNone;
    const std::vector<int32_t> &rec = replay ? rit->second.sizes : kNone;
    int rc;
    int64_t qneed = 2 * n0, ids = 3 * n0;
    if (replay) {
        int64_t tot = n0, mx = 0;
        for (int32_t n : rec) {
            tot += n;
            mx = std::max<int64_t>(mx, n);
        }
        qneed = std::max<int64_t>(mx, 1);
        ids = tot;
        if (dyn_ok) {   /* sized for device-sized frames too: a camera move then grows no set (a hipFree syncs the device) */
            qneed = std::max(qneed, dyn_q);
            ids = std::max(ids, dyn_ids);
        }
    } else if (dyn) {
        qneed = dyn_q;
        ids = dyn_ids;
    }
    if ((rc = wf_grow_ids(wb, si, ids, 0, ls)) != CRT_OK) return rc;
    if ((rc = wf_grow_queue(wb, si, 0, qneed)) != CRT_OK) return rc;
    if (async_frame && (rc = wf_grow_queue(wb, si, 1, qneed)) != CRT_OK) return rc;
    if (dyn && !w.h_counts) {
        void *p = nullptr;
        HIP_TRY(hipHostMalloc(&p, (kWfDynMaxLevels + 1) * sizeof(int32_t), hipHostMallocDefault));   /* + the overflow flag */
        w.h_counts = static_cast<int32_t *>(p);
        HIP_TRY(hipEventCreateWithFlags(&w.counts_ev, hipEventDisableTiming));
    }
    /* the pixels on the caller's stream once the levels are done; the set is
     * free again after them */
    auto finish = [&]() -> int {
        if (dyn) {   /* the level sizes, to record once they land (wf_harvest) */
            HIP_TRY(hipMemcpyAsync(w.h_counts, w.counts, (size_t)kMaxLevels * sizeof(int32_t), hipMemcpyDeviceToHost, ls));
            /* the set's overflow flag beside them, on the same stream: sizes of a
             * frame that overflowed (a queue or the ray ids) are not recorded */
            HIP_TRY(hipMemcpyAsync(w.h_counts + kWfDynMaxLevels, w.d_flag, sizeof(int32_t), hipMemcpyDeviceToHost, ls));
            HIP_TRY(hipEventRecord(w.counts_ev, ls));
            w.counts_pending = true;
            w.counts_tiles = (const void *)plan.d_tiles;
            w.counts_st = *st;
            w.counts_ntiles = plan.ntiles;
            w.counts_levels = kMaxLevels;
            w.counts_epoch = wb.epoch;
            w.counts_qcap = dyn_q;
            w.counts_idcap = (int64_t)w.cap - (int64_t)n0;   /* ray ids past the camera rays */
        }
        if (async_frame) {
            HIP_TRY(hipEventRecord(w.done_ev, ls));
            HIP_TRY(hipStreamWaitEvent(stream, w.done_ev, 0));
        }
        hipLaunchKernelGGL(k_wf_pixels, dim3((unsigned)((plan.ntiles + 3) / 4)), dim3(256), 0, stream, w.nodes, w.cols,
                           plan.d_tiles, plan.ntiles, d_out);
        HIP_TRY(hipGetLastError());
        if (async_frame)   /* the device flag is sticky: a later frame's copy cannot hide an earlier overflow */
            HIP_TRY(hipMemcpyAsync(w.h_flag, w.d_flag, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipEventRecord(w.free_ev, stream));
        if (async_frame) {
            HIP_TRY(hipEventRecord(w.flag_ev, stream));
            w.flag_pending = true;
        }
#ifdef CRT_WF_STAMPS
        if (const char *fn = std::getenv("CRT_WF_STAMPS_FILE")) {
            HIP_TRY(hipStreamSynchronize(stream));
            if (wf_stamps_dump(fn, kMaxLevels) != 0) return CRT_E_HIP;
        }
#endif
        return CRT_OK;
    };
    /* a recorded-size frame's levels are a fixed launch sequence: replayed
     * from a HIP graph captured the first time (one launch instead of ~2 per
     * level) */
    if (replay && sc->wf_graph) {
        for (const auto &g : wb.graphs)
            if (g.tiles == (const void *)plan.d_tiles && g.stream == ls && g.set == si && g.scene == (const void *)d_scene &&
                std::memcmp(&g.st, st, sizeof *st) == 0) {
                HIP_TRY(hipGraphLaunch(g.exec, ls));
                return finish();
            }
    }
    const bool capture = replay && sc->wf_graph;
    if (capture) HIP_TRY(hipStreamBeginCapture(ls, hipStreamCaptureModeRelaxed));
    auto cap_of = [](int64_t c) { return (int32_t)std::min<int64_t>(c, INT32_MAX); };
    std::vector<int32_t> sizes;
    auto enqueue = [&]() -> int {
    HIP_TRY(hipMemsetAsync(w.counts, 0, kMaxLevels * sizeof(int32_t), ls));
    unsigned long long *cnt = sc->d_counters;
    WLevel lv{nullptr, 0, 0, w.q[0], w.counts, (int32_t)n0, w.nodes, w.cols, 64,
              replay ? (rec.empty() ? 0 : rec[0]) : cap_of(w.qcap[0]), w.d_flag, nullptr, (int32_t)n0, cap_of(w.cap)};
    const int blocks0 = (plan.ntiles + 3) / 4;
#define CRT_WF0(T, COUNT)                                                                                   \
    hipLaunchKernelGGL((k_wf_level<T, true, COUNT>), dim3(blocks0), dim3(256), 0, ls, d_scene, ds,          \
                       plan.d_tiles, plan.ntiles, lv, cnt)
    if (primary == 14) {   /* level 0 on the BVH (camera bins there measured neutral, profiles/r03/ab_level0_bins) */
        if (count) CRT_WF0(14, true); else CRT_WF0(14, false);
    } else if (primary == 12 || primary == 13) {   /* level 0 keeps 8x8 tiles' packet walk (no window build) */
        if (count) CRT_WF0(12, true); else CRT_WF0(12, false);
    } else if (primary == 8) {
        if (count) CRT_WF0(8, true); else CRT_WF0(8, false);
    } else {
        if (count) CRT_WF0(7, true); else CRT_WF0(7, false);
    }
#undef CRT_WF0
    HIP_TRY(hipGetLastError());
    std::vector<std::pair<int64_t, int64_t>> levels;   /* (first id, count) of levels >= 1 */
    int64_t base = n0;
    int cur = 0;
    const int rpw = std::min(64, std::max(1, sc->wf_rays_per_wave));   /* coop walks: idle lanes take donated pieces */
    const int32_t dyn_cap = cap_of(std::min(w.qcap[0], w.qcap[1]));   /* device-sized levels: either queue holds this many */
    for (int L = 1; L < kMaxLevels; ++L) {
        int32_t n = 0;
        int32_t out_cap = 0;
        if (replay) {
            if (L - 1 >= (int)rec.size()) break;
            n = rec[L - 1];
            out_cap = L < (int)rec.size() ? rec[L] : 0;
        } else if (dyn) {   /* levels 1..max_ray_depth may hold rays (deeper children are never queued) */
            if (L > (int)ds.max_ray_depth) break;
            n = dyn_cap;
            out_cap = dyn_cap;
        } else {
            HIP_TRY(hipMemcpyAsync(&n, w.counts + (L - 1), sizeof n, hipMemcpyDeviceToHost, ls));
            HIP_TRY(hipStreamSynchronize(ls));
            if (n == 0) break;
            if (base + 3 * (int64_t)n > INT32_MAX) return set_error(CRT_E_UNSUPPORTED, "wavefront ray ids exceed 2^31");
            if ((rc = wf_grow_ids(wb, si, base + 3 * (int64_t)n, base, ls)) != CRT_OK) return rc;
            if ((rc = wf_grow_queue(wb, si, cur ^ 1, 2 * (int64_t)n)) != CRT_OK) return rc;
            out_cap = cap_of(w.qcap[cur ^ 1]);
            sizes.push_back(n);
        }
        /* rays per wave of this level: fewer (more helper lanes per ray) when
         * the level has fewer rays than ~4096 waves' worth, at least 8, at most
         * the wf_rpw cap — a level's time is its slowest waves'
         * (C3 3.60 -> 3.33 ms, profiles/r02/ab_c3_rpw) */
        const int rpw_l = sec == 14 ? 64 : std::min(rpw, std::max(8, (int)((n + 4095) / 4096)));
        WLevel l{w.q[cur], n, L, w.q[cur ^ 1], w.counts + L, (int32_t)(base + n), w.nodes, w.cols, rpw_l, out_cap,
                 w.d_flag, dyn ? w.counts : nullptr, (int32_t)n0, cap_of(w.cap)};
        /* device-sized: a fixed grid whose waves stride over the level */
        const int64_t waves = dyn ? std::min<int64_t>(((int64_t)n + rpw_l - 1) / rpw_l, std::max(64, sc->wf_dyn_waves))
                                  : ((int64_t)n + rpw_l - 1) / rpw_l;
        const int blocks = dyn ? (int)(((waves + 3) / 4 + 7) & ~7ll)   /* (device-sized: a multiple of the 8 XCDs) */
                               : (int)((waves + 3) / 4);
#define CRT_WF(SEC, COUNT)                                                                                  \
    hipLaunchKernelGGL((k_wf_level<SEC, false, COUNT>), dim3(blocks), dim3(256), 0, ls, d_scene, ds,         \
                       plan.d_tiles, plan.ntiles, l, cnt)
        if (sec == 14) {
            if (count) CRT_WF(14, true); else CRT_WF(14, false);
        } else if (sec == 10) {
            if (count) CRT_WF(10, true); else CRT_WF(10, false);
        } else {
            if (count) CRT_WF(4, true); else CRT_WF(4, false);
        }
#undef CRT_WF
        HIP_TRY(hipGetLastError());
        levels.emplace_back(dyn ? L : base, n);
        base += n;
        cur ^= 1;
    }
    for (auto it = levels.rbegin(); it != levels.rend(); ++it) {
        if (dyn)   /* (first = the level) */
            hipLaunchKernelGGL(k_wf_compose_dyn, dim3(1024), dim3(256), 0, ls, w.nodes, w.cols, w.counts,
                               (int32_t)it->first, (int32_t)n0, dyn_cap, cap_of(w.cap));
        else
            hipLaunchKernelGGL(k_wf_compose, dim3((unsigned)((it->second + 255) / 256)), dim3(256), 0, ls, w.nodes,
                               w.cols, (int32_t)it->first, (int32_t)it->second);
    }
    HIP_TRY(hipGetLastError());
    return CRT_OK;
    };
    rc = enqueue();
    if (capture) {
        hipGraph_t graph = nullptr;
        const hipError_t e = hipStreamEndCapture(ls, &graph);
        if (rc != CRT_OK) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        hipGraphExec_t exec = nullptr;
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_error(CRT_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
        wb.graphs.push_back(WfBuffers::Graph{(const void *)plan.d_tiles, *st, nullptr, ls, si, (const void *)d_scene, exec});
        HIP_TRY(hipGraphLaunch(exec, ls));
    } else if (rc != CRT_OK) {
        return rc;
    }
    if ((rc = finish()) != CRT_OK) return rc;
    if (!replay && !dyn && !count && sc->wf_replay) {
        wb.force_readback = false;
        WfBuffers::Rec &r = wb.recs[(const void *)plan.d_tiles];
        if (wb.shrink_records)
            for (int32_t &n : sizes) n = n > 1 ? n - 1 : n;
        r.sizes.swap(sizes);
        r.st = *st;
        r.ntiles = plan.ntiles;
    }
    return CRT_OK;
}

/* Pick and launch the kernel variant for this scene + settings. */
int launch_render(crt_hip_scene *sc, const crt_renderer_settings *st, const ShardPlan &plan, float *d_out,
                  hipStream_t stream, bool count, unsigned long long *stamps) {
    const bool gi = sc->info.gi_on && sc->has_diffuse && st->diffuse_reflection_ray_count > 0;
    const bool full = gi || sc->has_secondary;
    if (gi) {
        const int rc = ensure_gi_tables(sc);
        if (rc != CRT_OK) return rc;
    }
    if (sc->has_refractive && sc->info.refractions_on) {
        const int rc = ensure_pow5_table(sc);
        if (rc != CRT_OK) return rc;
    }
    if (sc->shadows) {
        const int rc = ensure_light_bins(sc, st);
        if (rc != CRT_OK) return rc;
    }
    if (plan.ntiles == 0) return CRT_OK;
    const DeviceScene *d_scene = nullptr;
    /* (a changed record written on the binning's stream instead, before the
     * event the render waits for, measured slower for orbit frames: the
     * ring's lazy slot-reuse event then orders the binning after the
     * previous render — 0.0675 -> 0.0736 ms) */
    const bool bins_frame = !full && bins_active(sc) && plan.bp.cell_tile;   /* (the branch below) */
    /* a wavefront frame writes a changed record on the stream its levels run
     * on (render_wavefront): on the caller's stream it would wait for the
     * previous frame's pixels, and frames with a new camera each could not
     * run side by side */
    const bool wf_frame = !sc->shadows && full && !gi && sc->wavefront && !stamps && !rec_machine_on(sc, st);
    if (!wf_frame) {
        const int rc = sync_device_record(sc, &d_scene, stream);
        if (rc != CRT_OK) return rc;
    }
    DSettings ds = to_dsettings(st);
    const bool sh_defer = sc->shadows && sc->shadow_defer && !full && !count && !stamps;
    /* Walks: camera rays take the packet walk (traversal 7, or 8 pruned).
     * Secondary rays scatter and take the cooperative walk: pruned (10) for
     * reflect/refract levels (C3), reference order (4) for GI fan-out — the
     * pruned form needs 134 VGPRs (3 waves/SIMD) and loses on C4 (378 vs 320
     * ms); with GI every ray of the per-lane frame-stack kernel takes that walk
     * (the packet walk's registers would cost a wave per SIMD).
     * CRT_SECONDARY / "secondary" overrides the secondary walk. */
    const bool pruned = sc->traversal != 7;
    int sec = sc->secondary;
    if (sec == 14 && !sc->ds.bnodes) sec = 10;   /* no BVH (device-built tree) */
    if (sec == 0) sec = !pruned ? 4 : sc->ds.bnodes ? 14 : gi ? 4 : 10;
    if (sc->shadows && !bins_frame) {
        /* shadow-ray frames (option "shadows"): frame-stack kernel, pruned
         * cooperative walk for every traced ray, per-lane shadow walks (any
         * hit through the BVH where the scene has one, crt_bvh.h occluded_bvh) */
        if (stamps) return set_error(CRT_E_UNSUPPORTED, "wave profiles of shadow-ray frames are not supported");
        const uint64_t nf = (uint64_t)st->max_ray_depth + 1;
        const int nb = (plan.ntiles + 3) / 4;
        unsigned long long *cn = sc->d_counters;
        if (!full) {   /* no recursion: the frame's camera walk, packet walks for shadow rays (shade_hit_shadowed) */
            int tr = camera_walk(sc, sc->traversal);
            if (tr == 13 && !plan.has_small) tr = 12;
            if (sh_defer) {
                const int rc = shadow_defer_begin(sc, ds, stream);
                if (rc != CRT_OK) return rc;
            }
#define CRT_LAUNCH_SH(TR, COUNT)                                                                            \
    hipLaunchKernelGGL((k_render_tiles<false, 0, TR, TR, COUNT, true>), dim3(nb), dim3(256), 0, stream, d_scene, ds, \
                       plan.d_tiles, plan.ntiles, d_out, cn, nullptr, BinsPlan{})
            if (tr == 14) {
                if (count) CRT_LAUNCH_SH(14, true); else CRT_LAUNCH_SH(14, false);
            } else if (tr == 13) {
                if (count) CRT_LAUNCH_SH(13, true); else CRT_LAUNCH_SH(13, false);
            } else if (tr == 12) {
                if (count) CRT_LAUNCH_SH(12, true); else CRT_LAUNCH_SH(12, false);
            } else {
                if (count) CRT_LAUNCH_SH(8, true); else CRT_LAUNCH_SH(8, false);
            }
#undef CRT_LAUNCH_SH
            HIP_TRY(hipGetLastError());
            return shadow_defer_end(sc, d_scene, ds, d_out, stream);
        }
#define CRT_LAUNCH_S(MAXF, COUNT)                                                                           \
    hipLaunchKernelGGL((k_render_tiles<true, MAXF, 10, 10, COUNT, true>), dim3(nb), dim3(256), 0, stream,      \
                       d_scene, ds, plan.d_tiles, plan.ntiles, d_out, cn, nullptr, BinsPlan{})
        if (nf <= 4) {
            if (count) CRT_LAUNCH_S(4, true); else CRT_LAUNCH_S(4, false);
        } else if (nf <= 16) {
            if (count) CRT_LAUNCH_S(16, true); else CRT_LAUNCH_S(16, false);
        } else if (nf <= 64) {
            if (count) CRT_LAUNCH_S(64, true); else CRT_LAUNCH_S(64, false);
        } else {
            return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > 63 with shadow rays is not supported");
        }
#undef CRT_LAUNCH_S
        HIP_TRY(hipGetLastError());
        return CRT_OK;
    }
    /* recursion without GI (C3): the per-lane state machine (rec_machine), or level by level (wavefront) */
    const bool rec_machine = full && !gi && rec_machine_on(sc, st) && !stamps;
    if (wf_frame)
        return render_wavefront(sc, ds, st, plan, d_out, stream, count, d_scene,
                                sec, camera_walk(sc, sc->traversal));
    /* frame-stack kernel: one walk for every ray */
    int trav = full ? sec : camera_walk(sc, sc->traversal);
    if (trav == 13 && !plan.has_small) trav = 12;   /* no split tiles: the leaner packet-only kernel */
    const int blocks = (plan.ntiles + 3) / 4;
    const uint64_t frames = (uint64_t)st->max_ray_depth + 1;
    unsigned long long *cnt = sc->d_counters;
#define CRT_LAUNCH_T(FULL, MAXF, TRAV, COUNT)                                                               \
    hipLaunchKernelGGL((k_render_tiles<FULL, MAXF, TRAV, TRAV, COUNT>), dim3(blocks), dim3(256), 0, stream,      \
                       d_scene, ds, plan.d_tiles, plan.ntiles, d_out, cnt, stamps, BinsPlan{})
#define CRT_LAUNCH(MAXF, COUNT)                                                                             \
    do {                                                                                                   \
        if (trav == 10 || trav == 14) CRT_LAUNCH_T(true, MAXF, 10, COUNT);                                  \
        else CRT_LAUNCH_T(true, MAXF, 4, COUNT);                                                           \
    } while (0)
    if (bins_frame) {
        /* this frame's camera bins (and its record), then the render over the
         * bins plan's grid */
        int par = 0;
        const int rc = bins_enqueue(sc, plan, stream, &par);
        if (rc != CRT_OK) return rc;
        BinsPlan bp = plan.bp;
        bp.par = par;
        bp.work += (size_t)par * bp.wslots;   /* this frame's set of the work lists */
#ifdef CRT_BINS_TRACE   /* diagnostic builds: the binning's decisions on stderr */
        std::fprintf(stderr, "launch bins plan=%p ntiles=%d waves=%d par=%d out=%p stream=%p\n", (const void *)&plan,
                     plan.ntiles, plan.waves, par, (void *)d_out, (void *)stream);
#endif
        const unsigned bb = (unsigned)((plan.waves + 3) / 4);
#define CRT_LAUNCH_B(COUNT, SH)                                                                             \
    hipLaunchKernelGGL((k_render_tiles<false, 0, 15, 15, COUNT, SH>), dim3(bb), dim3(256), 0, stream, d_scene, ds, \
                       plan.d_tiles, plan.waves, d_out, cnt, stamps, bp)
        if (sc->shadows) {   /* the course's earlier renderer: shadow rays (crt_shade.h shade_hit_shadowed) */
            if (sh_defer) {
                const int rc = shadow_defer_begin(sc, ds, stream);
                if (rc != CRT_OK) return rc;
            }
            if (count) CRT_LAUNCH_B(true, true); else CRT_LAUNCH_B(false, true);
            HIP_TRY(hipGetLastError());
            const int rc = shadow_defer_end(sc, d_scene, ds, d_out, stream);
            if (rc != CRT_OK) return rc;
        } else {
            if (count) CRT_LAUNCH_B(true, false); else CRT_LAUNCH_B(false, false);
        }
#undef CRT_LAUNCH_B
        HIP_TRY(hipGetLastError());
        /* this set's lists are free again — after every render that read
         * them: a set taken again (bins_reuse) by a frame on another stream
         * chains the earlier reader's event into this one */
        BinsDev &b = sc->bins;
        if (b.rdone_s[par] != stream && hipEventQuery(b.rdone[par]) != hipSuccess)
            HIP_TRY(hipStreamWaitEvent(stream, b.rdone[par], 0));
        HIP_TRY(hipEventRecord(b.rdone[par], stream));
        b.rdone_s[par] = stream;
    } else if (!full) {
        switch (trav) {
        case 7: if (count) CRT_LAUNCH_T(false, 0, 7, true); else CRT_LAUNCH_T(false, 0, 7, false); break;
        case 8: if (count) CRT_LAUNCH_T(false, 0, 8, true); else CRT_LAUNCH_T(false, 0, 8, false); break;
        case 12: if (count) CRT_LAUNCH_T(false, 0, 12, true); else CRT_LAUNCH_T(false, 0, 12, false); break;
        case 13: if (count) CRT_LAUNCH_T(false, 0, 13, true); else CRT_LAUNCH_T(false, 0, 13, false); break;
        case 14: if (count) CRT_LAUNCH_T(false, 0, 14, true); else CRT_LAUNCH_T(false, 0, 14, false); break;
        default: return set_error(CRT_E_INVALID, "no such camera walk");
        }
    } else if (rec_machine || (gi && (trav == 4 || trav == 10 || trav == 14) && sc->gi_refill && sc->d_next_px && !stamps &&
                               frames <= 64)) {
        /* GI: persistent waves with pixel refill (k_render_refill) */
        HIP_TRY(hipMemsetAsync(sc->d_next_px, 0, sizeof(int32_t), stream));
        const int nw = std::max(1, std::min(plan.ntiles, sc->refill_waves));
        const unsigned rb = (unsigned)((nw + 3) / 4);
#define CRT_REFILL_T(MAXF, T, COUNT)                                                                        \
    hipLaunchKernelGGL((k_render_refill<MAXF, T, COUNT>), dim3(rb), dim3(256), 0, stream, d_scene, ds,       \
                       plan.d_tiles, plan.ntiles, d_out, sc->d_next_px, cnt)
#define CRT_REFILL(MAXF, COUNT) CRT_REFILL_T(MAXF, 4, COUNT)
        if (rec_machine || (trav == 14 && sc->gi_machine && (uint64_t)st->diffuse_reflection_ray_count < (1ull << 29) &&
                            (int64_t)sc->info.width * sc->info.height < INT32_MAX)) {
            /* per-lane state machine over the BVH walk (crt_gi_machine.h) */
            const unsigned gb = (unsigned)std::max(1, std::min((plan.ntiles + 3) / 4, sc->gi_blocks));
            /* frames below the two LDS ones and the register one: 64 B per lane and depth */
            const int64_t gneed = (int64_t)gb * 256 * std::max<int64_t>(0, (int64_t)st->max_ray_depth - 3) * 64;
            if (gneed > sc->gi_frames_bytes) {
                HIP_TRY(hipStreamSynchronize(stream));
                if (sc->gi_frames) (void)hipFree(sc->gi_frames);
                sc->gi_frames = nullptr;
                sc->gi_frames_bytes = 0;
                HIP_TRY(hipMalloc(&sc->gi_frames, (size_t)gneed));
                sc->gi_frames_bytes = gneed;
            }
            float4 *gf = static_cast<float4 *>(sc->gi_frames);
            if (count)
                hipLaunchKernelGGL((k_render_gi<true>), dim3(gb), dim3(256), 0, stream, d_scene, ds, plan.d_tiles,
                                   plan.ntiles, d_out, sc->d_next_px, cnt, gf);
            else
                hipLaunchKernelGGL((k_render_gi<false>), dim3(gb), dim3(256), 0, stream, d_scene, ds, plan.d_tiles,
                                   plan.ntiles, d_out, sc->d_next_px, cnt, gf);
        } else if (frames <= 4 && trav == 10) {   /* pruned cooperative walk for GI (secondary = 10) */
            if (count) CRT_REFILL_T(4, 10, true); else CRT_REFILL_T(4, 10, false);
        } else if (frames <= 4) {
            if (count) CRT_REFILL(4, true); else CRT_REFILL(4, false);
        } else if (frames <= 16) {
            if (count) CRT_REFILL(16, true); else CRT_REFILL(16, false);
        } else {
            if (count) CRT_REFILL(64, true); else CRT_REFILL(64, false);
        }
#undef CRT_REFILL
#undef CRT_REFILL_T
    } else if (frames <= 4) {
        if (count) CRT_LAUNCH(4, true); else CRT_LAUNCH(4, false);
    } else if (frames <= 16) {
        if (count) CRT_LAUNCH(16, true); else CRT_LAUNCH(16, false);
    } else if (frames <= 64) {
        if (count) CRT_LAUNCH(64, true); else CRT_LAUNCH(64, false);
    } else {
        return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > 63 with recursive materials is not supported");
    }
#undef CRT_LAUNCH
#undef CRT_LAUNCH_T
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

int render_into(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, hipStream_t stream, bool count) {
    if (sc->grid_empty) {
        /* bucket grid rounds to zero buckets: the reference renders nothing and
         * returns the zero-initialised image (crt_renderer.cpp:158-174) */
        HIP_TRY(hipMemsetAsync(d_rgb, 0, (size_t)sc->info.width * sc->info.height * 3 * sizeof(float), stream));
        return CRT_OK;
    }
    int rc = ensure_plans(sc, st, stream, true);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_start, stream));
    rc = launch_render(sc, st, sc->full, d_rgb, stream, count);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_stop, stream));
    sc->events_valid = sc->record_events != 0;
    return used_device_record(sc, stream);
}

}  // namespace crt_amd


namespace crt_amd {

/* The frame's live-pixel mask (k_live_pixels), computed once per scene. */
int ensure_live_mask(crt_hip_scene *sc) {
    if (!sc->live_mask.empty() || sc->grid_empty) return CRT_OK;
    const DeviceScene *d_scene = nullptr;
    int rc = sync_device_record(sc, &d_scene, sc->stream);
    if (rc != CRT_OK) return rc;
    const int64_t npx = (int64_t)sc->info.width * sc->info.height;
    uint8_t *d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)npx));
    hipLaunchKernelGGL(k_live_pixels, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, sc->stream, d_scene, d);
    hipError_t e = hipGetLastError();
    std::vector<uint8_t> m((size_t)npx);
    if (e == hipSuccess) e = hipMemcpyAsync(m.data(), d, (size_t)npx, hipMemcpyDeviceToHost, sc->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("live mask: ") + hipGetErrorString(e));
    sc->live_mask.swap(m);
    return CRT_OK;
}

std::vector<DBucket> compact_tiles(crt_hip_scene *sc, int shard, int shard_count, int64_t *px,
                                   std::vector<DBucket> *dead) {
    return shard_live_tiles(sc->info.width, sc->info.height, sc->info.bucket_size, shard, shard_count,
                            sc->live_mask.empty() ? nullptr : sc->live_mask.data(), px, dead);
}

int render_shard_t(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count, float *d_packed,
                   void *stream, bool compact) {
    if (!sc || !d_packed) return set_error(CRT_E_INVALID, "null argument");
    if (shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    if ((rc = ensure_plans(sc, st, s)) != CRT_OK) return rc;
    if (compact && (rc = ensure_live_mask(sc)) != CRT_OK) return rc;
    auto &plans = compact ? sc->compact_plans : sc->shard_plans;
    auto key = std::make_pair(shard, shard_count);
    auto it = plans.find(key);
    if (it == plans.end()) {
        int64_t px = 0;
        const std::vector<DBucket> b = compact ? compact_tiles(sc, shard, shard_count, &px)
                                               : shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size,
                                                               shard, shard_count, &px);
        ShardPlan plan;
        if ((rc = make_tile_plan(sc, b, false, plan)) != CRT_OK) return rc;
        it = plans.emplace(key, plan).first;
    }
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_start, s));
    rc = launch_render(sc, st, it->second, d_packed, s, false);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_stop, s));
    sc->events_valid = sc->record_events != 0;
    return used_device_record(sc, s);
}

/* write_ppm's conversion of one component on the host (k_quantize). */
uint8_t quantize_host(float c) {
    const float x = c * 255.0f;
    int v = (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : (int)0x80000000;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

template <class T>
int unpack_shards_t(crt_hip_scene *sc, int shard_count, const T *d_gathered, T *d_rgb, void *stream, bool compact) {
    if (!sc || !d_gathered || !d_rgb || shard_count <= 0) return set_error(CRT_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(sc->device));
    if (compact) {
        const int rc = ensure_live_mask(sc);
        if (rc != CRT_OK) return rc;
    }
    auto &plans = compact ? sc->compact_unpack : sc->unpack_plans;
    auto it = plans.find(shard_count);
    if (it == plans.end()) {
        const int64_t stride = compact ? crt_hip_compact_stride(sc, shard_count) : crt_hip_shard_stride(sc, shard_count);
        if (stride < 0) return (int)stride;
        std::vector<UnpackBucket> ub;
        std::vector<DBucket> dead;
        for (int s = 0; s < shard_count; ++s) {
            int64_t px = 0;
            const std::vector<DBucket> b = compact ? compact_tiles(sc, s, shard_count, &px, &dead)
                                                   : shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size,
                                                                   s, shard_count, &px);
            for (const DBucket &x : b) ub.push_back(UnpackBucket{x.x, x.y, x.w, x.h, s * stride + 3 * x.packed_offset, 0});
        }
        for (const DBucket &x : dead) ub.push_back(UnpackBucket{x.x, x.y, x.w, x.h, -1, 0});
        UnpackBucket *d = nullptr;
        if (!ub.empty()) {
            HIP_TRY(hipMalloc(&d, ub.size() * sizeof(UnpackBucket)));
            HIP_TRY(hipMemcpy(d, ub.data(), ub.size() * sizeof(UnpackBucket), hipMemcpyHostToDevice));
        }
        it = plans.emplace(shard_count, std::make_pair(d, (int)ub.size())).first;
    }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    if (sc->grid_empty)
        HIP_TRY(hipMemsetAsync(d_rgb, 0, (size_t)sc->info.width * sc->info.height * 3 * sizeof(T), s));
    if (it->second.second > 0) {
        Rgb<T> bg;
        for (int k = 0; k < 3; ++k) {
            if constexpr (sizeof(T) == 1) bg.c[k] = quantize_host(sc->ds.background[k]);
            else bg.c[k] = sc->ds.background[k];
        }
        hipLaunchKernelGGL(k_unpack<T>, dim3(it->second.second), dim3(256), 0, s, it->second.first, d_gathered, d_rgb,
                           sc->info.width, bg);
        HIP_TRY(hipGetLastError());
    }
    return CRT_OK;
}

template int unpack_shards_t<float>(crt_hip_scene *, int, const float *, float *, void *, bool);
template int unpack_shards_t<uint8_t>(crt_hip_scene *, int, const uint8_t *, uint8_t *, void *, bool);

}  // namespace crt_amd

