/*
 * crt_render.hip — the camera-ray kernels: one wave per tile of the frame's
 * measured plan, the primary ray generated in-kernel (Camera::generate_ray,
 * crt_camera.cpp:7-35), the walk (crt_walks.h) and the shading (crt_shade.h)
 * in the same launch; replaces render_region + shade_ray
 * (crt_renderer.cpp:46-155) for frames without GI.  Also the calibration
 * probe of the tile plans.
 */
#define CRT_KERNEL_TU 1
#include "crt_kernels.h"
#include "crt_shade.h"

namespace crt_amd {

/* The tile a wave of a camera-bins grid renders (crt_kernel_common.h
 * BinsPlan): a quarter of a heavy cell, a medium, light or bvh cell of this
 * frame's work lists (with the cell's list: off, len), or a rest tile (len
 * -2: the wave reads its cell's list).  The list's count and the entry are
 * loaded together.  Returns 0: nothing to do (an unused list slot), 1: the
 * tile, 2: a fill wave (off: its index).  *next: the slot's further entries
 * (a frame whose camera lists more cells of the kind than the grid has
 * slots: the entries gcap apart; next->n = 0 for none). */
struct BinsNext {
    const BinsWork *work;   /* the slot's list */
    int i, n, step, q;      /* this entry, the list's length, entries between the slot's, quarter (-1: whole) */
};

__device__ __forceinline__ void bins_quarter(Tile &tl, int q, int quad) {
    const int xx = (q & 1) * 4, yy = (q >> 1) * 4;
    tl.x += xx;
    tl.y += yy;
    tl.w = max(0, min(4, tl.w - xx));
    tl.h = max(0, min(4, tl.h - yy));
    tl.out_base += (int64_t)yy * tl.out_stride + xx;
    tl.prio = quad ? 3 : 1;
}

__device__ __forceinline__ int bins_tile(const BinsPlan &bp, const Tile *__restrict__ tiles, int wave, Tile &tl,
                                         int &off, int &len, BinsNext &next) {
    /* no further entry unless a list slot below sets them (a rest tile's
     * continuation must end the kernel's loop: i + step >= n) */
    next.work = nullptr;
    next.i = 0;
    next.n = 0;
    next.step = 1;
    next.q = -1;
    int kind = 0, slot = wave >> 2, q = wave & 3;
    if (wave >= 4 * kBinShards * bp.gcap[0]) {
        slot = wave - 4 * kBinShards * bp.gcap[0];
        q = -1;
        kind = 1;
        while (kind < kBinKinds && slot >= kBinShards * bp.gcap[kind]) {
            slot -= kBinShards * bp.gcap[kind];
            ++kind;
        }
        if (kind == kBinKinds) {
            if (slot >= bp.nrest) {
                off = slot - bp.nrest;
                return 2;
            }
            tl = tiles[load_scalar(bp.rest, slot)];
            len = -2;
            return 1;
        }
    }
    const int sh = slot % kBinShards, i = slot / kBinShards;
    const int n = min(load_scalar(bp.phdr, bins_phdr_at(bp.par, kind, sh)), bp.ecap);
    const BinsWork *work = bp.work + bp.wbase[kind] + sh * bp.ecap;
    const BinsWork w = work[i];
    if (i >= n) return 0;
    next.work = work;
    next.i = i;
    next.n = n;
    next.step = bp.gcap[kind];
    next.q = q;
    tl = w.t;
    off = w.off;
    len = w.len;
    if (q >= 0) bins_quarter(tl, q, bp.quad);   /* (a quarter outside a partial cell: w or h 0, no pixel) */
    return 1;
}

/* A fill wave of the camera-bins grid: of its 16 cells, the ones the plan
 * renders as one tile whose list is empty get the background (every camera
 * ray of the cell misses: no triangle's hull projects there).  A full 8x8
 * tile on 16-B aligned rows is written as 48 float4, else pixel by pixel.
 * Work-count frames count these rays as traversals (the reference traces
 * them; they test nothing). */
__device__ void bins_fill(const DeviceScene &s, const BinsPlan &bp, const Tile *__restrict__ tiles, int fw,
                          float *__restrict__ out, unsigned long long *__restrict__ counters) {
    const int lane = (int)__lane_id();
    const int c = fw * 16 + (lane & 15);
    bool e = false;
    int k = -1;
    if (lane < 16 && c < bp.ncell) {   /* the cell's tile and list length (this frame's set) in one round of loads */
        k = bp.cell_tile[c];
        e = s.bin_len[(size_t)bp.par * bp.ncell + c] == 0 && k >= 0;
    }
    Tile t{};
    if (e) t = tiles[k];
    const float bg[3] = {s.background[0], s.background[1], s.background[2]};
    uint64_t todo = __ballot(e);
    while (todo) {
        const int j = __builtin_ctzll(todo);
        todo &= todo - 1;
        const int w = __shfl(t.w, j), h = __shfl(t.h, j), stride = __shfl(t.out_stride, j);
        const int64_t base = ((int64_t)(uint32_t)__shfl((int)(uint32_t)t.out_base, j)) |
                             ((int64_t)__shfl((int)(t.out_base >> 32), j) << 32);
        if (w == 8 && h == 8 && (base & 3) == 0 && (stride & 3) == 0) {
            if (lane < 48) {   /* row lane / 6, float4 lane % 6 of its 24 floats */
                const int row = lane / 6, q4 = lane % 6;
                float4 v;
                v.x = bg[(4 * q4) % 3];
                v.y = bg[(4 * q4 + 1) % 3];
                v.z = bg[(4 * q4 + 2) % 3];
                v.w = bg[(4 * q4 + 3) % 3];
                *reinterpret_cast<float4 *>(out + 3 * (base + (int64_t)row * stride) + 4 * q4) = v;
            }
        } else {
            const int x = lane & 7, y = lane >> 3;
            if (x < w && y < h) {
                float *o = out + 3 * (base + (int64_t)y * stride + x);
                o[0] = bg[0];
                o[1] = bg[1];
                o[2] = bg[2];
            }
        }
        if (counters && lane == 0) atomicAdd(&counters[0], (unsigned long long)(w * h));
    }
}

/* One tile of a render grid (k_render_tiles): camera bins cell (len >= 0:
 * the cell's list from its work-list entry; -2: read it here; -1: the BVH
 * walk), a split tile's window walk, or the frame-stack walk of an 8x8 tile. */
template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW>
__device__ __forceinline__ void render_tile(const DeviceScene &s, const DSettings &st, Tile tl, int bin_beg,
                                            int bin_len, float *__restrict__ out,
                                            unsigned long long *__restrict__ counters,
                                            unsigned long long *__restrict__ stamps, int bpar, int bncell,
                                            int wave, int lane) {
    /* the heaviest tiles set the frame length (their walks are long chains of
     * dependent loads): they get issue priority over the light waves that
     * share their SIMD (s_setprio; scheduling only, results unchanged) */
    if (tl.prio & 1) __builtin_amdgcn_s_setprio(3);
    if constexpr (TRAV == 13 && !FULL) {
        /* tiles of <= 16 rays (the measured plan's splits of heavy tiles): window walk */
        const int tw = uniform_i(tl.w), th = uniform_i(tl.h);
        const int npx = tw * th;
        if (npx <= 16) {
            const int R = npx <= 4 ? 4 : 16;
            const int r = lane & (R - 1), sl = lane / R;
            const bool act = r < npx;
            const int px = act ? r % tw : 0, py = act ? r / tw : 0;
            Vec o, d;
            camera_ray(s.cam, tl.x + px, tl.y + py, o, d);
            LaneCounts cw = {};
            float t;
            const int slot = R == 4 ? trace_window<COUNT, 4>(s, r, sl, act, o, d, t, cw)
                                    : trace_window<COUNT, 16>(s, r, sl, act, o, d, t, cw);
            Vec c;
            if constexpr (SHADOW)   /* wave-wide */
                c = shade_hit_shadowed<COUNT>(s, st, act && sl == 0, o, d, slot, t, cw,
                                              tl.out_base + (int64_t)py * tl.out_stride + px);
            if (act && sl == 0) {
                if constexpr (!SHADOW) c = shade_primary(s, st, o, d, slot, t);   /* (SHADOW: wave-wide above) */
                float *pxo = out + 3 * (tl.out_base + (int64_t)py * tl.out_stride + px);
                pxo[0] = c.x;
                pxo[1] = c.y;
                pxo[2] = c.z;
            }
            if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
            if (COUNT) {
                atomicAdd(&counters[0], (unsigned long long)cw.traversals);
                atomicAdd(&counters[1], (unsigned long long)cw.nodes);
                atomicAdd(&counters[2], (unsigned long long)cw.tris);
                atomicAdd(&counters[3], (unsigned long long)cw.hits);
                if (lane == 0) {
                    atomicAdd(&counters[4], (unsigned long long)cw.wave_nodes);
                    atomicAdd(&counters[5], (unsigned long long)cw.wave_tris);
                    atomicAdd(&counters[6], (unsigned long long)cw.wave_edges);
                    atomicAdd(&counters[7], 1ull);
                    atomicAdd(&counters[8], (unsigned long long)cw.wave_box);
                    atomicAdd(&counters[9], (unsigned long long)cw.wave_pass);
                    atomicAdd(&counters[10], 1ull);   /* window-walk waves */
                    atomicAdd(&counters[11], (unsigned long long)cw.win_steps);
                    atomicAdd(&counters[14], (unsigned long long)cw.win_rounds);
                }
                atomicAdd(&counters[12], (unsigned long long)cw.win_slots);
                atomicAdd(&counters[13], (unsigned long long)cw.win_reached);
            }
            return;
        }
    }
    if constexpr (TRAV == 15 && !FULL) {
        /* a tile inside one 8x8 camera-bins cell: the cell's candidate list */
        const int tx0 = uniform_i(tl.x), ty0 = uniform_i(tl.y), tw = uniform_i(tl.w), th = uniform_i(tl.h);
        const int cell = (ty0 >> 3) * s.bin_tx + (tx0 >> 3);
        const bool one = (tx0 & 7) + tw <= 8 && (ty0 & 7) + th <= 8;
        const int pc = bpar * bncell + cell;   /* this frame's set of the per-cell lists */
        const int len = uniform_i(bin_len != -2 ? bin_len : one ? load_scalar(s.bin_len, pc) : -1);
        if (len >= 0) {   /* -1: not inside one cell, or the cell's list is over the cap: the BVH walk below */
            const int beg = uniform_i(bin_len != -2 ? bin_beg : load_scalar(s.bin_off, pc)), end = beg + len;
            __shared__ CamCand stage[4 * kBinChunk];
            if ((tl.prio & 2) && tw <= 4 && th <= 4) {
                /* a split tile of a long list: four lanes per pixel (trace_bins_lanes) */
                const int p = lane >> 2, sl = lane & 3, lx = p & 3, ly = p >> 2;
                const bool act = lx < tw && ly < th;
                Vec o, d;
                camera_ray(s.cam, tx0 + (act ? lx : 0), ty0 + (act ? ly : 0), o, d);
                LaneCounts cw = {};
                float t;
                const int bit = 8 * ((ty0 & 7) + ly) + (tx0 & 7) + lx;
                CamCand *stw = stage + (threadIdx.x >> 6) * kBinChunk;
                const int slot = trace_bins_lanes<COUNT, 4>(s, stw, beg, end, bit, sl, act, o, d, t, cw);
                Vec c;
                if constexpr (SHADOW)   /* wave-wide */
                    c = shade_hit_shadowed<COUNT>(s, st, act && sl == 0, o, d, slot, t, cw,
                                                  tl.out_base + (int64_t)ly * tl.out_stride + lx);
                if (act && sl == 0) {
                    if constexpr (!SHADOW) c = shade_primary(s, st, o, d, slot, t);
                    float *pxo = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
                    pxo[0] = c.x;
                    pxo[1] = c.y;
                    pxo[2] = c.z;
                }
                if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
                if (COUNT) {
                    atomicAdd(&counters[0], (unsigned long long)cw.traversals);
                    atomicAdd(&counters[1], (unsigned long long)cw.nodes);
                    atomicAdd(&counters[2], (unsigned long long)cw.tris);
                    atomicAdd(&counters[3], (unsigned long long)cw.hits);
                    if (lane == 0) atomicAdd(&counters[7], 1ull);
                }
                return;
            }
            const int lx = lane & 7, ly = lane >> 3;
            const bool act = lx < tw && ly < th;
            Vec o, d;
            camera_ray(s.cam, tx0 + (act ? lx : 0), ty0 + (act ? ly : 0), o, d);
            LaneCounts cw = {};
            float t;
            const int bit = 8 * ((ty0 & 7) + ly) + (tx0 & 7) + lx;
            const int slot = trace_bins_wave<COUNT>(s, stage + (threadIdx.x >> 6) * kBinChunk, beg, end, bit, act, o,
                                                    d, t, cw, stamps ? &stamps[2 * wave] : nullptr);
            Vec c;
            if constexpr (SHADOW)   /* wave-wide */
                c = shade_hit_shadowed<COUNT>(s, st, act, o, d, slot, t, cw, tl.out_base + (int64_t)ly * tl.out_stride + lx);
            if (act) {
                if constexpr (!SHADOW) c = shade_primary(s, st, o, d, slot, t);
                float *pxo = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
                pxo[0] = c.x;
                pxo[1] = c.y;
                pxo[2] = c.z;
            }
            if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
            if (COUNT) {
                atomicAdd(&counters[0], (unsigned long long)cw.traversals);
                atomicAdd(&counters[1], (unsigned long long)cw.nodes);
                atomicAdd(&counters[2], (unsigned long long)cw.tris);
                atomicAdd(&counters[3], (unsigned long long)cw.hits);
                if (lane == 0) atomicAdd(&counters[7], 1ull);
            }
            return;
        }
    }
#if CRT_BVH_WINDOW
    if constexpr ((TRAV == 14 || TRAV == 15) && !FULL) {
        /* tiles of <= 16 rays (the measured plan's splits of heavy tiles):
         * each ray walked by a group of 64/R lanes (crt_walks.h trace_bvh_window) */
        const int tw = uniform_i(tl.w), th = uniform_i(tl.h);
        const int npx = tw * th;
        if (npx <= 16) {
            const int K = npx <= 4 ? 16 : 4;
            const int r = lane / K, sl = lane % K;
            const bool act = r < npx;
            const int px = act ? r % tw : 0, py = act ? r / tw : 0;
            Vec o, d;
            camera_ray(s.cam, tl.x + px, tl.y + py, o, d);
            LaneCounts cw = {};
            float t;
            const int slot = K == 16 ? trace_bvh_window<COUNT, 16>(s, sl, act, o, d, t, cw)
                                     : trace_bvh_window<COUNT, 4>(s, sl, act, o, d, t, cw);
            Vec c;
            if constexpr (SHADOW)   /* wave-wide */
                c = shade_hit_shadowed<COUNT>(s, st, act && sl == 0, o, d, slot, t, cw,
                                              tl.out_base + (int64_t)py * tl.out_stride + px);
            if (act && sl == 0) {
                if constexpr (!SHADOW) c = shade_primary(s, st, o, d, slot, t);
                float *pxo = out + 3 * (tl.out_base + (int64_t)py * tl.out_stride + px);
                pxo[0] = c.x;
                pxo[1] = c.y;
                pxo[2] = c.z;
            }
            if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
            if (COUNT) {
                atomicAdd(&counters[0], (unsigned long long)cw.traversals);
                atomicAdd(&counters[1], (unsigned long long)cw.nodes);
                atomicAdd(&counters[2], (unsigned long long)cw.tris);
                atomicAdd(&counters[3], (unsigned long long)cw.hits);
                if (lane == 0) atomicAdd(&counters[7], 1ull);
            }
            return;
        }
    }
#endif
    const int lx = lane & 7, ly = lane >> 3;
    const bool has_px = lx < tl.w && ly < tl.h;
    /* the sharing walks keep pixel-less lanes as helpers (they take donated node
     * ranges of the wave's rays); the other walks drop them */
    constexpr bool kHelpers = !FULL;   /* sharing walks use them; packet walks ignore them */
    if (!kHelpers && !has_px) return;
    LaneCounts cnt = {};
    constexpr bool kCoop = kIsCoop<TRAV> || kIsCoop<SEC>;   /* LDS only for the sharing walks */
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    Vec c;
    if constexpr (SHADOW && !FULL)
        c = shade_shadowed<(TRAV == 15 ? 14 : TRAV), COUNT>(s, st, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0),
                                                            cnt, &coop[kCoop ? (threadIdx.x >> 6) : 0], has_px,
                                                            tl.out_base + (int64_t)ly * tl.out_stride + lx);
    else
        c = shade_pixel<FULL, MAXF, (TRAV == 15 ? 14 : TRAV), (SEC == 15 ? 14 : SEC), COUNT, SHADOW>(
            s, st, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0), cnt, &coop[kCoop ? (threadIdx.x >> 6) : 0],
            has_px);
    if (has_px) {
        float *px = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
        px[0] = c.x;
        px[1] = c.y;
        px[2] = c.z;
    }
    if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
        if (lane == 0) {
            atomicAdd(&counters[4], (unsigned long long)cnt.wave_nodes);
            atomicAdd(&counters[5], (unsigned long long)cnt.wave_tris);
            atomicAdd(&counters[6], (unsigned long long)cnt.wave_edges);
            atomicAdd(&counters[7], 1ull);
            atomicAdd(&counters[8], (unsigned long long)cnt.wave_box);
            atomicAdd(&counters[9], (unsigned long long)cnt.wave_pass);
        }
    }
}


template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW>
__global__ CRT_RENDER_BOUNDS __attribute__((amdgpu_waves_per_eu(SHADOW && !FULL ? CRT_SHADOW_WAVES : TRAV == 13 ? CRT_WINDOW_WAVES : TRAV == 12 ? CRT_PACKET_WAVES : (TRAV == 14 || TRAV == 15) && !FULL ? CRT_BVH_WAVES : (FULL && MAXF == 4 ? CRT_GI_WAVES : 1)))) void k_render_tiles(const DeviceScene *__restrict__ scene, DSettings st,
                                                  const Tile *__restrict__ tiles,
                                                      int ntiles, float *__restrict__ out,
                                                      unsigned long long *__restrict__ counters,
                                                      unsigned long long *__restrict__ stamps, BinsPlan bp) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = (int)(threadIdx.x & 63);
    if (wave >= ntiles) return;
    /* The scene record is read through a pointer (not a by-value kernel
     * argument): its fields are then loaded where they are used, so shading
     * constants are not held in SGPRs across the tree walk (6 -> more waves/SIMD). */
    const DeviceScene &s = *scene;
    /* diagnostic build only (stamps != nullptr): wave start / end in s_memrealtime ticks (100 MHz) */
    if (stamps && lane == 0) stamps[2 * wave] = __builtin_amdgcn_s_memrealtime();
    if constexpr (TRAV == 15 && !FULL) {
        /* camera bins: the wave's work-list slot, then the entries a grid's
         * capacity further on when this frame's list outgrew the grid (the
         * camera moved since the sizing pass) */
        Tile tl;
        int bin_beg = 0, bin_len = -2;   /* the cell's list from the work list (-2: read it in render_tile) */
        BinsNext nx;
        const int r = bins_tile(bp, tiles, wave, tl, bin_beg, bin_len, nx);
        if (r == 2) bins_fill(s, bp, tiles, bin_beg, out, COUNT ? counters : nullptr);
        if (r != 1) return;
        const int bpar = bp.par, bncell = bp.ncell, quad = bp.quad;
        for (;;) {
            if (tl.w > 0 && tl.h > 0)   /* (a quarter outside a partial cell has no pixel) */
                render_tile<FULL, MAXF, TRAV, SEC, COUNT, SHADOW>(s, st, tl, bin_beg, bin_len, out, counters, stamps,
                                                                  bpar, bncell, wave, lane);
            nx.i += nx.step;
            if (nx.i >= nx.n) return;
            const BinsWork w = nx.work[nx.i];
            tl = w.t;
            bin_beg = w.off;
            bin_len = w.len;
            if (nx.q >= 0) bins_quarter(tl, nx.q, quad);
        }
    } else {
        render_tile<FULL, MAXF, TRAV, SEC, COUNT, SHADOW>(s, st, tiles[wave], 0, -2, out, counters, stamps, bp.par,
                                                          bp.ncell, wave, lane);
    }
}

/* Calibration probe (measured-cost tile plan): the camera rays of a tile
 * list traced with the frame's primary walk, no shading.  Each wave writes
 * its cost: for the packet walks the wave's node + triangle + edge steps
 * (what the wave pays: the union of its lanes' visit sets), for per-lane
 * walks the largest lane's node + triangle tests. */
template <int TRAV>
__global__ __launch_bounds__(256) void k_probe_tiles(const DeviceScene *__restrict__ scene,
                                                     const Tile *__restrict__ tiles, int ntiles,
                                                     uint32_t *__restrict__ wave_cost) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = (int)(threadIdx.x & 63);
    if (wave >= ntiles) return;
    const DeviceScene &s = *scene;
    const Tile tl = tiles[wave];
    const int lx = lane & 7, ly = lane >> 3;
    const bool has_px = lx < tl.w && ly < tl.h;
    Vec o, d;
    camera_ray(s.cam, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0), o, d);
    LaneCounts cnt = {};
    constexpr bool kCoop = kIsCoop<TRAV>;
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    float t;
    (void)trace<TRAV, true>(s, &coop[kCoop ? (threadIdx.x >> 6) : 0], has_px, o, d, t, cnt);
    constexpr bool kPacket = !kIsCoop<TRAV> && TRAV != 14;
    uint32_t c = kPacket ? cnt.wave_nodes + cnt.wave_tris + cnt.wave_edges : cnt.nodes + cnt.tris;
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o2 = (uint32_t)__shfl_xor((int)c, off);
        c = c > o2 ? c : o2;
    }
    if (lane == 0) wave_cost[wave] = c;
}

#define CRT_INST_TILES(F, M, T, S, C, SH) template __global__ CRT_TILES_SIG(F, M, T, S, C, SH)
#define CRT_INST_PROBE(T) template __global__ CRT_PROBE_SIG(T)
CRT_TILES_INSTANCES(CRT_INST_TILES)
CRT_PROBE_INSTANCES(CRT_INST_PROBE)

/* Deferred shadow rays, one record a lane (a group's lights side by side,
 * groups of neighbouring pixels after one another): the light's bins per
 * lane where the scene has them, the rays they leave undecided through the
 * wave's BVH walk, a failed proof through the exact kd walk — the answer of
 * shadow_occluded.  A persistent grid walks the records a wave at a time
 * (the walks' ballots need whole waves). */
__global__ __launch_bounds__(256) void k_shadow_vis(const DeviceScene *__restrict__ scene,
                                                    const ShRay *__restrict__ rays, ShCon *__restrict__ con,
                                                    const int32_t *__restrict__ count, int cap) {
    const DeviceScene &s = *scene;
    const int nl = s.light_count;
    const int ng = min(*count, cap);
    const int64_t n = (int64_t)((ng + 63) >> 6) * nl * 64;   /* whole chunks (sh_index) */
    const int lane = (int)(threadIdx.x & 63);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    LaneCounts cnt = {};
    for (int64_t base = (int64_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; base < n; base += nw * 64) {
        const int64_t i = base + lane;
        const int64_t g = ((i >> 6) / nl) * 64 + (i & 63);   /* the record's group and light (sh_index) */
        ShRay r;
        r.pix = -1;
        if (i < n && g < ng) r = rays[i];
        const bool act = r.pix >= 0;
        const int l = (int)((i >> 6) % nl);
        const Vec o = vec(r.ox, r.oy, r.oz), d = vec(r.dx, r.dy, r.dz);
        int res = 0;
        if (act) {
            res = -1;
            if (s.lbin_n) {
                WalkCounts wc = {0u, 0u};
                res = occluded_lbins<false>(s.lbins, s.lbin_off, s.lbin_par[l], s.lbin_n, s.prune_origin_max, s.nodes,
                                            s.slot_tri, s.ktopo, s.ktopo2, s.planes_ok != 0, o, d, r.r2, wc);
            }
        }
        if (s.bnodes && __ballot(act && res < 0) != 0ull) {
            const int rb = occluded_bvh_wave<false>(s, act && res < 0, o, d, r.r2, cnt);
            if (act && res < 0) res = rb;
        }
        if (act && res < 0) res = shadow_occluded_kd<false>(s, o, d, r.r2, cnt) ? 1 : 0;
        if (act) con[i].vis = res == 1 ? 0u : 1u;
    }
}

/* Each group's pixel: its visible lights' terms summed in light order, over
 * diffuse_reflection_ray_count + 1 (shade_hit_shadowed's operations). */
__global__ __launch_bounds__(256) void k_shadow_compose(const DeviceScene *__restrict__ scene, DSettings st,
                                                        const ShRay *__restrict__ rays, const ShCon *__restrict__ con,
                                                        const int32_t *__restrict__ count, int cap,
                                                        float *__restrict__ out) {
    const int nl = scene->light_count;
    const int n = min(*count, cap);
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < n; g += gridDim.x * blockDim.x) {
        const int32_t pix = rays[sh_index(g, 0, nl)].pix;
        if (pix < 0) continue;
        Vec acc = vec(0.f, 0.f, 0.f);
        for (int l = 0; l < nl; ++l) {
            const ShCon c = con[sh_index(g, l, nl)];
            if (c.vis) acc = vadd(acc, vec(c.x, c.y, c.z));
        }
        const Vec col = vdiv(acc, (float)(st.diffuse_reflection_ray_count + 1));
        float *po = out + 3 * (int64_t)pix;
        po[0] = col.x;
        po[1] = col.y;
        po[2] = col.z;
    }
}

/* empty kernel: its launch at scene creation loads this TU's code object
 * (warm_code_objects) */
__global__ void k_warm_render() {}

}  // namespace crt_amd
