/*
 * crt_render_wf.hip — the wavefront path (C3: reflection / refraction
 * recursion without GI, crt_renderer.cpp:103-135): one kernel per recursion
 * level, then the deepest-first composition and the pixels.  Host
 * orchestration: crt_host_render.hip render_wavefront.  Built with its own
 * LLVM scheduling strategy (Makefile WF_SCHED).
 */
#define CRT_KERNEL_TU 1
/* the wavefront levels' BVH walk also loads each node's first triangle with
 * its successors (crt_bvh.h walk_bvh PF 2): an alive leaf then costs no load
 * round of its own (C3 lone frame 1.84 -> 1.77 ms; both triangles, PF 3: 1.81) */
#ifndef CRT_BVH_PREFETCH
#define CRT_BVH_PREFETCH 2
#endif
#ifdef CRT_WF_STAMPS
/* diagnostic builds only: per level and wave, s_memrealtime (100 MHz) at the
 * wave's start, once its BVH walk is done (crt_bvh.h CRT_WALK_HOOK), once its
 * trace is done (proof and fallbacks) and at its end, and how many of its
 * lanes ran the fallback walk (CRT_FALLBACK_HOOK) */
#include <hip/hip_runtime.h>
namespace crt_amd {
__device__ __forceinline__ unsigned long long *wf_phase_lds() {
    __shared__ unsigned long long p[4][2];
    return &p[threadIdx.x >> 6][0];
}
}  // namespace crt_amd
#if defined(__HIP_DEVICE_COMPILE__)
#define CRT_WALK_HOOK()                                                                                  \
    do {                                                                                                 \
        if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1)                              \
            crt_amd::wf_phase_lds()[0] = __builtin_amdgcn_s_memrealtime();                                \
    } while (0)
#define CRT_FALLBACK_HOOK() atomicAdd(&crt_amd::wf_phase_lds()[1], 1ull)
#endif
#endif
#include "crt_kernels.h"
#include "crt_shade.h"
#ifdef CRT_WF_STAMPS
#include <cstdio>
#include <vector>
#endif

namespace crt_amd {

#ifdef CRT_WF_STAMPS
/* per level and wave: start, walk done, trace done, end, fallback lanes;
 * COUNT frames: the sum and the max over its lanes of node + triangle tests */
constexpr int kWfStampWaves = 65536;
__device__ unsigned long long g_wf_stamps[16][kWfStampWaves][7];
int wf_stamps_dump(const char *fn, int levels) {
    std::vector<unsigned long long> h((size_t)16 * kWfStampWaves * 7);
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_wf_stamps), h.size() * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    FILE *f = std::fopen(fn, "w");
    if (!f) return -1;
    for (int L = 0; L < levels && L < 16; ++L)
        for (int w = 0; w < kWfStampWaves; ++w) {
            const unsigned long long *e = &h[((size_t)L * kWfStampWaves + w) * 7];
            if (e[0])
                std::fprintf(f, "%d %d %llu %llu %llu %llu %llu %llu %llu\n", L, w, e[0], e[1], e[2], e[3], e[4], e[5], e[6]);
        }
    std::fclose(f);
    std::fill(h.begin(), h.end(), 0ull);   /* the next frame's stamps start clean */
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wf_stamps), h.data(), h.size() * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#define WF_SLOT g_wf_stamps[LEVEL0 ? 0 : min(lv.depth, 15)][gid >> 6]
/* k: 0 start, 1 walk done (from LDS), 2 trace done, 3 end (+ the fallback count) */
#define WF_STAMP(k)                                                                                      \
    do {                                                                                                 \
        if (k == 0 && lane == 0) {                                                                       \
            wf_phase_lds()[0] = 0;                                                                       \
            wf_phase_lds()[1] = 0;                                                                       \
        }                                                                                                \
        if (lane == 0 && (gid >> 6) < kWfStampWaves) {                                                   \
            if (k == 2) WF_SLOT[1] = wf_phase_lds()[0];                                                  \
            if (k == 3) WF_SLOT[4] = wf_phase_lds()[1];                                                  \
            WF_SLOT[k == 0 ? 0 : k] = __builtin_amdgcn_s_memrealtime();                                  \
        }                                                                                                \
    } while (0)
/* COUNT frames: the wave's sum and max of node + triangle tests per lane */
#define WF_STEPS()                                                                                       \
    do {                                                                                                 \
        if (COUNT) {                                                                                     \
            unsigned st_sum = cnt.nodes + cnt.tris, st_max = st_sum;                                     \
            for (int m = 1; m < 64; m <<= 1) {                                                           \
                st_sum += (unsigned)__shfl_xor((int)st_sum, m);                                          \
                st_max = max(st_max, (unsigned)__shfl_xor((int)st_max, m));                              \
            }                                                                                            \
            if (lane == 0 && (gid >> 6) < kWfStampWaves) {                                               \
                WF_SLOT[5] = st_sum;                                                                     \
                WF_SLOT[6] = st_max;                                                                     \
            }                                                                                            \
        }                                                                                                \
    } while (0)
#else
#define WF_STAMP(k)
#define WF_STEPS()
#endif

template <int TRAV, bool LEVEL0, bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LEVEL0 ? CRT_WF0_WAVES : CRT_WF_WAVES))) void k_wf_level(const DeviceScene *__restrict__ scene, DSettings st,
                                                  const Tile *__restrict__ tiles, int ntiles, WLevel lv,
                                                  unsigned long long *__restrict__ counters) {
    const DeviceScene &s = *scene;
    int blk = (int)blockIdx.x;
    if (!LEVEL0) {
        /* blocks go round-robin to the 8 XCDs: give each XCD a contiguous range
         * of the queue (neighbouring rays share nodes in that XCD's L2; C3
         * 1.80 -> 1.76 ms, profiles/r03/ab_wf_xcd).  Level 0's tiles are
         * sorted heaviest first: they keep the round-robin deal. */
        const int nb = (int)gridDim.x, q = nb >> 3, r = nb & 7, x = blk & 7;
        blk = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (blk >> 3);
    }
    const int gid = (int)(blk * blockDim.x + threadIdx.x);
    const int lane = (int)(threadIdx.x & 63);
    WF_STAMP(0);
    /* this level's size and its children's first id: given, or (device-sized
     * frames) from the counts the levels before wrote */
    int n = lv.n, out_base = lv.out_base;
    if (!LEVEL0 && lv.dyn) {
        int64_t b = lv.n0;
        for (int k = 0; k < lv.depth; ++k) b += lv.dyn[k];
        n = min(lv.dyn[lv.depth - 1], lv.n);
        out_base = b < (int64_t)INT32_MAX ? (int)b : INT32_MAX;
    }
    constexpr bool kCoop = kIsCoop<TRAV>;
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    /* the level's waves: one pass over the grid, or (device-sized levels, a
     * fixed grid) each XCD strides over its own eighth of the level, as the
     * remap above gives each XCD a contiguous range */
    int wv = gid >> 6, wv_end = 0x7fffffff, wv_step = 0;
    if (!LEVEL0 && lv.dyn) {
        const int nw = (n + lv.rpw - 1) / lv.rpw, chunk = (nw + 7) >> 3, xcd = (int)blockIdx.x & 7;
        wv = xcd * chunk + ((int)blockIdx.x >> 3) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
        wv_end = min(nw, (xcd + 1) * chunk);
        wv_step = ((int)gridDim.x >> 3) * (int)(blockDim.x >> 6);
    }
    for (;; wv += wv_step) {   /* one pass unless the level is device-sized */
    if (wv >= wv_end) return;
    bool has;
    Vec o = vec(0.f, 0.f, 0.f), d = vec(0.f, 0.f, 1.f);
    int id = gid, depth = 0;
    Tile tl = {};
    if (LEVEL0) {
        const int wave = gid >> 6;
        if (wave >= ntiles) return;
        tl = tiles[wave];
        if (tl.prio & 1) __builtin_amdgcn_s_setprio(3);
        const int lx = lane & 7, ly = lane >> 3;
        has = lx < tl.w && ly < tl.h;
        if (has) camera_ray(s.cam, tl.x + lx, tl.y + ly, o, d);
    } else {
        const int ray0 = wv * lv.rpw;
        if (ray0 >= n) return;             /* whole wave past the queue */
        const int ray = ray0 + lane;
        has = lane < lv.rpw && ray < n;
        if (has) {
            const WRay r = lv.in[ray];
            o = vec(r.ox, r.oy, r.oz);
            d = vec(r.dx, r.dy, r.dz);
            id = r.id;
            depth = r.depth;
            has = (uint32_t)r.id < (uint32_t)lv.id_cap;   /* a skipped slot of an overflowing wave (id -1) */
        }
    }
    LaneCounts cnt = {};
    float t;
    int slot;
    slot = trace<TRAV, COUNT>(s, &coop[kCoop ? (threadIdx.x >> 6) : 0], has, o, d, t, cnt);
    WF_STAMP(2);

    WNode node = {wFinal, -1, -1, 0, 0.f, 0.f, 0.f, 0.f};
    Vec col = vec(0.f, 0.f, 0.f);
    int nch = 0;
    Vec co[2], cd[2];
    if (has) {
        if (slot < 0) {
            col = vec(s.background[0], s.background[1], s.background[2]);
        } else {
            HitRec h;
            make_hit(s, o, d, t, slot, h);
            const DMaterial m = s.materials[h.mat];
            if (m.type == CRT_MATERIAL_DIFFUSE) {
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                col = diffuse_finish(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb);
            } else if (m.type == CRT_MATERIAL_REFLECTIVE) {                 /* :103-107 */
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (s.reflections_on) {
                    node.kind = wReflect;
                    node.a0 = alb.x; node.a1 = alb.y; node.a2 = alb.z;
                    co[0] = vadd(h.p, vscale(h.n, st.reflection_bias));
                    cd[0] = vsub(d, vscale(vscale(h.n, 2.0f), vdot(d, h.n)));
                    nch = 1;
                } else {
                    col = alb;
                }
            } else if (m.type == CRT_MATERIAL_REFRACTIVE) {                 /* :109-135 */
                if (s.refractions_on) {
                    Vec n = h.n;
                    float n_out = 1.0f, n_in = m.ior;
                    if (vdot(d, n) > 0.0f) {
                        n = vneg(n);
                        const float tmp = n_in; n_in = n_out; n_out = tmp;
                    }
                    bool has_refr = false;
                    Vec rd = d;
                    {   /* Vector::refract (crt_vector.cpp:11-27) */
                        const float ca = -vdot(rd, n);
                        const float sa = sqrtf(1.0f - ca * ca);
                        if (!(sa > n_in / n_out)) {
                            const float sb = sa * n_out / n_in;
                            const float cb = sqrtf(1.0f - sb * sb);
                            rd = vadd(rd, vscale(n, ca));
                            rd = vnormalize(rd);
                            rd = vscale(rd, sb);
                            rd = vadd(rd, vscale(vneg(n), cb));
                            has_refr = true;
                        }
                    }
                    node.kind = has_refr ? wRefract2 : wRefract1;
                    node.a0 = fresnel_of(s, vdot(d, n));
                    co[0] = vadd(h.p, vscale(n, st.reflection_bias));
                    cd[0] = vsub(d, vscale(vscale(n, 2.0f), vdot(d, n)));
                    co[1] = vadd(h.p, vscale(vneg(n), 1e-2f));   /* refract_at's default bias (crt_ray.h:30-50) */
                    cd[1] = rd;
                    nch = has_refr ? 2 : 1;
                }
            } else {                                                         /* Constant :137-139 */
                col = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
            }
        }
    }
    /* children deeper than max_ray_depth are black without a trace: not queued */
    if ((uint32_t)depth + 1u > st.max_ray_depth) nch = 0;
    const unsigned long long b1 = __ballot(nch >= 1), b2 = __ballot(nch >= 2);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int total = __popcll(b1) + __popcll(b2);
    if (total > 0) {
        int base = 0;
        if (lane == __ffsll((long long)(b1 | b2)) - 1) {
            base = atomicAdd(lv.out_count, total);
            if (base + total > lv.out_cap || (int64_t)out_base + base + total > lv.id_cap) atomicOr(lv.overflow, 1);
        }
        base = __shfl(base, __ffsll((long long)(b1 | b2)) - 1);
        /* a lane's children side by side */
        const int k0 = base + __popcll(b1 & lt) + __popcll(b2 & lt);
        const int k1 = k0 + 1;
        /* never past the queue or the ids (the frame is then reported, not
         * used): the wave's reserved slots that exist are still filled — a
         * ray the next level skips (id -1) and, under each reserved id, a
         * final black activation — so a device-sized level, which takes every
         * reserved slot, reads no stale ray and the compose no stale node */
        if (base + total > lv.out_cap || (int64_t)out_base + base + total > lv.id_cap) {
            for (int c = 0; c < nch; ++c) {
                const int k = c == 0 ? k0 : k1;
                if (k < lv.out_cap) {
                    WRay r = {};
                    r.id = -1;
                    lv.out[k] = r;
                }
                if ((int64_t)out_base + k < lv.id_cap) {
                    WNode z = {};
                    z.kind = wFinal;
                    z.c0 = z.c1 = -1;
                    lv.nodes[out_base + k] = z;
                    lv.cols[out_base + k] = DVec4{0.f, 0.f, 0.f, 0.f};
                }
            }
            nch = 0;
        }
        for (int c = 0; c < nch; ++c) {
            const int k = c == 0 ? k0 : k1;
            WRay r;
            r.ox = co[c].x; r.oy = co[c].y; r.oz = co[c].z;
            r.dx = cd[c].x; r.dy = cd[c].y; r.dz = cd[c].z;
            r.id = out_base + k;
            r.depth = depth + 1;
            lv.out[k] = r;
            if (c == 0) node.c0 = r.id; else node.c1 = r.id;
        }
    }
    if (has) {
        lv.nodes[id] = node;
        if (node.kind == wFinal) lv.cols[id] = DVec4{col.x, col.y, col.z, 0.f};
    }
    WF_STEPS();
    WF_STAMP(3);
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
        /* levels >= 1 (coop walks): loop rounds per wave — sum, longest wave, waves */
        if (!LEVEL0 && kCoop && lane == 0) {
            atomicAdd(&counters[4], (unsigned long long)cnt.wave_nodes);
            atomicMax(&counters[6], (unsigned long long)cnt.wave_nodes);
            atomicAdd(&counters[7], 1ull);
        }
    }
    if (LEVEL0 || !lv.dyn) break;
    }
}

__device__ __forceinline__ Vec wf_compose(const WNode &nd, const DVec4 *__restrict__ cols, Vec own) {
    if (nd.kind == wFinal) return own;
    const Vec black = vec(0.f, 0.f, 0.f);
    const Vec c0 = nd.c0 >= 0 ? vec(cols[nd.c0].x, cols[nd.c0].y, cols[nd.c0].z) : black;
    if (nd.kind == wReflect) return vmul_quirk(vec(nd.a0, nd.a1, nd.a2), c0);
    if (nd.kind == wRefract1) return c0;   /* total internal reflection */
    const Vec c1 = nd.c1 >= 0 ? vec(cols[nd.c1].x, cols[nd.c1].y, cols[nd.c1].z) : black;
    const float fr = nd.a0;
    return vadd(vscale(c0, fr), vscale(c1, 1.0f - fr));
}

/* levels >= 1, deepest first: colour of every activation of the level */
__global__ __launch_bounds__(256) void k_wf_compose(const WNode *__restrict__ nodes, DVec4 *__restrict__ cols,
                                                    int32_t begin, int32_t n) {
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= n) return;
    const int id = begin + k;
    const WNode nd = nodes[id];
    if (nd.kind == wFinal) return;
    const Vec c = wf_compose(nd, cols, vec(0.f, 0.f, 0.f));
    cols[id] = DVec4{c.x, c.y, c.z, 0.f};
}

/* k_wf_compose for a device-sized frame: level `level`'s first id and size
 * from the counts (clamped to the queue and id capacities the level wrote) */
__global__ __launch_bounds__(256) void k_wf_compose_dyn(const WNode *__restrict__ nodes, DVec4 *__restrict__ cols,
                                                        const int32_t *__restrict__ counts, int32_t level, int32_t n0,
                                                        int32_t qcap, int32_t id_cap) {
    int64_t b = n0;
    for (int k = 0; k < level - 1; ++k) b += counts[k];
    const int64_t nq = min(counts[level - 1], qcap), nid = (int64_t)id_cap - b;
    const int64_t n = nq < nid ? nq : nid;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t id = b + k;
        const WNode nd = nodes[id];
        if (nd.kind == wFinal) continue;
        const Vec c = wf_compose(nd, cols, vec(0.f, 0.f, 0.f));
        cols[id] = DVec4{c.x, c.y, c.z, 0.f};
    }
}

/* level 0: compose the camera rays and write the pixels */
__global__ __launch_bounds__(256) void k_wf_pixels(const WNode *__restrict__ nodes, const DVec4 *__restrict__ cols,
                                                   const Tile *__restrict__ tiles, int ntiles,
                                                   float *__restrict__ out) {
    const int gid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int wave = gid >> 6, lane = gid & 63;
    if (wave >= ntiles) return;
    const Tile tl = tiles[wave];
    const int lx = lane & 7, ly = lane >> 3;
    if (!(lx < tl.w && ly < tl.h)) return;
    const WNode nd = nodes[gid];
    const Vec own = vec(cols[gid].x, cols[gid].y, cols[gid].z);
    const Vec c = wf_compose(nd, cols, own);
    float *px = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
    px[0] = c.x;
    px[1] = c.y;
    px[2] = c.z;
}

#define CRT_INST_WF(T, L0, C) template __global__ CRT_WF_SIG(T, L0, C)
CRT_WF_INSTANCES(CRT_INST_WF)

/* empty kernel: its launch at scene creation loads this TU's code object
 * (warm_code_objects) */
__global__ void k_warm_wf() {}

}  // namespace crt_amd
