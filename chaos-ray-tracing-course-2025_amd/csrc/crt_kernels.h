/*
 * crt_kernels.h — the render path's kernels as the host layer sees them:
 * their records, launch-shape defaults, declarations and the explicit
 * instantiation lists (each kernel family is compiled in one translation
 * unit: crt_render.hip tiles + probe, crt_render_gi.hip GI, crt_render_wf.hip
 * wavefront, crt_side_kernels.hip the small ones).
 */
#pragma once
#include "crt_kernel_common.h"

#ifndef CRT_GI_WAVES
#define CRT_GI_WAVES 5       /* min waves/SIMD asked of the depth<=3 frame-stack (GI) kernels: 96 VGPRs
                                * + 17 spilled beat 114 VGPRs at 4 waves (C4 1080^2: 102.8 vs 111.7 ms) and
                                * 80 VGPRs at 6 waves (116.6 ms) in same-box A/B */
#endif
#ifndef CRT_WINDOW_WAVES
#define CRT_WINDOW_WAVES 5   /* min waves/SIMD asked of the walk-13 kernel: 96 VGPRs (1 spilled); C2 0.1233 ms at
                              * its best plan vs 0.127-0.130 at 4 waves (profiles/r02/w5tune) */
#endif
#ifndef CRT_RENDER_BOUNDS
#define CRT_RENDER_BOUNDS __launch_bounds__(256)
#endif
#ifndef CRT_BVH_WINDOW
#define CRT_BVH_WINDOW 1     /* split tiles of camera frames on the BVH: one ray per group of lanes (trace_bvh_window) */
#endif
#ifndef CRT_BVH_WAVES
#ifndef CRT_SHADOW_WAVES
#define CRT_SHADOW_WAVES 3   /* min waves/SIMD asked of the shadow-ray kernels without recursion (1: no bound; 3: 0.41 against 0.52 ms, C2 with shadows) */
#endif
#define CRT_BVH_WAVES 1      /* min waves/SIMD asked of the camera BVH-walk (14) kernel (1: no bound) */
#endif
#ifndef CRT_PACKET_WAVES
#define CRT_PACKET_WAVES 5   /* min waves/SIMD asked of the walk-12 kernel (as walk 13) */
#endif
#ifndef CRT_GI10_WAVES
#define CRT_GI10_WAVES 4     /* min waves/SIMD of the refill kernel with the pruned walk (TRAV 10) */
#endif
#ifndef CRT_WF_WAVES
#define CRT_WF_WAVES 1       /* min waves/SIMD asked of the wavefront levels >= 1 */
#endif
#ifndef CRT_WF0_WAVES
#define CRT_WF0_WAVES 1      /* ... and of level 0 (camera rays) */
#endif

namespace crt_amd {
/* ---- wavefront path (C3, crt_render_wf.hip) ---- */
/* With GI off, shade_ray (crt_renderer.cpp:46-145) draws no random numbers:
 * each activation's colour is a pure function of its ray and of its
 * children's colours.  So the recursion is run level by level: every ray of
 * depth L is traced by one lane (no per-lane frame stack, no lane waiting for
 * its pixel's other branches), its children are appended to the level-L+1
 * queue, and a backward pass composes each activation's colour from its
 * children with the reference's operations (reflective: albedo * L with the
 * Vector quirk; refractive: fresnel blend, or the reflection colour on total
 * internal reflection).  A child deeper than max_ray_depth is black without
 * a trace, as in the reference (:47-48).  Level 0 is the camera rays of the
 * tile plan (packet walk); deeper levels are scattered rays (range-sharing
 * walk). */
enum WKind : int32_t { wFinal = 0, wReflect = 1, wRefract2 = 2, wRefract1 = 3 };

struct alignas(16) WRay {
    float ox, oy, oz, dx, dy, dz;
    int32_t id, depth;
};

struct alignas(16) WNode {
    int32_t kind, c0, c1, pad;   /* children ids, -1 = black (deeper than max_ray_depth) */
    float a0, a1, a2, a3;        /* reflective: albedo | refractive: a0 = fresnel */
};

struct WLevel {
    const WRay *in;
    int32_t n;               /* rays of this level (levels >= 1) */
    int32_t depth;
    WRay *out;               /* children of this level */
    int32_t *out_count;
    int32_t out_base;        /* id of out[0] */
    WNode *nodes;            /* by ray id */
    DVec4 *cols;             /* by ray id */
    int32_t rpw;             /* levels >= 1: rays per wave (lanes rpw..63 start idle and take donated pieces) */
    int32_t out_cap;         /* children this level may queue (recorded level sizes: exactly the next level) */
    int32_t *overflow;       /* set when a level queued more children than out_cap (none written) */
    /* device-sized frames: the levels' counts (level L's size is dyn[L - 1],
     * its first ray id n0 + dyn[0] + ... + dyn[L - 2]); n is then the queue's
     * capacity and the waves stride over the level; nullptr: n rays, one pass */
    const int32_t *dyn;
    int32_t n0;              /* camera rays (level 0's ids) */
    int32_t id_cap;          /* ray ids the node / colour arrays hold */
};

template <class T>
struct Rgb { T c[3]; };

/* One image row of the compact image copy (crt_api.hip image_to_host), in
 * pinned host memory: its pixels [x0, x1) hold every pixel whose bits differ
 * from the background's (x0 = x1: none). */
struct HostRow {
    int32_t x0, x1;
};

/* ---- declarations (definitions: the kernel TUs) ---- */
template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW = false>
__global__ void k_render_tiles(const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles,
                               int ntiles, float *__restrict__ out, unsigned long long *__restrict__ counters,
                               unsigned long long *__restrict__ stamps, BinsPlan bp);
template <int MAXF, int TRAV, bool COUNT>
__global__ void k_render_refill(const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles,
                                int ntiles, float *__restrict__ out, int32_t *__restrict__ next_px,
                                unsigned long long *__restrict__ counters);
template <bool COUNT>
__global__ void k_render_gi(const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles,
                            int ntiles, float *__restrict__ out, int32_t *__restrict__ next_px,
                            unsigned long long *__restrict__ counters, float4 *__restrict__ gframes);
template <int TRAV>
__global__ void k_probe_tiles(const DeviceScene *__restrict__ scene, const Tile *__restrict__ tiles, int ntiles,
                              uint32_t *__restrict__ wave_cost);
template <int TRAV, bool LEVEL0, bool COUNT>
__global__ void k_wf_level(const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles,
                           int ntiles, WLevel lv, unsigned long long *__restrict__ counters);
__global__ void k_wf_compose(const WNode *__restrict__ nodes, DVec4 *__restrict__ cols, int32_t begin, int32_t n);
__global__ void k_wf_compose_dyn(const WNode *__restrict__ nodes, DVec4 *__restrict__ cols,
                                 const int32_t *__restrict__ counts, int32_t level, int32_t n0, int32_t qcap,
                                 int32_t id_cap);
__global__ void k_wf_pixels(const WNode *__restrict__ nodes, const DVec4 *__restrict__ cols,
                            const Tile *__restrict__ tiles, int ntiles, float *__restrict__ out);
__global__ void k_trace_rays(DeviceScene s, const float *__restrict__ rays, int64_t n, crt_hit *__restrict__ hits,
                             int walk);
template <class T>
__global__ void k_unpack(const UnpackBucket *__restrict__ buckets, const T *__restrict__ src, T *__restrict__ dst,
                         int width, Rgb<T> bg);
__global__ void k_live_pixels(const DeviceScene *__restrict__ scene, uint8_t *__restrict__ live);
__global__ void k_put_record(DeviceScene *__restrict__ dst, DeviceScene v);
__global__ void k_quantize(const float *__restrict__ src, uint8_t *__restrict__ dst, int64_t n, float maxf, int maxi);
__global__ void k_row_spans(const float *__restrict__ img, int width, Rgb<uint32_t> bg, int2 *__restrict__ spans,
                            HostRow *__restrict__ rows);
__global__ void k_rows_to_host(const float *__restrict__ img, int width, int height, int y0,
                               const int2 *__restrict__ spans, float *__restrict__ host);
__global__ void k_warm_render();
/* deferred shadow rays (crt_layout.h ShRay / ShCon): visibility of every
 * record, then each group's pixel (crt_render.hip) */
__global__ void k_shadow_vis(const DeviceScene *__restrict__ scene, const ShRay *__restrict__ rays,
                             ShCon *__restrict__ con, const int32_t *__restrict__ count, int cap);
__global__ void k_shadow_compose(const DeviceScene *__restrict__ scene, DSettings st, const ShRay *__restrict__ rays,
                                 const ShCon *__restrict__ con, const int32_t *__restrict__ count, int cap,
                                 float *__restrict__ out);
__global__ void k_warm_gi();
__global__ void k_warm_wf();
__global__ void k_warm_side();
__global__ void k_warm_bins();

/* ---- instantiation lists (X(args...)) ---- */
#define CRT_TILES_INSTANCES(X)                                                                              \
    X(false, 0, 7, 7, false, false) X(false, 0, 7, 7, true, false) X(false, 0, 8, 8, false, false)        \
    X(false, 0, 8, 8, true, false) X(false, 0, 12, 12, false, false) X(false, 0, 12, 12, true, false)      \
    X(false, 0, 13, 13, false, false) X(false, 0, 13, 13, true, false) X(false, 0, 14, 14, false, false)   \
    X(false, 0, 14, 14, true, false) X(false, 0, 15, 15, false, false) X(false, 0, 15, 15, true, false)   \
    X(false, 0, 8, 8, false, true) X(false, 0, 8, 8, true, true) X(false, 0, 12, 12, false, true)          \
    X(false, 0, 12, 12, true, true) X(false, 0, 13, 13, false, true) X(false, 0, 13, 13, true, true)       \
    X(false, 0, 14, 14, false, true) X(false, 0, 14, 14, true, true) X(false, 0, 15, 15, false, true)      \
    X(false, 0, 15, 15, true, true)                                                                         \
    X(true, 4, 4, 4, false, false) X(true, 4, 4, 4, true, false) X(true, 16, 4, 4, false, false)           \
    X(true, 16, 4, 4, true, false) X(true, 64, 4, 4, false, false) X(true, 64, 4, 4, true, false)          \
    X(true, 4, 10, 10, false, false) X(true, 4, 10, 10, true, false) X(true, 16, 10, 10, false, false)     \
    X(true, 16, 10, 10, true, false) X(true, 64, 10, 10, false, false) X(true, 64, 10, 10, true, false)    \
    X(true, 4, 10, 10, false, true) X(true, 4, 10, 10, true, true) X(true, 16, 10, 10, false, true)        \
    X(true, 16, 10, 10, true, true) X(true, 64, 10, 10, false, true) X(true, 64, 10, 10, true, true)
#define CRT_TILES_SIG(F, M, T, S, C, SH) void k_render_tiles<F, M, T, S, C, SH>(const DeviceScene *__restrict__, \
    DSettings, const Tile *__restrict__, int, float *__restrict__, unsigned long long *__restrict__,          \
    unsigned long long *__restrict__, BinsPlan);
#define CRT_REFILL_INSTANCES(X) X(4, 4, false) X(4, 4, true) X(4, 10, false) X(4, 10, true) \
    X(16, 4, false) X(16, 4, true) X(64, 4, false) X(64, 4, true)
#define CRT_REFILL_SIG(MAXF, T, C) void k_render_refill<MAXF, T, C>(const DeviceScene *__restrict__, DSettings, \
    const Tile *__restrict__, int, float *__restrict__, int32_t *__restrict__, unsigned long long *__restrict__);
#define CRT_GIM_INSTANCES(X) X(false) X(true)
#define CRT_GIM_SIG(C) void k_render_gi<C>(const DeviceScene *__restrict__, DSettings, const Tile *__restrict__, int, \
    float *__restrict__, int32_t *__restrict__, unsigned long long *__restrict__, float4 *__restrict__);
#define CRT_PROBE_INSTANCES(X) X(7) X(8) X(12) X(13) X(14)
#define CRT_PROBE_SIG(T) void k_probe_tiles<T>(const DeviceScene *__restrict__, const Tile *__restrict__, int, \
    uint32_t *__restrict__);
#define CRT_WF_INSTANCES(X) X(4, false, false) X(4, false, true) X(10, false, false) X(10, false, true)        \
    X(14, false, false) X(14, false, true) X(7, true, false) X(7, true, true) X(8, true, false) X(8, true, true) \
    X(12, true, false) X(12, true, true) X(14, true, false) X(14, true, true)
#define CRT_WF_SIG(T, L0, C) void k_wf_level<T, L0, C>(const DeviceScene *__restrict__, DSettings, \
    const Tile *__restrict__, int, WLevel, unsigned long long *__restrict__);

#define CRT_EXTERN_TILES(F, M, T, S, C, SH) extern template __global__ CRT_TILES_SIG(F, M, T, S, C, SH)
#define CRT_EXTERN_REFILL(MAXF, T, C) extern template __global__ CRT_REFILL_SIG(MAXF, T, C)
#define CRT_EXTERN_GIM(C) extern template __global__ CRT_GIM_SIG(C)
#define CRT_EXTERN_PROBE(T) extern template __global__ CRT_PROBE_SIG(T)
#define CRT_EXTERN_WF(T, L0, C) extern template __global__ CRT_WF_SIG(T, L0, C)
#ifndef CRT_KERNEL_TU
CRT_TILES_INSTANCES(CRT_EXTERN_TILES)
CRT_REFILL_INSTANCES(CRT_EXTERN_REFILL)
CRT_GIM_INSTANCES(CRT_EXTERN_GIM)
CRT_PROBE_INSTANCES(CRT_EXTERN_PROBE)
CRT_WF_INSTANCES(CRT_EXTERN_WF)
extern template __global__ void k_unpack<float>(const UnpackBucket *__restrict__, const float *__restrict__,
                                                float *__restrict__, int, Rgb<float>);
extern template __global__ void k_unpack<uint8_t>(const UnpackBucket *__restrict__, const uint8_t *__restrict__,
                                                  uint8_t *__restrict__, int, Rgb<uint8_t>);
#endif

}  // namespace crt_amd
