/*
 * crt_kernel_common.h — records and small device helpers shared by the render
 * kernels (crt_render*.hip) and the host layer (crt_host_render.hip).
 */
#pragma once
#include <hip/hip_runtime.h>

#include "crt_bvh.h"
#include "crt_device.h"
#include "crt_host.h"

namespace crt_amd {

constexpr float kPi = 3.14159265358979323846f;   /* std::numbers::pi_v<float> */

struct alignas(16) Tile {
    int32_t x, y, w, h;        /* pixel rectangle, w,h <= 8 */
    int64_t out_base;          /* output pixel index of (x, y) */
    int32_t out_stride;        /* output pixels per row */
    int32_t prio;              /* bit 0: one of the frame's heaviest waves — raised issue priority;
                                * bit 1: camera-bins split tile, four lanes per pixel */
};

/* Counters of the device binning are sharded by cell (cell % kBinShards): a
 * device-scope atomic on one word serialises at ~88 per microsecond. */
constexpr int kBinShards = 16;

/* Camera-bins dispatch of a tile plan (crt_bins.hip): the render grid's first
 * 4 x kBinShards x ch waves take the cells k_bins_sort queued as heavy (four
 * 4x4 waves each; slot i of shard s at 4 (i kBinShards + s)), the next
 * kBinShards x cm the medium ones (one 8x8 wave each), the rest the plan's
 * base tiles in plan order, skipping the ones a priority wave took. */
struct BinsPlan {
    int32_t *cell_tile;   /* per cell: the plan's one tile inside it; -1 none (the cell is not rendered), -2 several */
    int32_t *taken;       /* per base tile: rendered by a priority wave this frame */
    int32_t *prio;        /* base-tile indices: heavy kBinShards x ch, then medium kBinShards x cm */
    int32_t *phdr;        /* cells queued this frame: counter bins_phdr_at(parity, heavy 0 / medium 1, shard) */
    int32_t ch, cm, nbase;
    int32_t split, medium, quad;
    int32_t par;          /* the frame's parity (which counters it uses) */
};

/* Per-frame counters of the device binning (crt_bins.hip), two sets used by
 * alternate frames: a frame's first kernel zeroes the other set for the next.
 * Every counter has a 256-B line of its own (atomics on one line serialise,
 * whatever word they name). */
constexpr int kBinPad = 64;   /* int32 per counter */
struct alignas(256) BinsCtr {
    int32_t v;
    int32_t pad[kBinPad - 1];
};
struct BinsHdr {
    BinsCtr n_every;
    BinsCtr ne[kBinShards];    /* non-empty cells listed per shard */
    BinsCtr rec[kBinShards];   /* records reserved per shard */
};
/* a plan's priority-list counters (BinsPlan::phdr): kind 0 heavy, 1 medium */
__host__ __device__ constexpr int bins_phdr_at(int par, int kind, int sh) {
    return ((par * 2 + kind) * kBinShards + sh) * kBinPad;
}
constexpr int kBinsPhdrInts = 4 * kBinShards * kBinPad;

/* Where each shard's records go in the camera-bins record buffer. */
struct BinsCaps {
    int32_t base[kBinShards];
    int32_t cap[kBinShards];
};

struct alignas(16) UnpackBucket {
    int32_t x, y, w, h;
    int64_t src;               /* float offset of the bucket inside the gathered buffer */
    int64_t pad;
};

enum FrameKind : int32_t { kDiffuseGI = 0, kReflect = 1, kRefractA = 2, kRefractB = 3 };

/* A pending shade_ray activation (crt_renderer.cpp:46-145) waiting for a child. */
struct Frame {
    int32_t kind, depth, i, has_refr;
    Vec acc;    /* diffuse: GI sum | reflect: albedo | refract: reflection colour */
    Vec p, n;   /* diffuse: hit point and shading normal                         */
    Vec a, b;   /* diffuse: right, forward basis | refract: refraction ray o, d   */
    Vec alb;    /* diffuse: albedo sample | refract: .x = fresnel                */
};

/* global (address space 1) load: a global_load instead of a flat one, whose
 * completion is tracked by vmcnt alone (flat loads also count in lgkmcnt, so
 * every wait on them drains the LDS queue too) */
template <class T>
__device__ __forceinline__ T load_global(const T *p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    using GT = const __attribute__((address_space(1))) T;
    return ((GT *)p)[i];
#else
    return p[i];
#endif
}


struct LaneCounts {
    uint32_t traversals, nodes, tris, hits;
    /* wave-uniform steps of the packet walks (kept by every lane, added once per wave) */
    uint32_t wave_nodes, wave_tris, wave_edges;
    uint32_t wave_box, wave_pass;   /* packet walks: node steps with a box test run / with a lane passing */
    uint32_t win_steps, win_slots, win_reached, win_rounds;   /* window walk (crt_wave_counts) */
};

__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

/* Scene records are read-only for the whole launch: reading them through the
 * constant address space lets a wave-uniform index become an s_load into SGPRs. */
template <class T>
__device__ __forceinline__ T load_scalar(const T *p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    using CT = const __attribute__((address_space(4))) T;
    return ((CT *)p)[i];
#else
    return p[i];
#endif
}

/* Same, at a 32-bit byte offset from a wave-uniform base (SMEM base + offset
 * addressing: no 64-bit address arithmetic per load). */
template <class T>
__device__ __forceinline__ T load_scalar_at(const char *base, uint32_t byte_off) {
#if defined(__HIP_DEVICE_COMPILE__)
    using CT = const __attribute__((address_space(4))) T;
    return *(CT *)((const __attribute__((address_space(4))) char *)base + byte_off);
#else
    return *(const T *)(base + byte_off);
#endif
}

}  // namespace crt_amd
