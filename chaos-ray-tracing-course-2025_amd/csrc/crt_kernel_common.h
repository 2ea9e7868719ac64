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

/* Camera-bins dispatch of a tile plan (crt_bins.hip).  Every frame's
 * k_bins_sort puts each cell the plan renders as one tile into a work list by
 * its list length n — heavy (n >= split: four 4x4 waves, four lanes a pixel),
 * medium (n >= kBinsMedium), light (n >= 1), bvh (over the cap: the BVH walk) —
 * with the tile and the cell's (offset, length).  The render grid is the lists
 * in that order (kind q: kBinShards x cap[q] slots, slot i of shard s at
 * i kBinShards + s; heavy slots four waves each), then the plan's `rest` tiles
 * (not inside one cell, or sharing a cell), which read the cell's list
 * themselves, then the fill waves: 16 cells each, the background written to
 * the tiles of the cells with no candidate (every pixel misses).  Each list
 * holds up to ecap entries per shard (every cell of the shard fits); the grid
 * has gcap[q] slots per shard and kind, the scene's sizing-pass counts (at
 * least 1): a frame whose camera lists more cells of a kind than the grid
 * holds has each slot's wave take the entries gcap[q] apart in turn. */
constexpr int kBinKinds = 4;   /* heavy, medium, light, bvh */
struct alignas(16) BinsWork {
    Tile t;
    int32_t off, len;   /* the cell's records (len -1: the BVH walk) */
    int32_t cell, pad;
};
struct BinsPlan {
    int32_t *cell_tile;   /* per cell: the plan's one tile inside it; -1 none (the cell is not rendered), -2 several */
    const Tile *tiles;    /* the plan's tiles */
    BinsWork *work;       /* the lists: kind q, shard s, entry i at wbase[q] + s ecap + i */
    int32_t *phdr;        /* entries listed this frame: counter bins_phdr_at(set, kind, shard) */
    const int32_t *rest;  /* tiles the lists do not hold */
    int32_t gcap[kBinKinds], wbase[kBinKinds];   /* grid slots per shard; each kind's first entry */
    int32_t ecap;         /* entries per shard and kind (the shard's cells) */
    int32_t nrest, nfill, ncell;
    int32_t wslots;       /* work-list slots of one set (work: kBinSets sets; the frame's at par * wslots) */
    int32_t split, medium, quad;
    int32_t par;          /* the frame's set, frame % kBinSets (which counters and lists it uses) */
};

/* The device binning's per-frame counters, kBinSets sets taken in turn
 * (frame k uses set k % kBinSets; its first kernel zeroes set (k + 1) %
 * kBinSets for the next frame).
 * Every counter has a 256-B line of its own (atomics on one line serialise,
 * whatever word they name). */
constexpr int kBinPad = 64;   /* int32 per counter */
struct alignas(256) BinsCtr {
    int32_t v;
    int32_t pad[kBinPad - 1];
};
struct BinsHdr {
    BinsCtr n_every;
    BinsCtr nrem;              /* groups whose pairs past the first kExpand k_bins_pairs scatters */
    BinsCtr ne[kBinShards];    /* non-empty cells listed per shard */
    BinsCtr nb[kBinShards];    /* cells of more than 16 candidates listed per shard */
    BinsCtr rec[kBinShards];   /* records reserved per shard */
};
/* Sets of per-frame lists (records, per-cell off/len, work lists and their
 * counters, the binning's counts): frame k takes set k % kBinSets, so the
 * binnings of the next kBinSets - 1 frames may run while frame k renders. */
#ifndef CRT_BIN_SETS
#define CRT_BIN_SETS 3
#endif
constexpr int kBinSets = CRT_BIN_SETS;
static_assert(kBinSets >= 2, "a frame's binning clears the next frame's set");
/* a plan's work-list counters (BinsPlan::phdr) */
__host__ __device__ constexpr int bins_phdr_at(int par, int kind, int sh) {
    return ((par * kBinKinds + kind) * kBinShards + sh) * kBinPad;
}
constexpr int kBinsPhdrInts = kBinSets * kBinKinds * kBinShards * kBinPad;

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
