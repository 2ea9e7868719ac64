/*
 * crt_bins.hip — camera bins built on the device inside every camera frame
 * (crt_bins.h; walked by crt_walks.h trace_bins_wave / trace_bins_lanes).
 *
 * The reference traces every camera ray through its tree inside the timed
 * render_image call (crt_renderer.cpp:147-155, timed at main.cpp:37-39); the
 * lists that let a camera ray test only the triangles its 8x8 cell can hit
 * depend on the camera and the resolution, so they are rebuilt by every frame
 * that walks them, before its render kernel:
 *
 *   k_bins_project  one block per 32 triangles, 8 lanes each (one hull corner
 *                   per lane): the hull's projection (pixel rectangle, dmin,
 *                   everywhere); then the group's (triangle, cell) pairs, spread
 *                   over the block's 256 threads, take a slot of their cell
 *                   (atomic count) and write the key (dmin, id) there
 *                   (kBinCellCap slots per cell); a cell's first pair appends
 *                   it to its shard's non-empty list, its 17th to the long
 *                   list.  A group with more than kExpand pairs queues the
 *                   rest for k_bins_pairs, which spreads them over its grid
 *                   (launched when the scene's sizing pass queued groups).
 *                   Also zeroes this frame's per-cell lengths and the other
 *                   set's counts (kBinSets sets taken in turn).
 *   k_bins_sort     the long lists one a wave, the others four a wave (16
 *                   lanes each): the cell's keys plus the everywhere ids
 *                   ranked in LDS, written as CamCand records (static part
 *                   from the per-triangle template, dmin, the cell's pixel
 *                   mask, and `rest`, the OR of the masks from here to the
 *                   list's end) into a range reserved with one atomic; the
 *                   cell's (offset, length); and its entry in the tile plan's
 *                   work lists by length (crt_kernel_common.h BinsPlan: heavy
 *                   cells four 4x4 waves, then medium, light, BVH; empty cells
 *                   get the background from the render's fill waves).
 *
 * Each step is a chain of dependent memory round trips (~1-2 us each at this
 * size), not bandwidth: the kernels are shaped to issue what they can in one
 * round (a cell's count, tile and first keys together; the record range's
 * atomic with the templates' loads), and every per-frame counter has a
 * 256-B line of its own, sharded by cell (device atomics on one line
 * serialise).
 *
 * The lists equal the host checker's (crt_bvh_build.cpp build_camera_bins)
 * record for record (tests/test_gpu_bins.py); the records of different cells
 * sit in the buffer in no particular order (each cell's range is reserved by
 * an atomic), which no reader depends on.  Scene create runs k_bins_project
 * once to size the buffers (records, work lists, grids) and to decide whether the
 * scene takes bins at all (crt_bins.h caps); a frame whose lists would not fit
 * renders the cells that do not fit on the BVH walk — the same image.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "crt_bins.h"
#include "crt_scene_impl.h"

namespace crt_amd {

#ifdef CRT_BINS_CHECK
/* diagnostic builds only: every index of the binning kernels checked against
 * its buffer's size; the first violation is recorded (and the index clamped
 * to 0, so the kernels stay on their control flow) */
struct BinsDbg {
    int32_t code, idx, bound, pad;
    int32_t nt, ncell, rec_cap, ne_cap;
};
__device__ BinsDbg g_bins_dbg;
__device__ int bins_ck(int64_t i, int64_t n, int code) {
    if (i < 0 || i >= n) {
        if (atomicCAS(&g_bins_dbg.code, 0, code) == 0) {
            g_bins_dbg.idx = (int32_t)i;
            g_bins_dbg.bound = (int32_t)n;
        }
        return 0;
    }
    return (int)i;
}
#define BCK(i, n, code) bins_ck((int64_t)(i), (int64_t)(n), (code))
#define BDBG(f) g_bins_dbg.f
#else
#define BCK(i, n, code) (i)
#endif

#ifdef CRT_BINS_STAMPS
/* diagnostic builds only: per block of k_bins_project, s_memrealtime (100 MHz)
 * at its start, after the projection, after the pair-count scan and at its end */
__device__ unsigned long long g_bins_stamps[8192 * 4];
#define BSTAMP(k) \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_bins_stamps[4 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime()
/* ... and per block of k_bins_sort: start, counters read, cell read, list written, end; the list length */
__device__ unsigned long long g_bins_stamps4[16384 * 6];
#define BSTAMP4(k) \
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_bins_stamps4[6 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime()
/* (k_bins_sort: wave 0 of each block) */
#else
#define BSTAMP(k)
#define BSTAMP4(k)
#endif

namespace {

#ifndef CRT_BINS_CNT_STRIDE
#define CRT_BINS_CNT_STRIDE 16   /* int32 between two cells' counters (atomics on one line serialise) */
#endif
constexpr int kCntStride = CRT_BINS_CNT_STRIDE;
#ifndef CRT_PAIRS_PER_BLOCK
#define CRT_PAIRS_PER_BLOCK 512
#endif
constexpr int kProjTris = 32;     /* triangles per k_bins_project block: 8 lanes each (one hull corner per lane) */

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t v, int d) {
    const int lo = __shfl_down((int)(uint32_t)v, d), hi = __shfl_down((int)(uint32_t)(v >> 32), d);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ double shfl_xor_f64(double v, int m) {
    const uint64_t u = shfl_xor_u64((uint64_t)__double_as_longlong(v), m);
    return __longlong_as_double((long long)u);
}

/* ascending bitonic sort of one key per lane over the wave */
__device__ __forceinline__ uint64_t wave_sort(uint64_t key, int lane) {
    for (int k = 2; k <= 64; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = shfl_xor_u64(key, j);
            const bool up = (lane & k) == 0, low = (lane & j) == 0;
            key = (low == up) ? (key < o ? key : o) : (key < o ? o : key);
        }
    return key;
}

/* inclusive suffix OR over the wave (lanes past the list hold 0) */
__device__ __forceinline__ uint64_t wave_suffix_or(uint64_t v, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = shfl_down_u64(v, d);
        if (lane + d < 64) v |= u;
    }
    return v;
}

}  // namespace

/* (triangle, cell) pairs -> cell slots: the atomics of a thread's pairs in
 * flight together; each pair writes its key (dmin, id) to its slot
 * (kBinCellCap slots per cell), the first pair of a cell lists the cell in its
 * shard's non-empty list, the 17th in its shard's list of long ones.  cell < 0:
 * no pair. */
constexpr int kSortGroup = 16;   /* k_bins_sort: lanes per cell of its first pass (longer lists: a wave each) */

template <int U>
__device__ __forceinline__ void bins_scatter(const int (&cell)[U], const uint64_t (&key)[U], int32_t *__restrict__ cnt,
                                             uint64_t *__restrict__ keys, int32_t *__restrict__ nonempty,
                                             int32_t *__restrict__ bigl, int cap_shard, BinsHdr *__restrict__ hdr) {
    int slot[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        slot[u] = cell[u] >= 0 ? atomicAdd(&cnt[(size_t)BCK(cell[u], BDBG(ncell), 7) * kCntStride], 1) : kBinCellCap;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (cell[u] < 0 || !keys) continue;   /* (no keys: the create's counting pass, bins_view) */
        if (slot[u] < kBinCellCap)
            keys[BCK((size_t)cell[u] * kBinCellCap + slot[u], (int64_t)BDBG(ncell) * kBinCellCap, 8)] = key[u];
        if (slot[u] == 0) {
            const int sh = cell[u] % kBinShards;
            nonempty[BCK(sh * cap_shard + atomicAdd(&hdr->ne[BCK(sh, kBinShards, 9)].v, 1), BDBG(ne_cap), 10)] = cell[u];
        } else if (slot[u] == kSortGroup) {   /* the cell's list outgrows a 16-lane group: a wave of its own */
            const int sh = cell[u] % kBinShards;
            bigl[BCK(sh * cap_shard + atomicAdd(&hdr->nb[sh].v, 1), BDBG(ne_cap), 13)] = cell[u];
        }
    }
}

/* the cell of pair j of an item's rectangle (row-major over its cells) */
__device__ __forceinline__ int bins_pair_cell(const BinItem &it, int j, int tx) {
    const int x0 = it.px0 >> 3, w = (it.px1 >> 3) - x0 + 1;
    return ((it.py0 >> 3) + j / w) * tx + x0 + j % w;
}

constexpr int kPairsPerThread = 4;
constexpr int kExpand = 256 * kPairsPerThread;
constexpr int kMaxGroups = 8192;   /* 2^18 triangles (bins are built up to the BVH's limit) */

/* The queued groups' pairs past the first kExpand, spread evenly over the
 * blocks of k_bins_pairs (bid of nblk): each block scans the queued groups' remaining
 * counts in LDS, finds each of its pairs' group, then its triangle (the
 * group's prefixes), then its cell. */
__device__ void bins_pairs(const BinItem *__restrict__ items, const int32_t *__restrict__ tpref,
                           const int32_t *__restrict__ gsum, const int32_t *__restrict__ rem, int nt, int tx,
                           int32_t *__restrict__ cnt, uint64_t *__restrict__ keys, int32_t *__restrict__ nonempty,
                           int32_t *__restrict__ bigl, int cap_shard, BinsHdr *__restrict__ hdr, int bid, int nblk,
                           int qmax) {
    __shared__ int32_t gp[kMaxGroups + 1];
    __shared__ int32_t part[256];
    const int tid = (int)threadIdx.x;
    const int nq = min(hdr->nrem.v, qmax);   /* k_bins_project queues no more (the rest scatter themselves) */
    /* exclusive prefix of the queued groups' remaining counts: each thread sums a run, then the runs are scanned */
    const int per = (nq + 255) / 256, g0 = tid * per, g1 = min(nq, g0 + per);
    int run = 0;
    for (int k = g0; k < g1; ++k) run += gsum[BCK(rem[k], BDBG(nt), 36)] - kExpand;
    part[tid] = run;
    __syncthreads();
    if (tid < 64) {
        int a = 0;
        for (int k = 0; k < 4; ++k) a += part[4 * tid + k];
        int incl = a;
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (tid >= d) incl += v;
        }
        int base = incl - a;
        for (int k = 0; k < 4; ++k) {
            const int v = part[4 * tid + k];
            part[4 * tid + k] = base;
            base += v;
        }
        if (tid == 63) gp[kMaxGroups] = incl;
    }
    __syncthreads();
    {
        int acc = part[tid];
        for (int k = g0; k < g1; ++k) {
            gp[k] = acc;
            acc += gsum[rem[k]] - kExpand;
        }
    }
    __syncthreads();
    const int total = gp[kMaxGroups];
    const int p0 = (int)((int64_t)total * bid / nblk), p1 = (int)((int64_t)total * (bid + 1) / nblk);
    for (int pb = p0 + tid; pb < p1; pb += 256 * 2) {
        int cell[2];
        uint64_t key[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = pb + u * 256;
            cell[u] = -1;
            if (p >= p1) continue;
            int lo = 0, hi = nq - 1;   /* the last queued group whose pairs start at or before p */
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (gp[mid] <= p) lo = mid;
                else hi = mid - 1;
            }
            const int r = kExpand + p - gp[lo];   /* the pair inside its group */
            /* ... and the triangle inside the group: the group's prefixes in one
             * round of loads (kProjTris contiguous ints), the last one <= r */
            const int a0 = rem[lo] * kProjTris, na = min(nt - a0, kProjTris);
            const int4 *tp4 = reinterpret_cast<const int4 *>(tpref + BCK(a0, BDBG(nt), 34));
            int4 v[kProjTris / 4];
#pragma unroll
            for (int q = 0; q < kProjTris / 4; ++q) v[q] = load_global(tp4, q);
            int a = a0, pr = 0;
#pragma unroll
            for (int q = 0; q < kProjTris / 4; ++q) {
                const int e[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                for (int z = 0; z < 4; ++z)
                    if (4 * q + z < na && e[z] <= r) {
                        a = a0 + 4 * q + z;
                        pr = e[z];
                    }
            }
            const BinItem it = items[BCK(a, BDBG(nt), 35)];
            cell[u] = bins_pair_cell(it, r - pr, tx);
            key[u] = bin_key(it.dmin, a);
        }
        bins_scatter<2>(cell, key, cnt, keys, nonempty, bigl, cap_shard, hdr);
    }
}


/* Projection + scatter, one block per group of kProjTris triangles: 8 lanes
 * per triangle (lane q projects hull corner q; the bounds are reduced over
 * the 8) give the item; the group's pair counts are scanned in LDS and the
 * block's 256 threads scatter the group's first kExpand (triangle, cell)
 * pairs themselves — a group with more (a triangle covering thousands of
 * cells) queues its rest for k_bins_pairs.
 * Also the everywhere list, this frame's per-cell lengths (zero) and the other
 * set's counters (zero for the next frame). */
__global__ __launch_bounds__(256) void k_bins_project(const CamCand *__restrict__ tpl, int nt, BinCamera cam,
                                                      BinItem *__restrict__ items, int32_t *__restrict__ tpref,
                                                      int32_t *__restrict__ gsum, int32_t *__restrict__ every,
                                                      BinsHdr *__restrict__ hdr2, int par,
                                                      int32_t *__restrict__ phdr2, int32_t *__restrict__ bin_len,
                                                      int ncell, int tx, int32_t *__restrict__ cnt2,
                                                      uint64_t *__restrict__ keys, int32_t *__restrict__ nonempty,
                                                      int32_t *__restrict__ bigl, int cap_shard, int32_t *__restrict__ rem,
                                                      int queue) {
    __shared__ int32_t npl[kProjTris];
    __shared__ int32_t spre[kProjTris + 1];
    __shared__ BinItem sit[kProjTris];
    const int tid = (int)threadIdx.x;
    BSTAMP(0);
    BinsHdr *hdr = hdr2 + par;
    int32_t *cnt = cnt2 + (size_t)par * ncell * kCntStride;
    /* the next set's counters start the next frame at zero (this frame
     * does not touch them; the previous one is done with them) */
    if (blockIdx.x == 0) {
        BinsHdr *o = hdr2 + (par + 1) % kBinSets;
        if (tid == 0) o->n_every.v = 0;
        if (tid == 1) o->nrem.v = 0;
        if (tid < kBinShards) {
            o->ne[tid].v = 0;
            o->nb[tid].v = 0;
            o->rec[tid].v = 0;
        }
        /* this frame's work-list counters (k_bins_sort appends after this
         * kernel; the render kBinSets frames back, same set, is done with them) */
        if (phdr2 && tid < kBinKinds * kBinShards)
            phdr2[BCK(bins_phdr_at(par, tid / kBinShards, tid % kBinShards), kBinsPhdrInts, 1)] = 0;
    }
    /* this frame's per-cell lengths start empty (k_bins_sort sets the listed
     * cells'); the next set's counts start the next frame at zero */
    for (int i = (int)(blockIdx.x * blockDim.x) + tid; i < ncell; i += (int)(gridDim.x * blockDim.x)) {
        bin_len[BCK(i, BDBG(ncell), 2)] = 0;
        cnt2[((size_t)((par + 1) % kBinSets) * ncell + BCK(i, BDBG(ncell), 2)) * kCntStride] = 0;
    }
    const int tl = tid >> 3, q = tid & 7;
    const int t0 = (int)blockIdx.x * kProjTris, t = t0 + tl;
    double lo[3] = {0.0, 0.0, 0.0}, hi[3] = {0.0, 0.0, 0.0};
    double X0 = INFINITY, X1 = -INFINITY, Y0 = INFINITY, Y1 = -INFINITY;
    int behind = 0;
    if (t < nt) {
        const float *b = reinterpret_cast<const float *>(tpl + BCK(t, BDBG(nt), 4));   /* lo_x, hi_x, lo_y, ... */
        lo[0] = b[0]; hi[0] = b[1]; lo[1] = b[2]; hi[1] = b[3]; lo[2] = b[4]; hi[2] = b[5];
        double X, Y;
        if (bin_corner(lo, hi, q, cam, X, Y)) {
            X0 = X1 = X;
            Y0 = Y1 = Y;
        } else {
            behind = 1;
        }
    }
    for (int d = 1; d < 8; d <<= 1) {
        X0 = fmin(X0, shfl_xor_f64(X0, d));
        X1 = fmax(X1, shfl_xor_f64(X1, d));
        Y0 = fmin(Y0, shfl_xor_f64(Y0, d));
        Y1 = fmax(Y1, shfl_xor_f64(Y1, d));
        behind |= __shfl_xor(behind, d);
    }
    if (q == 0) {
        int np = 0;
        BinItem it{};
        it.px0 = 1;   /* no pixels */
        if (t < nt) {
            it = bin_finish(behind != 0, X0, X1, Y0, Y1, bin_dmin(lo, hi, cam), cam);
            items[BCK(t, BDBG(nt), 5)] = it;
            if (it.every) {
                const int k = atomicAdd(&hdr->n_every.v, 1);
                if (k < kBinMaxEverywhere) every[BCK(k, kBinMaxEverywhere, 6)] = t;
            } else if (it.px0 <= it.px1) {
                np = ((it.px1 >> 3) - (it.px0 >> 3) + 1) * ((it.py1 >> 3) - (it.py0 >> 3) + 1);
            }
        }
        npl[tl] = np;
        sit[tl] = it;
    }
    BSTAMP(1);
    __syncthreads();
    if (tid < 64) {   /* wave 0: the group's exclusive prefix and sum */
        const int np = tid < kProjTris ? npl[tid] : 0;
        int incl = np;
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (tid >= d) incl += v;
        }
        const int tt = t0 + tid;
        if (tid < kProjTris) spre[tid] = incl - np;
        if (tid < kProjTris && tt < nt) tpref[BCK(tt, BDBG(nt), 33)] = incl - np;
        if (tid == kProjTris - 1) {
            spre[kProjTris] = incl;
            gsum[blockIdx.x] = incl;
        }
    }
    /* the group's pairs past kExpand go to k_bins_pairs when it is launched
     * (queue) and holds a slot for the group (its LDS scan takes kMaxGroups);
     * otherwise the block scatters them itself, kExpand a round */
    __shared__ int s_queued;
    __syncthreads();   /* spre: wave 0's scan */
    const int G = spre[kProjTris];
    if (tid == 0) {
        int qd = 0;
        if (G > kExpand && queue) {
            const int k = atomicAdd(&hdr->nrem.v, 1);
            if (k < queue) {   /* (queue: the groups k_bins_pairs takes, <= kMaxGroups) */
                rem[BCK(k, BDBG(nt), 38)] = (int)blockIdx.x;
                qd = 1;
            }
        }
        s_queued = qd;
    }
    __syncthreads();
    BSTAMP(2);
    const int lim = s_queued ? kExpand : G;
    for (int base = 0; base < lim; base += kExpand) {
        const int E = min(lim - base, kExpand);
        if (tid >= E) break;
        int cell[kPairsPerThread];   /* pairs base + tid + 256 u of the group */
        uint64_t key[kPairsPerThread];
#pragma unroll
        for (int u = 0; u < kPairsPerThread; ++u) {
            const int p = tid + 256 * u;
            cell[u] = -1;
            if (p >= E) continue;
            const int pg = base + p;
            int a = 0;   /* the last triangle whose pairs start at or before pg */
#pragma unroll
            for (int st = kProjTris / 2; st > 0; st >>= 1)
                if (spre[a + st] <= pg) a += st;
            const BinItem it = sit[a];
            cell[u] = bins_pair_cell(it, pg - spre[a], tx);
            key[u] = bin_key(it.dmin, t0 + a);   /* the cell's sort key: (dmin, id) */
        }
        bins_scatter<kPairsPerThread>(cell, key, cnt, keys, nonempty, bigl, cap_shard, hdr);
    }
    BSTAMP(3);
}


/* k_bins_sort: one wave per listed cell (every cell when some hull is
 * everywhere), four independent waves a block.  The cell's keys (its own
 * from the scatter, then the everywhere ids at dmin 0) are ranked in LDS —
 * each key's rank is the number of smaller keys (keys are distinct: they hold
 * the id) — and put in order; then the records are written chunk by chunk from
 * the list's end, so `rest` (the OR of the masks from here to the end) is
 * carried: the static part from the triangle's template, dmin from the key,
 * the cell's pixels inside the triangle's rectangle. */
constexpr int kSortWaves = 4;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int kPer>   /* keys per lane: n <= 64 kPer */
__device__ void bins_emit(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items,
                          const uint64_t *__restrict__ own, int m, const int32_t *__restrict__ every, int n, int cx,
                          int cy, CamCand *__restrict__ out, uint64_t *sk, int lane) {
    uint64_t mine[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        const int j = lane + 64 * r;
        mine[r] = ~0ull;
        if (j < n) mine[r] = j < m ? own[BCK(j, kBinCellCap, 11)] : bin_key(0.0f, every[BCK(j - m, kBinMaxEverywhere, 12)]);
        if (j < n) sk[j] = mine[r];
    }
    wave_lds_sync();
    int rank[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) rank[r] = 0;
    for (int i = 0; i < n; ++i) {   /* broadcast reads: every lane compares its keys with key i */
        const uint64_t k = sk[i];
#pragma unroll
        for (int r = 0; r < kPer; ++r) rank[r] += k < mine[r] ? 1 : 0;
    }
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < kPer; ++r)
        if (lane + 64 * r < n) sk[rank[r]] = mine[r];
    wave_lds_sync();
    uint64_t carry = 0ull;
    static_assert(sizeof(CamCand) == 6 * sizeof(float4), "CamCand is six float4");
    for (int base = ((n - 1) >> 6) << 6; base >= 0; base -= 64) {
        const int j = base + lane;
        uint64_t mask = 0ull;
        float4 q[6];   /* the record in registers (loaded with the item: one round trip) */
        float dmin = 0.0f;
        if (j < n) {
            const int t = (int)(uint32_t)sk[j];
            const BinItem it = items[BCK(t, BDBG(nt), 19)];
            const float4 *src = reinterpret_cast<const float4 *>(tpl + BCK(t, BDBG(nt), 20));
#pragma unroll
            for (int r = 0; r < 6; ++r) q[r] = load_global(src, r);
            mask = bin_mask(it, cx, cy);
            dmin = it.dmin;
        }
        const uint64_t rest = wave_suffix_or(mask, lane) | carry;
        {
            const int lo = __shfl((int)(uint32_t)rest, 0), hi = __shfl((int)(uint32_t)(rest >> 32), 0);
            carry = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
        }
        if (j < n) {   /* dmin: float 6; mask: floats 20-21; rest: 22-23 */
            q[1].z = dmin;
            q[5].x = __uint_as_float((uint32_t)mask);
            q[5].y = __uint_as_float((uint32_t)(mask >> 32));
            q[5].z = __uint_as_float((uint32_t)rest);
            q[5].w = __uint_as_float((uint32_t)(rest >> 32));
            float4 *dst = reinterpret_cast<float4 *>(out + j);
#pragma unroll
            for (int r = 0; r < 6; ++r) dst[r] = q[r];
        }
    }
    wave_lds_sync();   /* sk is reused by the wave's next cell */
}

/* n <= 64 (nearly every cell): one candidate per lane (key: this lane's, in
 * no order).  The cell's record range is reserved (lane 0's atomic on the
 * shard's counter) while the lane's template and item load and the keys are
 * ranked; the record is written straight to its ranked position, and only the
 * masks and `rest` go through LDS (sk[0..63] keys, [64..127] masks by rank,
 * [128..191] rest by rank).  Returns the range's start (-1: the shard's
 * region is full, the cell walks the BVH). */
__device__ int bins_emit64(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items, uint64_t key, int n,
                           int cx, int cy, CamCand *__restrict__ region, int cap, int32_t *__restrict__ ctr,
                           uint64_t *sk, int lane) {
    const bool on = lane < n;
    int tick = 0;
    if (lane == 0) tick = atomicAdd(ctr, n);
    const int t = (int)(uint32_t)key;
    BinItem it{};
    float4 q[6];
    if (on) {   /* in flight with the atomic during the ranking */
        it = items[BCK(t, BDBG(nt), 19)];
        const float4 *src = reinterpret_cast<const float4 *>(tpl + BCK(t, BDBG(nt), 20));
#pragma unroll
        for (int r = 0; r < 6; ++r) q[r] = load_global(src, r);
    }
    if (on) sk[lane] = key;
    wave_lds_sync();
    int rank = 0;
    for (int i = 0; i < n; ++i) rank += sk[i] < key ? 1 : 0;
    const uint64_t mask = on ? bin_mask(it, cx, cy) : 0ull;
    if (on) sk[64 + rank] = mask;
    wave_lds_sync();
    const uint64_t rest = wave_suffix_or(on ? sk[64 + lane] : 0ull, lane);   /* lane i: the rank-i record's rest */
    if (on) sk[128 + lane] = rest;
    wave_lds_sync();
    int start = __shfl(tick, 0);
    if (start > cap - n) start = -1;   /* does not fit: the cell walks the BVH */
    if (on && start >= 0) {   /* dmin: float 6; mask: floats 20-21; rest: 22-23 */
        const uint64_t rr = sk[128 + rank];
        q[1].z = it.dmin;
        q[5].x = __uint_as_float((uint32_t)mask);
        q[5].y = __uint_as_float((uint32_t)(mask >> 32));
        q[5].z = __uint_as_float((uint32_t)rr);
        q[5].w = __uint_as_float((uint32_t)(rr >> 32));
        float4 *dst = reinterpret_cast<float4 *>(region + start + rank);
#pragma unroll
        for (int r = 0; r < 6; ++r) dst[r] = q[r];
    }
    wave_lds_sync();   /* sk is reused by the wave's next cell */
    return start;
}

/* The queued groups' pairs past the first kExpand (bins_pairs), over this
 * kernel's grid; launched only when the scene's sizing pass queued groups
 * (the projection is the scene's fixed camera: every frame queues the same). */
__global__ __launch_bounds__(256) void k_bins_pairs(const BinItem *__restrict__ items,
                                                    const int32_t *__restrict__ tpref,
                                                    const int32_t *__restrict__ gsum, const int32_t *__restrict__ rem,
                                                    int nt, int tx, int32_t *__restrict__ cnt,
                                                    uint64_t *__restrict__ keys, int32_t *__restrict__ nonempty,
                                                    int32_t *__restrict__ bigl, int cap_shard, BinsHdr *__restrict__ hdr2,
                                                    int par, int qmax) {
    bins_pairs(items, tpref, gsum, rem, nt, tx, cnt, keys, nonempty, bigl, cap_shard, hdr2 + par, (int)blockIdx.x,
               (int)gridDim.x, qmax);
}

/* A cell into its work list (BinsPlan): one lane. */
__device__ __forceinline__ void bins_list(const BinsPlan &bp, int kind, int sh, Tile t, int off, int len, int c) {
    const int s2 = atomicAdd(&bp.phdr[bins_phdr_at(bp.par, kind, sh)], 1);
    (void)BCK(s2, bp.ecap, 28);   /* a list holds every cell of its shard */
    if (s2 < bp.ecap) {
        BinsWork w;
        w.t = t;
        w.off = off;
        w.len = len;
        w.cell = c;
        w.pad = 0;
        bp.work[bp.wbase[kind] + sh * bp.ecap + s2] = w;
    }
}

__device__ __forceinline__ int bins_kind(const BinsPlan &bp, int n, int start) {
    return start < 0 ? 3 : n >= bp.split ? 0 : n >= bp.medium ? 1 : 2;
}

/* One cell's list by the whole wave (n > 16 candidates; n <= 64 in one pass,
 * longer ones ranked from LDS); its (offset, length) and work-list entry.
 * c, m, n, k wave-uniform. */
__device__ void bins_sort_wave(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items,
                               const uint64_t *__restrict__ keys, const int32_t *__restrict__ every, int ev,
                               BinsHdr *__restrict__ hdr, CamCand *__restrict__ recs, const BinsCaps &caps,
                               int32_t *__restrict__ bin_off, int32_t *__restrict__ bin_len, int tx,
                               const BinsPlan &bp, int c, int m, int n, int k, uint64_t *sk, int lane) {
    const int sh = c % kBinShards;
    Tile tl{};
    if (k >= 0 && bp.work && lane == 0) tl = bp.tiles[k];   /* in flight with the list's loads */
    int s2 = -1;
    if (n <= kBinCellCap) {
        const uint64_t *own = keys + (size_t)c * kBinCellCap;
        if (n <= 64) {
            const uint64_t kl = own[BCK(lane, kBinCellCap, 12)];
            const int e = __shfl(ev, max(lane - m, 0));
            const uint64_t key = lane < m ? kl : lane < n ? bin_key(0.0f, e) : ~0ull;
            s2 = bins_emit64(tpl, items, key, n, c % tx, c / tx, recs + caps.base[BCK(sh, kBinShards, 24)], caps.cap[sh],
                             &hdr->rec[sh].v, sk, lane);
        } else {
            if (lane == 0) s2 = atomicAdd(&hdr->rec[sh].v, n);
            s2 = __shfl(s2, 0);
            if (s2 > caps.cap[sh] - n) s2 = -1;   /* does not fit: the cell walks the BVH */
            if (s2 >= 0) {
                CamCand *out = recs + caps.base[BCK(sh, kBinShards, 24)] + s2;
                if (n <= 128) bins_emit<2>(tpl, items, own, m, every, n, c % tx, c / tx, out, sk, lane);
                else if (n <= 256) bins_emit<4>(tpl, items, own, m, every, n, c % tx, c / tx, out, sk, lane);
                else bins_emit<kBinCellCap / 64>(tpl, items, own, m, every, n, c % tx, c / tx, out, sk, lane);
            }
        }
    }
    if (lane == 0) {
        bin_off[BCK(c, BDBG(ncell), 26)] = s2 >= 0 ? caps.base[sh] + s2 : 0;
        bin_len[BCK(c, BDBG(ncell), 27)] = s2 >= 0 ? n : -1;
        if (k >= 0 && bp.work)
            bins_list(bp, bins_kind(bp, n, s2), sh, tl, s2 >= 0 ? caps.base[sh] + s2 : 0, s2 >= 0 ? n : -1, c);
    }
}

/* k_bins_sort: the frame's non-empty cells (every cell when some hull is
 * everywhere).  The grid's first long_waves waves take the cells of more than
 * 16 candidates (the scatter's long lists), one a wave; the others take the
 * non-empty lists four cells a wave, 16 lanes each, skipping the long ones
 * (a cell within 16 of its own but over 16 with the everywhere ids is
 * finished by the whole wave after).  A cell's keys (its own from the
 * scatter, then the everywhere ids at dmin 0) are ranked in LDS — each key's
 * rank is the number of smaller keys (keys are distinct: they hold the id) —
 * and each record written at its rank in a range reserved with one atomic:
 * the static part from the triangle's template, dmin from the item, the
 * cell's pixels inside the triangle's rectangle, and `rest` (the OR of the
 * masks from here to the list's end).  Then the cell's (offset, length) and
 * its work-list entry.  Slot i of a list set: shard i % kBinShards, entry
 * i / kBinShards. */
constexpr int kSortSlots = 64 / kSortGroup;   /* cells a wave of the first pass */

#ifndef CRT_SORT_WAVES
#define CRT_SORT_WAVES 1   /* min waves/SIMD asked of k_bins_sort (A/B builds) */
#endif
__global__ __launch_bounds__(64 * kSortWaves) __attribute__((amdgpu_waves_per_eu(CRT_SORT_WAVES))) void k_bins_sort(
    const CamCand *__restrict__ tpl, const BinItem *__restrict__ items, int32_t *__restrict__ cnt,
    const uint64_t *__restrict__ keys, const int32_t *__restrict__ every, const int32_t *__restrict__ nonempty,
    const int32_t *__restrict__ bigl, int cap_shard, int long_waves, BinsHdr *__restrict__ hdr2, int par,
    CamCand *__restrict__ recs, BinsCaps caps, int32_t *__restrict__ bin_off, int32_t *__restrict__ bin_len, int tx,
    int ncell, BinsPlan bp) {
    __shared__ uint64_t sks[kSortWaves][kBinCellCap];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const int l = lane & (kSortGroup - 1), gq = lane / kSortGroup;
    uint64_t *sk = sks[wv];
    uint64_t *gk = sk + 3 * kSortGroup * gq;   /* the group's keys, masks by rank, rest by rank */
    BSTAMP4(0);
    BinsHdr *hdr = hdr2 + par;
    const int wave = (int)blockIdx.x * kSortWaves + wv, nwaves = (int)gridDim.x * kSortWaves;
    /* the everywhere count and ids (lane j: the j-th), the shards' list lengths (lane s: shard s) */
    const int n_every = hdr->n_every.v;
    const int ev = lane < kBinMaxEverywhere ? every[lane] : 0;   /* valid below n_every */
    const int nl = lane < kBinShards ? (wave < long_waves ? hdr->nb[lane].v : hdr->ne[lane].v) : 0;
    const bool all = n_every > 0;   /* everywhere hulls: every cell has a list */
    int mx = nl;   /* the longest shard list, over the whole wave */
    for (int d = 1; d < 64; d <<= 1) mx = max(mx, __shfl_xor(mx, d));
    BSTAMP4(1);
    if (wave < long_waves) {   /* the long lists, one a wave */
        const int nslots = __builtin_amdgcn_readfirstlane(kBinShards * mx);
        for (int i = wave; i < nslots; i += long_waves) {
            const int sh0 = i % kBinShards, e = i / kBinShards;
            if (e >= __shfl(nl, sh0)) continue;
            const int c = __builtin_amdgcn_readfirstlane(bigl[BCK(sh0 * cap_shard + e, BDBG(ne_cap), 14)]);
            const int m = cnt[(size_t)BCK(c, BDBG(ncell), 22) * kCntStride];
            const int k = bp.cell_tile ? bp.cell_tile[BCK(c, BDBG(ncell), 23)] : -2;   /* -1: not rendered */
            const int n = n_every > kBinMaxEverywhere ? kBinCellCap + 1 : m + n_every;
            if (k != -1)
                bins_sort_wave(tpl, items, keys, every, ev, hdr, recs, caps, bin_off, bin_len, tx, bp, c, m, n, k, sk,
                               lane);
        }
        BSTAMP4(4);
        return;
    }
    const int nslots = __builtin_amdgcn_readfirstlane(all ? ncell : kBinShards * mx);   /* wave-uniform: the
                                                       loop body holds the wave's shuffles and LDS hand-offs */
    const int w1 = wave - long_waves, nw1 = nwaves - long_waves;
    for (int base = w1 * kSortSlots; base < nslots; base += nw1 * kSortSlots) {
        const int i = base + gq;
        int c = -1;
        if (i < nslots) {
            if (all) {
                c = i;
            } else {
                const int sh0 = i % kBinShards, e = i / kBinShards;
                if (e < __shfl(nl, sh0)) c = nonempty[BCK(sh0 * cap_shard + e, BDBG(ne_cap), 21)];
            }
        }
        /* the group's cell: its count, tile and first 16 keys in one round of loads */
        const bool cv = c >= 0;
        const int m = cv ? cnt[(size_t)BCK(c, BDBG(ncell), 22) * kCntStride] : 0;
        const int k = !cv ? -1 : bp.cell_tile ? bp.cell_tile[BCK(c, BDBG(ncell), 23)] : -2;   /* -1: not rendered */
        const uint64_t kl = cv ? keys[BCK((size_t)c * kBinCellCap + l, (int64_t)BDBG(ncell) * kBinCellCap, 11)] : ~0ull;
        const int n = n_every > kBinMaxEverywhere ? kBinCellCap + 1 : m + n_every;
        const int sh = cv ? c % kBinShards : 0;
        const bool mine = k != -1 && m <= kSortGroup;   /* longer own lists: the long waves */
        const bool small = mine && n <= kSortGroup;
        /* ---- cells of at most 16 candidates: the group's 16 lanes ---- */
        const bool on = small && l < n;
        int tick = 0;
        if (small && l == 0) tick = atomicAdd(&hdr->rec[sh].v, n);
        const int e2 = __shfl(ev, max(l - m, 0));
        const uint64_t key = !on ? ~0ull : l < m ? kl : bin_key(0.0f, e2);
        const int t = (int)(uint32_t)key;
        Tile tl{};
        if (small && k >= 0 && bp.work) tl = bp.tiles[k];   /* the cell's tile (its list entry) */
        BinItem it{};
        float4 q[6];
        if (on) {   /* in flight with the atomic and the tile during the ranking */
            it = items[BCK(t, BDBG(nt), 19)];
            const float4 *src = reinterpret_cast<const float4 *>(tpl + BCK(t, BDBG(nt), 20));
#pragma unroll
            for (int r = 0; r < 6; ++r) q[r] = load_global(src, r);
        }
        gk[l] = key;
        wave_lds_sync();
        int rank = 0;
#pragma unroll
        for (int j = 0; j < kSortGroup; ++j) rank += gk[j] < key ? 1 : 0;
        const uint64_t mask = on ? bin_mask(it, c % tx, c / tx) : 0ull;
        gk[kSortGroup + (on ? rank : l)] = mask;   /* positions past the list: 0 */
        wave_lds_sync();
        uint64_t rest = gk[kSortGroup + l];
#pragma unroll
        for (int d = 1; d < kSortGroup; d <<= 1) {
            const uint64_t u = shfl_down_u64(rest, d);
            if (l + d < kSortGroup) rest |= u;
        }
        gk[2 * kSortGroup + l] = rest;
        wave_lds_sync();
        int start = __shfl(tick, lane & ~(kSortGroup - 1));
        if (start > caps.cap[sh] - n) start = -1;   /* does not fit: the cell walks the BVH */
        if (on && start >= 0) {   /* dmin: float 6; mask: floats 20-21; rest: 22-23 */
            const uint64_t rr = gk[2 * kSortGroup + rank];
            q[1].z = it.dmin;
            q[5].x = __uint_as_float((uint32_t)mask);
            q[5].y = __uint_as_float((uint32_t)(mask >> 32));
            q[5].z = __uint_as_float((uint32_t)rr);
            q[5].w = __uint_as_float((uint32_t)(rr >> 32));
            float4 *dst = reinterpret_cast<float4 *>(recs + caps.base[BCK(sh, kBinShards, 24)] + start + rank);
#pragma unroll
            for (int r = 0; r < 6; ++r) dst[r] = q[r];
        }
        if (small && l == 0) {
            bin_off[BCK(c, BDBG(ncell), 26)] = start >= 0 ? caps.base[sh] + start : 0;
            bin_len[BCK(c, BDBG(ncell), 27)] = start >= 0 ? n : -1;
            if (k >= 0 && bp.work)
                bins_list(bp, bins_kind(bp, n, start), sh, tl, start >= 0 ? caps.base[sh] + start : 0, start >= 0 ? n : -1, c);
        }
        wave_lds_sync();   /* sk is reused below */
        BSTAMP4(2);
        /* ---- within 16 of its own, over 16 with the everywhere ids: the whole wave ---- */
        uint64_t more = __ballot(l == 0 && mine && !small);
        while (more) {
            const int src = __builtin_ctzll(more);
            more &= more - 1;
            const int c2 = __builtin_amdgcn_readfirstlane(__shfl(c, src));
            bins_sort_wave(tpl, items, keys, every, ev, hdr, recs, caps, bin_off, bin_len, tx, bp, c2,
                           __shfl(m, src), __shfl(n, src), __shfl(k, src), sk, lane);
        }
    }
    BSTAMP4(4);
}

/* empty kernel: its launch at scene creation loads this TU's code object */
__global__ void k_warm_bins() {}

/* ---- host side ---- */

/* The buffers of the current camera view (all but the per-triangle ones);
 * the scene then walks without bins until bins_view builds them again. */
void bins_free_view(crt_hip_scene *sc) {
    BinsDev &b = sc->bins;
    if (b.stream) (void)hipStreamSynchronize(b.stream);
    for (void *p : b.allocs) (void)hipFree(p);
    b.allocs.clear();
    for (int i = 0; i < kBinSets; ++i) {
        if (b.bdone[i]) (void)hipEventDestroy(b.bdone[i]);
        if (b.rdone[i]) (void)hipEventDestroy(b.rdone[i]);
        b.bdone[i] = b.rdone[i] = nullptr;
    }
    if (b.stream) (void)hipStreamDestroy(b.stream);
    b.stream = nullptr;
    b.cam = BinCamera{};
    b.tx = b.ncell = b.cap_shard = b.long_waves = b.sort_blocks = b.pair_blocks = 0;
    b.cnt = nullptr;
    b.keys = nullptr;
    b.every = b.nonempty = b.bigl = nullptr;
    b.hdr = nullptr;
    b.frame = 0;
    b.last = -1;
    b.binned_plan = nullptr;
    b.caps = BinsCaps{};
    b.recs = nullptr;
    b.rec_cap = 0;
    b.off = b.len = nullptr;
    b.count.clear();
    b.records = 0;
    sc->ds.bins = nullptr;
    sc->ds.bin_off = nullptr;
    sc->ds.bin_len = nullptr;
    sc->ds.bin_tx = 0;
}

void bins_free(crt_hip_scene *sc) {
    bins_free_view(sc);
    BinsDev &b = sc->bins;
    for (void *p : b.keep) (void)hipFree(p);
    b = BinsDev{};
}

namespace {

template <class T>
int bins_alloc(crt_hip_scene *sc, T **p, size_t n, bool zero = false, bool keep = false) {
    void *q = nullptr;
    HIP_TRY(hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T)));
    (keep ? sc->bins.keep : sc->bins.allocs).push_back(q);
    if (zero) HIP_TRY(hipMemset(q, 0, std::max<size_t>(1, n) * sizeof(T)));
    sc->info.device_bytes += (int64_t)(n * sizeof(T));
    *p = static_cast<T *>(q);
    return CRT_OK;
}

int launch_project(crt_hip_scene *sc, hipStream_t s, int par, int32_t *phdr) {
    BinsDev &b = sc->bins;
    const int groups = (b.nt + kProjTris - 1) / kProjTris;
    hipLaunchKernelGGL(k_bins_project, dim3((unsigned)groups), dim3(256), 0, s, b.tpl, b.nt, b.cam, b.items, b.tpref,
                       b.gsum, b.every, b.hdr, par, phdr, b.len + (size_t)par * b.ncell, b.ncell, b.tx, b.cnt, b.keys,
                       b.nonempty, b.bigl,
                       b.cap_shard, b.rem, b.pair_blocks > 0 ? b.qmax : 0);
    HIP_TRY(hipGetLastError());
    if (b.pair_blocks > 0) {
        hipLaunchKernelGGL(k_bins_pairs, dim3((unsigned)b.pair_blocks), dim3(256), 0, s, b.items, b.tpref, b.gsum,
                           b.rem, b.nt, b.tx, b.cnt + (size_t)par * b.ncell * kCntStride, b.keys, b.nonempty, b.bigl,
                           b.cap_shard, b.hdr, par, b.qmax);
        HIP_TRY(hipGetLastError());
    }
    return CRT_OK;
}

}  // namespace

/* diagnostic builds (CRT_BINS_CHECK): report a violation of the last frame
 * and arm the checks with this frame's buffer sizes */
int bins_dbg_arm(crt_hip_scene *sc, const ShardPlan &plan) {
#ifdef CRT_BINS_CHECK
    BinsDev &b = sc->bins;
    BinsDbg d{};
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(&d, HIP_SYMBOL(g_bins_dbg), sizeof d));
    if (d.code)
        return set_error(CRT_E_STATE, "bins check: code " + std::to_string(d.code) + " index " + std::to_string(d.idx) +
                                          " bound " + std::to_string(d.bound));
    d.nt = b.nt;
    d.ncell = b.ncell;
    d.rec_cap = kBinSets * b.rec_cap;
    d.ne_cap = kBinShards * b.cap_shard;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_bins_dbg), &d, sizeof d));
#else
    (void)sc;
    (void)plan;
#endif
    return CRT_OK;
}

/* Scene create: the per-triangle templates and the buffers, sized by one
 * projection pass of this camera (its counts are read back; the lists are
 * rebuilt by every frame).  Leaves sc->ds.bins null when the scene takes no
 * bins. */
int bins_setup(crt_hip_scene *sc, const HostScene &hs) {
    BinsDev &b = sc->bins;
    if (hs.tri_attr.empty()) return CRT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    /* per triangle, kept for every view: the records' static parts and the
     * projection's scratch */
    b.nt = (int)hs.tri_attr.size();
    b.qmax = kMaxGroups;   /* tests lower it (option "bins_qmax"): the groups past it scatter their own pairs */
    std::vector<CamCand> tpl;
    bin_templates(hs, tpl);
    int rc;
    if ((rc = bins_alloc(sc, &b.tpl, tpl.size(), false, true)) != CRT_OK) return rc;
    HIP_TRY(hipMemcpy(b.tpl, tpl.data(), tpl.size() * sizeof(CamCand), hipMemcpyHostToDevice));
    if ((rc = bins_alloc(sc, &b.items, (size_t)b.nt, false, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.tpref, (size_t)((b.nt + kProjTris - 1) / kProjTris) * kProjTris, false, true)) != CRT_OK)
        return rc;
    if ((rc = bins_alloc(sc, &b.gsum, (size_t)((b.nt + kProjTris - 1) / kProjTris), false, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.rem, (size_t)((b.nt + kProjTris - 1) / kProjTris), false, true)) != CRT_OK) return rc;
    rc = bins_view(sc);
    b.setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

/* The buffers of the scene's current camera and resolution (sc->ds.cam),
 * sized by one projection pass of that camera; leaves sc->ds.bins null when
 * this view takes no bins (bin_camera_of fails: the camera outside the hull
 * margins' origin bound, a singular rotation; or the lists would be too long). */
int bins_view(crt_hip_scene *sc) {
    BinsDev &b = sc->bins;
    if (!b.tpl) return CRT_OK;
    BinCamera cam;
    if (!bin_camera_of(sc->ds.cam, sc->prune_origin_max, cam)) return CRT_OK;
    b.cam = cam;
    b.tx = cam.tx;
    b.ncell = cam.tx * cam.ty;
    b.cap_shard = (b.ncell + kBinShards - 1) / kBinShards;
    int rc;
    b.pair_blocks = 0;   /* the sizing pass: every group counts its own pairs */
    if ((rc = bins_alloc(sc, &b.cnt, (size_t)kBinSets * b.ncell * kCntStride, true)) != CRT_OK) return rc;   /* per set */
    if ((rc = bins_alloc(sc, &b.every, (size_t)kBinMaxEverywhere)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.hdr, kBinSets, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.off, (size_t)kBinSets * b.ncell, true)) != CRT_OK) return rc;   /* per set */
    if ((rc = bins_alloc(sc, &b.len, (size_t)kBinSets * b.ncell, true)) != CRT_OK) return rc;
    /* sizing pass: counts per cell of this camera (the projection without
     * keys: nothing is scattered, and a view the counts reject never
     * allocates its ~0.5 GB of 4K keys — C5: 80 ms of a create) */
    b.keys = nullptr;
    b.nonempty = b.bigl = nullptr;
    if ((rc = bins_dbg_arm(sc, ShardPlan{})) != CRT_OK) return rc;
    if ((rc = launch_project(sc, sc->stream, 0, nullptr)) != CRT_OK) return rc;
    std::vector<int32_t> cnt((size_t)b.ncell * kCntStride), gsum((size_t)((b.nt + kProjTris - 1) / kProjTris));
    BinsHdr h;
    HIP_TRY(hipMemcpyAsync(cnt.data(), b.cnt, cnt.size() * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(gsum.data(), b.gsum, gsum.size() * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(&h, b.hdr, sizeof h, hipMemcpyDeviceToHost, sc->stream));
    const int n_every = h.n_every.v;
    HIP_TRY(hipStreamSynchronize(sc->stream));
    HIP_TRY(hipMemsetAsync(b.cnt, 0, kBinSets * cnt.size() * sizeof(int32_t), sc->stream));
    HIP_TRY(hipMemsetAsync(b.hdr, 0, kBinSets * sizeof(BinsHdr), sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    b.frame = 0;
    b.last = -1;
    b.count.assign((size_t)b.ncell, 0);
    int64_t queued = 0;   /* pairs past the first kExpand of their group */
    for (const int32_t g : gsum) queued += std::max(0, g - kExpand);
    b.pair_blocks = queued ? (int)std::max<int64_t>(8, std::min<int64_t>(2048, (queued + CRT_PAIRS_PER_BLOCK - 1) / CRT_PAIRS_PER_BLOCK)) : 0;
    int64_t total = 0, shard_rec[kBinShards] = {0}, shard_listed[kBinShards] = {0}, shard_long[kBinShards] = {0};
    for (int c = 0; c < b.ncell; ++c) {
        const int64_t n = (int64_t)cnt[(size_t)c * kCntStride] + n_every;
        if (n > kBinCellCap || n_every > kBinMaxEverywhere) {
            b.count[(size_t)c] = -1;
        } else {
            b.count[(size_t)c] = (int32_t)n;
            total += n;
            shard_rec[c % kBinShards] += n;
        }
        shard_listed[c % kBinShards] += cnt[(size_t)c * kCntStride] > 0;
        shard_long[c % kBinShards] += cnt[(size_t)c * kCntStride] > kSortGroup;
    }
    bool over = false;   /* some cell over the cap: it walks the BVH */
    for (int c = 0; c < b.ncell; ++c) over = over || b.count[(size_t)c] < 0;
    if (n_every > kBinMaxEverywhere || total > sc->bins_mean_cap * b.ncell || total >= INT32_MAX / 4 ||
        (over && !sc->ds.bnodes)) {
        bins_free_view(sc);   /* the scene walks the BVH (or the kd tree) */
        return CRT_OK;
    }
    if ((rc = bins_alloc(sc, &b.keys, (size_t)b.ncell * kBinCellCap)) != CRT_OK) return rc;   /* 64-bit keys */
    if ((rc = bins_alloc(sc, &b.nonempty, (size_t)kBinShards * b.cap_shard)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.bigl, (size_t)kBinShards * b.cap_shard)) != CRT_OK) return rc;
    /* each shard's records in a region of its own, sized from the pass with
     * room for a camera that moves (crt_hip_scene_set_camera): a cell whose
     * list does not fit walks the BVH */
    int64_t base = 0;
    for (int s2 = 0; s2 < kBinShards; ++s2) {
        const int64_t cap = 2 * shard_rec[s2] + 1024;
        b.caps.base[s2] = (int32_t)base;
        b.caps.cap[s2] = (int32_t)cap;
        base += cap;
    }
    b.rec_cap = (int32_t)base;
    if ((int64_t)kBinSets * base >= INT32_MAX) {   /* record offsets are int32 */
        bins_free_view(sc);
        return CRT_OK;
    }
    if ((rc = bins_alloc(sc, &b.recs, (size_t)kBinSets * b.rec_cap)) != CRT_OK) return rc;   /* per set */
    /* the frames pipeline: the binning's stream and the sets' events
     * (recorded once, so the first frames find their lists free) */
    HIP_TRY(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking));
    for (int i = 0; i < kBinSets; ++i) {
        HIP_TRY(hipEventCreateWithFlags(&b.bdone[i], CRT_PIPE_EV_FLAGS));
        HIP_TRY(hipEventCreateWithFlags(&b.rdone[i], CRT_PIPE_EV_FLAGS));
        HIP_TRY(hipEventRecord(b.rdone[i], sc->stream));
        HIP_TRY(hipEventRecord(b.bdone[i], sc->stream));
        b.rdone_s[i] = b.bdone_s[i] = sc->stream;
    }
    /* k_bins_sort's grid: a wave per long list (at least kBinShards waves),
     * then the listed cells (every cell when some hull is everywhere),
     * kSortSlots a wave */
    const int64_t most = *std::max_element(shard_listed, shard_listed + kBinShards);
    const int64_t most_long = *std::max_element(shard_long, shard_long + kBinShards);
    const int64_t slots = n_every > 0 ? b.ncell : kBinShards * most;
    b.long_waves = (int)std::max<int64_t>(kBinShards, kBinShards * most_long);
    const int64_t waves = b.long_waves + (slots + kSortSlots - 1) / kSortSlots;
    b.sort_blocks = (int)((waves + kSortWaves - 1) / kSortWaves);
    b.records = total;
    sc->ds.bins = b.recs;
    sc->ds.bin_off = b.off;
    sc->ds.bin_len = b.len;
    sc->ds.bin_tx = b.tx;
    return CRT_OK;
}

/* A plan's camera-bins dispatch (BinsPlan): the work lists' capacities from
 * the sizing pass's counts (per kind, the fullest shard), the cells the plan
 * renders as one tile each, and the `rest` tiles. */
int bins_plan(crt_hip_scene *sc, ShardPlan &plan) {
    BinsDev &b = sc->bins;
    const int nb = plan.ntiles;
    std::vector<int32_t> cell_tile((size_t)b.ncell, -1);
    std::vector<uint8_t> inside((size_t)nb, 0);
    for (int k = 0; k < nb; ++k) {
        const Tile &t = plan.tiles[(size_t)k];
        if ((t.x & 7) + t.w > 8 || (t.y & 7) + t.h > 8) continue;   /* not inside one cell: BVH walk */
        inside[(size_t)k] = 1;
        int32_t &e = cell_tile[(size_t)(t.y >> 3) * b.tx + (t.x >> 3)];
        e = e == -1 ? k : -2;   /* several tiles in one cell: each reads the cell's list */
    }
    BinsPlan &bp = plan.bp;
    bp = BinsPlan{};
    bp.split = sc->bins_split;
    bp.medium = kBinsMedium;
    bp.quad = sc->bins_quad;
    int per[kBinKinds][kBinShards] = {};
    for (int c = 0; c < b.ncell; ++c) {
        if (cell_tile[(size_t)c] < 0) continue;
        const int n = b.count[(size_t)c];
        if (n == 0) continue;   /* the background: a fill wave */
        ++per[n < 0 ? 3 : n >= bp.split ? 0 : n >= bp.medium ? 1 : 2][c % kBinShards];
    }
    std::vector<int32_t> rest;
    for (int k = 0; k < nb; ++k) {
        const Tile &t = plan.tiles[(size_t)k];
        if (!inside[(size_t)k] && !sc->ds.bnodes) return CRT_OK;   /* no BVH for it: not a bins plan (the kd walk) */
        if (!inside[(size_t)k] || cell_tile[(size_t)(t.y >> 3) * b.tx + (t.x >> 3)] == -2) rest.push_back(k);
    }
    /* the lists hold every cell of a shard (a moved camera may list any cell
     * of any kind); the grid takes the sizing pass's counts plus bins_slack %
     * (a moved camera's extra cells of a kind: slots beyond take several
     * entries), at least one slot per shard and kind */
    bp.ecap = b.cap_shard;
    int64_t slots = 0;
    for (int q = 0; q < kBinKinds; ++q) {
        const int64_t most = *std::max_element(per[q], per[q] + kBinShards);
        bp.gcap[q] = (int32_t)std::min<int64_t>(b.cap_shard, std::max<int64_t>(1, most + (most * sc->bins_slack + 99) / 100));
        bp.wbase[q] = (int32_t)slots;
        slots += (int64_t)kBinShards * bp.ecap;
    }
    bp.nrest = (int32_t)rest.size();
    bp.ncell = b.ncell;
    bp.nfill = (b.ncell + 15) / 16;   /* 16 cells a fill wave */
    void *p[4] = {nullptr, nullptr, nullptr, nullptr};
    bp.wslots = (int32_t)slots;
    const size_t sizes[4] = {(size_t)b.ncell * sizeof(int32_t), (size_t)std::max<int64_t>(1, kBinSets * slots) * sizeof(BinsWork),
                             (size_t)kBinsPhdrInts * sizeof(int32_t), std::max<size_t>(1, rest.size()) * sizeof(int32_t)};
    for (int i = 0; i < 4; ++i) {
        HIP_TRY(hipMalloc(&p[i], sizes[i]));
        sc->plan_allocs.push_back(p[i]);
        HIP_TRY(hipMemset(p[i], 0, sizes[i]));
    }
    HIP_TRY(hipMemcpy(p[0], cell_tile.data(), sizes[0], hipMemcpyHostToDevice));
    if (!rest.empty()) HIP_TRY(hipMemcpy(p[3], rest.data(), rest.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    bp.cell_tile = static_cast<int32_t *>(p[0]);
    bp.tiles = plan.d_tiles;
    bp.work = static_cast<BinsWork *>(p[1]);
    bp.phdr = static_cast<int32_t *>(p[2]);
    bp.rest = static_cast<int32_t *>(p[3]);
    plan.waves = 4 * kBinShards * bp.gcap[0] + kBinShards * (bp.gcap[1] + bp.gcap[2] + bp.gcap[3]) + bp.nrest + bp.nfill;
    return CRT_OK;
}

/* The frame's lists, before its render on `s`; returns the frame's set
 * (the render reads that set of lists and records rdone[set] after it).
 * While the previous frame still renders (frames issued back to back), the
 * binning runs on the binning's own stream — after the render kBinSets frames
 * back (same set) is done with the set and after the previous binning — and
 * `s` waits for it: the next frames' binnings overlap frame k's render.
 * Otherwise (one frame at a time) `s` takes the binning itself, after the
 * same two events.  A frame with the camera and plan of the last binning
 * (bins_reuse, not `force`) takes that binning's set as it is: `s` only
 * waits for the binning if it ran elsewhere. */
int bins_enqueue(crt_hip_scene *sc, const ShardPlan &plan, hipStream_t s, int *par_out, bool force) {
    BinsDev &b = sc->bins;
#ifdef CRT_BINS_TRACE   /* diagnostic builds (BINS_FLAGS=-DCRT_BINS_TRACE): each decision on stderr */
    if (true)
#else
    if (false)
#endif
        std::fprintf(stderr, "bins_enqueue plan=%p work=%p waves=%d last=%d binned=%p frame=%llu force=%d cam_same=%d\n",
                     (const void *)&plan, (const void *)plan.bp.work, plan.waves, b.last, b.binned_plan,
                     (unsigned long long)b.frame, (int)force, (int)(std::memcmp(&b.binned, &b.cam, sizeof b.cam) == 0));
    if (!force && sc->bins_reuse && b.last >= 0 && b.binned_plan == plan.bp.work && plan.bp.work &&
        std::memcmp(&b.binned, &b.cam, sizeof b.cam) == 0) {
        const int par = b.last;
        if (b.bdone_s[par] != s && hipEventQuery(b.bdone[par]) != hipSuccess)
            HIP_TRY(hipStreamWaitEvent(s, b.bdone[par], 0));
        ++b.reuses;
        if (par_out) *par_out = par;
        return CRT_OK;
    }
    const int par = (int)(b.frame++ % kBinSets);
    const int prev = (par + kBinSets - 1) % kBinSets;
    {
        const int rc0 = bins_dbg_arm(sc, plan);
        if (rc0 != CRT_OK) return rc0;
    }
    /* the previous frame still renders: overlap it.  Wherever the binning
     * runs, it waits for the render kBinSets frames back (same set of lists)
     * and for the previous binning (the binnings share their scratch: items,
     * keys, counts, lists) — whichever streams those ran on, so a caller that
     * issues frames on different streams cannot reopen a scratch race; a wait
     * on an event already reached on the same stream costs nothing */
    const bool overlap = hipEventQuery(b.rdone[prev]) == hipErrorNotReady;
    const hipStream_t bs = overlap ? b.stream : s;
    auto after = [&](hipEvent_t e, hipStream_t es) -> hipError_t {   /* (implied on its own stream, or done) */
        return es == bs || hipEventQuery(e) == hipSuccess ? hipSuccess : hipStreamWaitEvent(bs, e, 0);
    };
    HIP_TRY(after(b.rdone[par], b.rdone_s[par]));
    HIP_TRY(after(b.bdone[prev], b.bdone_s[prev]));
    int rc = launch_project(sc, bs, par, plan.bp.phdr);
    if (rc != CRT_OK) return rc;
    BinsPlan bp = plan.bp;
    bp.par = par;
    if (bp.work) bp.work += (size_t)par * bp.wslots;
    BinsCaps caps = b.caps;   /* this set's part of the record buffer */
    for (int i = 0; i < kBinShards; ++i) caps.base[i] += par * b.rec_cap;
    hipLaunchKernelGGL(k_bins_sort, dim3((unsigned)b.sort_blocks), dim3(64 * kSortWaves), 0, bs, b.tpl, b.items,
                       b.cnt + (size_t)par * b.ncell * kCntStride,
                       b.keys, b.every, b.nonempty, b.bigl, b.cap_shard, b.long_waves, b.hdr, par, b.recs, caps,
                       b.off + (size_t)par * b.ncell, b.len + (size_t)par * b.ncell, b.tx, b.ncell, bp);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(b.bdone[par], bs));
    b.bdone_s[par] = bs;
#ifdef CRT_BINS_CHECK
    {   /* diagnostic builds: this binning's violations before its render runs,
         * and the render's inputs read back and checked on the host */
        const int rc1 = bins_dbg_arm(sc, plan);
        if (rc1 != CRT_OK) return rc1;
        if (plan.bp.work) {
            const BinsPlan &q = plan.bp;
            std::vector<int32_t> ph((size_t)kBinsPhdrInts), ln((size_t)b.ncell), of((size_t)b.ncell);
            std::vector<BinsWork> wk((size_t)q.wslots);
            HIP_TRY(hipMemcpy(ph.data(), q.phdr, ph.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(wk.data(), q.work + (size_t)par * q.wslots, wk.size() * sizeof(BinsWork),
                              hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(ln.data(), b.len + (size_t)par * b.ncell, ln.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(of.data(), b.off + (size_t)par * b.ncell, of.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
            int bad = 0;
            const int64_t rtot = (int64_t)kBinSets * b.rec_cap;
            for (int k2 = 0; k2 < kBinKinds; ++k2)
                for (int s3 = 0; s3 < kBinShards; ++s3) {
                    const int n = std::min(ph[(size_t)bins_phdr_at(par, k2, s3)], q.ecap);
                    for (int i = 0; i < n; ++i) {
                        const BinsWork &w = wk[(size_t)q.wbase[k2] + (size_t)s3 * q.ecap + i];
                        bool ok = w.cell >= 0 && w.cell < b.ncell && w.len >= -1 && w.len <= kBinCellCap &&
                                  (w.len < 0 || (w.off >= 0 && (int64_t)w.off + w.len <= rtot));
                        bool found = false;
                        for (const Tile &t : plan.tiles)
                            if (std::memcmp(&t, &w.t, sizeof t) == 0) found = true;
                        if ((!ok || !found) && bad++ < 8)
                            std::fprintf(stderr, "bins check: kind %d shard %d entry %d cell %d off %d len %d tile (%d %d %d %d) %s\n",
                                         k2, s3, i, w.cell, w.off, w.len, w.t.x, w.t.y, w.t.w, w.t.h,
                                         found ? "" : "NOT A PLAN TILE");
                    }
                }
            for (int c = 0; c < b.ncell; ++c)
                if (ln[(size_t)c] > 0 && (of[(size_t)c] < 0 || (int64_t)of[(size_t)c] + ln[(size_t)c] > rtot) && bad++ < 16)
                    std::fprintf(stderr, "bins check: cell %d off %d len %d\n", c, of[(size_t)c], ln[(size_t)c]);
            std::fprintf(stderr, "bins check: plan %p set %d: %d bad\n", (const void *)&plan, par, bad);
            if (bad) return set_error(CRT_E_STATE, "bins check: bad render inputs");
            if (const char *e = std::getenv("CRT_BINS_NORENDER"))   /* from this binning on: no render */
                if ((long long)b.frame - 1 >= std::atoll(e)) return set_error(CRT_E_STATE, "bins check: render skipped");
        }
    }
#endif
    if (overlap) HIP_TRY(hipStreamWaitEvent(s, b.bdone[par], 0));
    b.last = par;
    b.binned = b.cam;
    b.binned_plan = plan.bp.work;
    ++b.binnings;
    if (par_out) *par_out = par;
#ifdef CRT_BINS_STAMPS
    if (const char *fn = std::getenv("CRT_BINS_STAMPS_FILE")) {
        static int dumped = 0;
        if (++dumped == 20) {   /* one warm frame */
            HIP_TRY(hipStreamSynchronize(s));
            const int nb = (b.nt + kProjTris - 1) / kProjTris;
            std::vector<unsigned long long> st((size_t)nb * 4);
            HIP_TRY(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_bins_stamps), st.size() * sizeof(unsigned long long)));
            if (FILE *f = std::fopen(fn, "w")) {
                for (int i = 0; i < nb; ++i)
                    std::fprintf(f, "%llu %llu %llu %llu\n", st[4 * i], st[4 * i + 1], st[4 * i + 2], st[4 * i + 3]);
                std::fclose(f);
            }
            const int ns = std::min(b.sort_blocks, 16384);
            std::vector<unsigned long long> s4((size_t)ns * 6);
            HIP_TRY(hipMemcpyFromSymbol(s4.data(), HIP_SYMBOL(g_bins_stamps4), s4.size() * sizeof(unsigned long long)));
            if (FILE *f = std::fopen((std::string(fn) + ".sort").c_str(), "w")) {
                for (int i = 0; i < ns; ++i)
                    std::fprintf(f, "%llu %llu %llu %llu %llu %llu\n", s4[6 * i], s4[6 * i + 1], s4[6 * i + 2],
                                 s4[6 * i + 3], s4[6 * i + 4], s4[6 * i + 5]);
                std::fclose(f);
            }
        }
    }
#endif
    return CRT_OK;
}

}  // namespace crt_amd

extern "C" {

int64_t crt_hip_camera_bins(crt_hip_scene *sc, int32_t *len_out, void *recs_out, int64_t cap) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    BinsDev &b = sc->bins;
    const int ncell = ((sc->info.width + 7) / 8) * ((sc->info.height + 7) / 8);
    if (!sc->ds.bins) {
        if (len_out) std::memset(len_out, 0, (size_t)ncell * sizeof(int32_t));
        return 0;
    }
    HIP_TRY(hipStreamSynchronize(sc->stream));
    ShardPlan none;   /* no tile plan: every cell's list */
    int rc = bins_enqueue(sc, none, sc->stream, nullptr, true);
    if (rc != CRT_OK) return rc;
    if ((rc = bins_dbg_arm(sc, none)) != CRT_OK) return rc;   /* diagnostic builds: this frame's violations */
    const int par = (int)((b.frame - 1) % kBinSets);   /* the set that frame used */
    std::vector<int32_t> off((size_t)b.ncell), len((size_t)b.ncell);
    std::vector<CamCand> recs((size_t)kBinSets * b.rec_cap);   /* every set's region (offsets are absolute) */
    HIP_TRY(hipMemcpyAsync(off.data(), b.off + (size_t)par * b.ncell, off.size() * sizeof(int32_t),
                           hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(len.data(), b.len + (size_t)par * b.ncell, len.size() * sizeof(int32_t),
                           hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(recs.data(), b.recs, recs.size() * sizeof(CamCand), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    int64_t total = 0;
    for (int c = 0; c < b.ncell; ++c) total += std::max(0, len[(size_t)c]);
    if (len_out) std::memcpy(len_out, len.data(), len.size() * sizeof(int32_t));
    if (!recs_out) return total;
    if (cap < total) return set_error(CRT_E_INVALID, "record buffer too small");
    CamCand *o = static_cast<CamCand *>(recs_out);
    for (int c = 0; c < b.ncell; ++c)
        for (int j = 0; j < len[(size_t)c]; ++j) *o++ = recs[(size_t)off[(size_t)c] + j];
    return total;
}

int crt_hip_bins_time(crt_hip_scene *sc, int32_t frames, double *ms) {
    if (!sc || !ms || frames < 1) return set_error(CRT_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(sc->device));
    *ms = 0.0;
    if (!sc->ds.bins || !sc->full.bp.cell_tile) return CRT_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    int rc = CRT_OK;
    for (int w = 0; w < 3 && rc == CRT_OK; ++w) rc = bins_enqueue(sc, sc->full, sc->stream, nullptr, true);   /* warm */
    hipError_t e = rc == CRT_OK ? hipEventRecord(e0, sc->stream) : hipSuccess;
    for (int f = 0; f < frames && rc == CRT_OK && e == hipSuccess; ++f)
        rc = bins_enqueue(sc, sc->full, sc->stream, nullptr, true);
    if (rc == CRT_OK && e == hipSuccess) e = hipEventRecord(e1, sc->stream);
    if (rc == CRT_OK && e == hipSuccess) e = hipEventSynchronize(e1);
    float f = 0.f;
    if (rc == CRT_OK && e == hipSuccess) e = hipEventElapsedTime(&f, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != CRT_OK) return rc;
    if (e != hipSuccess) return set_error(CRT_E_HIP, hipGetErrorString(e));
    *ms = (double)f / frames;
    return CRT_OK;
}

int64_t crt_host_camera_bins(const crt_host_scene *h, int32_t *len_out, void *recs_out, int64_t cap) {
    if (!h) return set_error(CRT_E_INVALID, "null argument");
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;
    const int rc = build_camera_bins(hs, bins, off, &over);
    if (rc != CRT_OK) return rc;
    const int ncell = ((hs.width + 7) / 8) * ((hs.height + 7) / 8);
    if (len_out) {
        for (int c = 0; c < ncell; ++c)
            len_out[c] = off.empty() ? 0 : over[(size_t)c] ? -1 : off[(size_t)c + 1] - off[(size_t)c];
    }
    if (!recs_out) return (int64_t)bins.size();
    if (cap < (int64_t)bins.size()) return set_error(CRT_E_INVALID, "record buffer too small");
    if (!bins.empty()) std::memcpy(recs_out, bins.data(), bins.size() * sizeof(CamCand));
    return (int64_t)bins.size();
}

}  // extern "C"
