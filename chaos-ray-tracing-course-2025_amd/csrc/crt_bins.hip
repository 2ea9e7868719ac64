/*
 * crt_bins.hip — camera bins built on the device inside every camera frame
 * (crt_bins.h; walked by crt_walks.h trace_bins_wave / trace_bins_lanes).
 *
 * The reference traces every camera ray through its tree inside the timed
 * render_image call (crt_renderer.cpp:147-155, timed at main.cpp:37-39); the
 * lists that let a camera ray test only the triangles its 8x8 cell can hit
 * depend on the camera and the resolution, so they are rebuilt by every frame
 * that walks them, before its render kernel, in two launches:
 *
 *   k_bins_project  one thread per triangle: its hull's projection (bin_project:
 *                   pixel rectangle, dmin, everywhere); then every (triangle,
 *                   cell) pair of the block's 64 triangles, spread over the
 *                   block's 256 threads, takes a slot of its cell (atomic
 *                   count) and writes the triangle id there (kBinCellCap slots
 *                   per cell); the first pair of a cell appends the cell to the
 *                   frame's non-empty list.  Also clears the per-cell list
 *                   lengths and the tile plan's per-frame state.
 *   k_bins_sort     one wave per non-empty cell (every cell when some hull is
 *                   everywhere): its ids plus the everywhere ids, sorted by
 *                   (dmin, id) (bitonic, registers up to 64, LDS up to the cap),
 *                   written as CamCand records (static part from the per-triangle
 *                   template, dmin, the cell's pixel mask, and `rest`, the OR of
 *                   the masks from here to the list's end) into a range reserved
 *                   with one atomic; the cell's (offset, length); and the tile
 *                   plan's priority lists: a cell with bins_split or more
 *                   candidates is queued for four 4x4 waves, one with
 *                   kBinsMedium or more for an early 8x8 wave (the render's
 *                   other waves walk the remaining cells in frame order).
 *
 * The lists equal the host checker's (crt_bvh_build.cpp build_camera_bins)
 * record for record (tests/test_gpu_bins.py); the records of different cells
 * sit in the buffer in no particular order (each cell's range is reserved by
 * an atomic), which no reader depends on.  Scene create runs k_bins_project
 * once to size the buffers (records, priority slots) and to decide whether the
 * scene takes bins at all (crt_bins.h caps); a frame whose lists would not fit
 * renders the cells that do not fit on the BVH walk — the same image.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "crt_bins.h"
#include "crt_scene_impl.h"

namespace crt_amd {

namespace {

constexpr int kProjTris = 64;     /* triangles per k_bins_project block (256 threads) */

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t v, int d) {
    const int lo = __shfl_down((int)(uint32_t)v, d), hi = __shfl_down((int)(uint32_t)(v >> 32), d);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
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

__global__ __launch_bounds__(256) void k_bins_project(const CamCand *__restrict__ tpl, int nt, BinCamera cam,
                                                      BinItem *__restrict__ items, int32_t *__restrict__ cnt,
                                                      int32_t *__restrict__ keys, int32_t *__restrict__ every,
                                                      int32_t *__restrict__ nonempty, BinsHdr *__restrict__ hdr,
                                                      int32_t *__restrict__ bin_len, int ncell,
                                                      int32_t *__restrict__ taken, int ntaken,
                                                      int32_t *__restrict__ phdr) {
    __shared__ int32_t pref[kProjTris + 1];
    __shared__ int32_t cw[kProjTris], cx0[kProjTris], cy0[kProjTris];
    const int tid = (int)threadIdx.x;
    /* this frame's per-cell lengths and plan state start empty (k_bins_sort fills them) */
    const int g = (int)(blockIdx.x * blockDim.x) + tid, gn = (int)(gridDim.x * blockDim.x);
    for (int i = g; i < ncell; i += gn) bin_len[i] = 0;
    for (int i = g; i < ntaken; i += gn) taken[i] = 0;
    if (g == 0 && phdr) {
        phdr[0] = 0;
        phdr[1] = 0;
    }
    if (tid < kProjTris) {   /* wave 0: one triangle per lane */
        const int t = (int)blockIdx.x * kProjTris + tid;
        int np = 0;
        if (t < nt) {
            const float *b = reinterpret_cast<const float *>(tpl + t);   /* lo_x, hi_x, lo_y, hi_y, lo_z, hi_z */
            const float lo[3] = {b[0], b[2], b[4]}, hi[3] = {b[1], b[3], b[5]};
            const BinItem it = bin_project(lo, hi, cam);
            items[t] = it;
            if (it.every) {
                const int k = atomicAdd(&hdr->n_every, 1);
                if (k < kBinMaxEverywhere) every[k] = t;
            } else if (it.px0 <= it.px1) {
                const int x0 = it.px0 >> 3, x1 = it.px1 >> 3, y0 = it.py0 >> 3, y1 = it.py1 >> 3;
                np = (x1 - x0 + 1) * (y1 - y0 + 1);
                cw[tid] = x1 - x0 + 1;
                cx0[tid] = x0;
                cy0[tid] = y0;
            }
        }
        int incl = np;
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (tid >= d) incl += v;
        }
        pref[tid] = incl - np;
        if (tid == 63) pref[kProjTris] = incl;
    }
    __syncthreads();
    const int total = pref[kProjTris];
    for (int p = tid; p < total; p += (int)blockDim.x) {
        int lo = 0, hi = kProjTris - 1;   /* the last triangle whose pairs start at or before p */
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pref[mid] <= p) lo = mid;
            else hi = mid - 1;
        }
        const int j = p - pref[lo], w = cw[lo];
        const int cell = (cy0[lo] + j / w) * cam.tx + cx0[lo] + j % w;
        const int slot = atomicAdd(&cnt[cell], 1);
        if (slot == 0) nonempty[atomicAdd(&hdr->n_nonempty, 1)] = cell;
        if (slot < kBinCellCap) keys[(size_t)cell * kBinCellCap + slot] = (int)blockIdx.x * kProjTris + lo;
    }
}

/* One cell's list: n candidates (m own ids in keys, then the everywhere ids),
 * sorted, written from `start`.  n <= 64: one candidate per lane in registers. */
__device__ void bins_emit_small(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items,
                                const int32_t *__restrict__ ids, int m, const int32_t *__restrict__ every, int n,
                                int cx, int cy, CamCand *__restrict__ out, int lane) {
    uint64_t key = ~0ull;
    if (lane < n) {
        const int t = lane < m ? ids[lane] : every[lane - m];
        key = bin_key(items[t].dmin, t);
    }
    key = wave_sort(key, lane);
    uint64_t mask = 0ull;
    int t = 0;
    BinItem it{};
    if (lane < n) {
        t = (int)(uint32_t)key;
        it = items[t];
        mask = bin_mask(it, cx, cy);
    }
    const uint64_t rest = wave_suffix_or(mask, lane);
    if (lane < n) {
        CamCand c = tpl[t];
        c.dmin = it.dmin;
        c.mask = mask;
        c.rest = rest;
        out[lane] = c;
    }
}

/* n in (64, kBinCellCap]: bitonic sort in LDS (sk, padded to a power of two),
 * then the records written chunk by chunk from the list's end (rest carried). */
__device__ void bins_emit_large(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items,
                                const int32_t *__restrict__ ids, int m, const int32_t *__restrict__ every, int n,
                                int cx, int cy, CamCand *__restrict__ out, uint64_t *sk, int lane) {
    int P = 128;
    while (P < n) P <<= 1;
    for (int j = lane; j < P; j += 64) {
        uint64_t key = ~0ull;
        if (j < n) {
            const int t = j < m ? ids[j] : every[j - m];
            key = bin_key(items[t].dmin, t);
        }
        sk[j] = key;
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = lane; i < (P >> 1); i += 64) {
                const int a = 2 * stride * (i / stride) + (i % stride), b = a + stride;
                const bool up = (a & size) == 0;
                const uint64_t ka = sk[a], kb = sk[b];
                if ((ka > kb) == up) {
                    sk[a] = kb;
                    sk[b] = ka;
                }
            }
            __syncthreads();
        }
    uint64_t carry = 0ull;
    for (int base = ((n - 1) >> 6) << 6; base >= 0; base -= 64) {
        const int j = base + lane;
        uint64_t mask = 0ull;
        int t = 0;
        BinItem it{};
        if (j < n) {
            t = (int)(uint32_t)sk[j];
            it = items[t];
            mask = bin_mask(it, cx, cy);
        }
        const uint64_t rest = wave_suffix_or(mask, lane) | carry;
        carry = (uint64_t)__shfl((long long)rest, 0);
        if (j < n) {
            CamCand c = tpl[t];
            c.dmin = it.dmin;
            c.mask = mask;
            c.rest = rest;
            out[j] = c;
        }
    }
    __syncthreads();   /* sk is reused by the next cell */
}

__global__ __launch_bounds__(64) void k_bins_sort(const CamCand *__restrict__ tpl, const BinItem *__restrict__ items,
                                                  int32_t *__restrict__ cnt, const int32_t *__restrict__ keys,
                                                  const int32_t *__restrict__ every,
                                                  const int32_t *__restrict__ nonempty, BinsHdr *__restrict__ hdr,
                                                  CamCand *__restrict__ recs, int32_t rec_cap,
                                                  int32_t *__restrict__ bin_off, int32_t *__restrict__ bin_len,
                                                  int tx, int ncell, BinsPlan bp) {
    __shared__ uint64_t sk[kBinCellCap];
    const int lane = (int)threadIdx.x;
    const int n_every = hdr->n_every;
    const bool all = n_every > 0;   /* everywhere hulls: every cell has a list */
    const int nlist = all ? ncell : hdr->n_nonempty;
    for (int i = (int)blockIdx.x; i < nlist; i += (int)gridDim.x) {
        const int c = all ? i : nonempty[i];
        const int m = cnt[c];
        const int k = bp.cell_tile ? bp.cell_tile[c] : -2;   /* -1: no tile of this plan reads the cell */
        const int n = n_every > kBinMaxEverywhere ? kBinCellCap + 1 : m + n_every;
        int start = -1;
        if (k != -1 && n <= kBinCellCap) {
            if (lane == 0) start = atomicAdd(&hdr->total, n);
            start = __shfl(start, 0);
            if (start > rec_cap - n) start = -1;   /* does not fit: the cell walks the BVH */
        }
        if (start >= 0) {
            const int cx = c % tx, cy = c / tx;
            const int32_t *ids = keys + (size_t)c * kBinCellCap;
            if (n <= 64) bins_emit_small(tpl, items, ids, m, every, n, cx, cy, recs + start, lane);
            else bins_emit_large(tpl, items, ids, m, every, n, cx, cy, recs + start, sk, lane);
        }
        if (lane == 0) {
            if (k != -1) {
                bin_off[c] = start >= 0 ? start : 0;
                bin_len[c] = start >= 0 ? n : -1;
            }
            if (k >= 0 && start >= 0) {   /* the plan's priority lists */
                if (n >= bp.split) {
                    const int s = atomicAdd(&bp.phdr[0], 1);
                    if (s < bp.e_h) {
                        bp.prio[s] = k;
                        bp.taken[k] = 1;
                    }
                } else if (n >= bp.medium) {
                    const int s = atomicAdd(&bp.phdr[1], 1);
                    if (s < bp.e_m) {
                        bp.prio[bp.e_h + s] = k;
                        bp.taken[k] = 1;
                    }
                }
            }
            if (m) cnt[c] = 0;   /* next frame's counts start at zero */
        }
    }
    /* the last block resets the frame's counters for the next frame (every block
     * has read them by the time it arrives here) */
    if (lane == 0) {
        __threadfence();
        if (atomicAdd(&hdr->done, 1) == (int)gridDim.x - 1) {
            __threadfence();
            hdr->last_every = hdr->n_every;
            hdr->last_nonempty = hdr->n_nonempty;
            hdr->last_total = hdr->total;
            hdr->n_every = 0;
            hdr->n_nonempty = 0;
            hdr->total = 0;
            hdr->done = 0;
            __threadfence();
        }
    }
}

/* empty kernel: its launch at scene creation loads this TU's code object */
__global__ void k_warm_bins() {}

/* ---- host side ---- */

void bins_free(crt_hip_scene *sc) {
    BinsDev &b = sc->bins;
    for (void *p : b.allocs) (void)hipFree(p);
    b = BinsDev{};
    sc->ds.bins = nullptr;
    sc->ds.bin_off = nullptr;
    sc->ds.bin_len = nullptr;
}

namespace {

template <class T>
int bins_alloc(crt_hip_scene *sc, T **p, size_t n, bool zero = false) {
    void *q = nullptr;
    HIP_TRY(hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T)));
    sc->bins.allocs.push_back(q);
    if (zero) HIP_TRY(hipMemset(q, 0, std::max<size_t>(1, n) * sizeof(T)));
    sc->info.device_bytes += (int64_t)(n * sizeof(T));
    *p = static_cast<T *>(q);
    return CRT_OK;
}

int launch_project(crt_hip_scene *sc, hipStream_t s, int32_t *taken, int ntaken, int32_t *phdr) {
    BinsDev &b = sc->bins;
    const unsigned blocks = (unsigned)((b.nt + kProjTris - 1) / kProjTris);
    hipLaunchKernelGGL(k_bins_project, dim3(blocks), dim3(256), 0, s, b.tpl, b.nt, b.cam, b.items, b.cnt, b.keys,
                       b.every, b.nonempty, b.hdr, b.len, b.ncell, taken, ntaken, phdr);
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

}  // namespace

/* Scene create: the per-triangle templates and the buffers, sized by one
 * projection pass of this camera (its counts are read back; the lists are
 * rebuilt by every frame).  Leaves sc->ds.bins null when the scene takes no
 * bins. */
int bins_setup(crt_hip_scene *sc, const HostScene &hs) {
    BinsDev &b = sc->bins;
    BinCamera cam;
    if (!bin_camera(hs, cam)) return CRT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    b.cam = cam;
    b.nt = (int)hs.tri_attr.size();
    b.tx = cam.tx;
    b.ncell = cam.tx * cam.ty;
    std::vector<CamCand> tpl;
    bin_templates(hs, tpl);
    int rc;
    if ((rc = bins_alloc(sc, &b.tpl, tpl.size())) != CRT_OK) return rc;
    HIP_TRY(hipMemcpy(b.tpl, tpl.data(), tpl.size() * sizeof(CamCand), hipMemcpyHostToDevice));
    if ((rc = bins_alloc(sc, &b.items, (size_t)b.nt)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.cnt, (size_t)b.ncell, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.keys, (size_t)b.ncell * kBinCellCap)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.every, (size_t)kBinMaxEverywhere)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.nonempty, (size_t)b.ncell)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.hdr, 1, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.off, (size_t)b.ncell, true)) != CRT_OK) return rc;
    if ((rc = bins_alloc(sc, &b.len, (size_t)b.ncell, true)) != CRT_OK) return rc;
    /* sizing pass: counts per cell of this camera */
    if ((rc = launch_project(sc, sc->stream, nullptr, 0, nullptr)) != CRT_OK) return rc;
    std::vector<int32_t> cnt((size_t)b.ncell);
    BinsHdr h;
    HIP_TRY(hipMemcpyAsync(cnt.data(), b.cnt, cnt.size() * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(&h, b.hdr, sizeof h, hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    HIP_TRY(hipMemsetAsync(b.cnt, 0, cnt.size() * sizeof(int32_t), sc->stream));
    HIP_TRY(hipMemsetAsync(b.hdr, 0, sizeof(BinsHdr), sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    b.count.assign((size_t)b.ncell, 0);
    int64_t total = 0, listed = 0;
    for (int c = 0; c < b.ncell; ++c) {
        const int64_t n = (int64_t)cnt[(size_t)c] + h.n_every;
        if (n > kBinCellCap || h.n_every > kBinMaxEverywhere) {
            b.count[(size_t)c] = -1;
        } else {
            b.count[(size_t)c] = (int32_t)n;
            total += n;
        }
        listed += n > 0;
    }
    if (h.n_every > kBinMaxEverywhere || total > kBinMeanCap * b.ncell || total >= INT32_MAX / 2) {
        bins_free(sc);   /* the scene walks the BVH */
        return CRT_OK;
    }
    b.rec_cap = (int32_t)std::min<int64_t>(INT32_MAX / 2, total + total / 8 + 1024);
    if ((rc = bins_alloc(sc, &b.recs, (size_t)b.rec_cap)) != CRT_OK) return rc;
    b.sort_blocks = (int)std::max<int64_t>(64, std::min<int64_t>(16384, h.n_every > 0 ? b.ncell : listed));
    b.records = total;
    b.setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    sc->ds.bins = b.recs;
    sc->ds.bin_off = b.off;
    sc->ds.bin_len = b.len;
    sc->ds.bin_tx = b.tx;
    return CRT_OK;
}

/* A plan's camera-bins dispatch (BinsPlan): the base tiles stay in plan order;
 * the render grid puts 4 x e_h heavy-split waves and e_m medium waves before
 * them.  Capacities from the sizing pass's counts, with slack. */
int bins_plan(crt_hip_scene *sc, ShardPlan &plan) {
    BinsDev &b = sc->bins;
    const int nb = plan.ntiles;
    std::vector<int32_t> cell_tile((size_t)b.ncell, -1);
    for (int k = 0; k < nb; ++k) {
        const Tile &t = plan.tiles[(size_t)k];
        if ((t.x & 7) + t.w > 8 || (t.y & 7) + t.h > 8) continue;   /* not inside one cell: BVH walk */
        int32_t &e = cell_tile[(size_t)(t.y >> 3) * b.tx + (t.x >> 3)];
        e = e == -1 ? k : -2;   /* several tiles in one cell: none of them split */
    }
    int heavy = 0, medium = 0;
    for (int c = 0; c < b.ncell; ++c) {
        if (cell_tile[(size_t)c] < 0) continue;
        const int n = b.count[(size_t)c];
        if (n >= sc->bins_split) ++heavy;
        else if (n >= kBinsMedium) ++medium;
    }
    BinsPlan &bp = plan.bp;
    bp.e_h = heavy + heavy / 4 + 8;
    bp.e_m = medium + medium / 4 + 16;
    bp.split = sc->bins_split;
    bp.medium = kBinsMedium;
    bp.quad = sc->bins_quad;
    bp.nbase = nb;
    std::vector<void *> ps(4, nullptr);
    const size_t sizes[4] = {(size_t)b.ncell, (size_t)std::max(1, nb), (size_t)(bp.e_h + bp.e_m), 2};
    for (int i = 0; i < 4; ++i) {
        HIP_TRY(hipMalloc(&ps[(size_t)i], sizes[i] * sizeof(int32_t)));
        sc->plan_allocs.push_back(ps[(size_t)i]);
        HIP_TRY(hipMemset(ps[(size_t)i], 0, sizes[i] * sizeof(int32_t)));
    }
    HIP_TRY(hipMemcpy(ps[0], cell_tile.data(), cell_tile.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    bp.cell_tile = static_cast<int32_t *>(ps[0]);
    bp.taken = static_cast<int32_t *>(ps[1]);
    bp.prio = static_cast<int32_t *>(ps[2]);
    bp.phdr = static_cast<int32_t *>(ps[3]);
    plan.waves = 4 * bp.e_h + bp.e_m + nb;
    return CRT_OK;
}

/* The frame's lists, on `s`, before its render kernel. */
int bins_enqueue(crt_hip_scene *sc, const ShardPlan &plan, hipStream_t s) {
    BinsDev &b = sc->bins;
    int rc = launch_project(sc, s, plan.bp.taken, plan.bp.taken ? plan.bp.nbase : 0, plan.bp.phdr);
    if (rc != CRT_OK) return rc;
    hipLaunchKernelGGL(k_bins_sort, dim3((unsigned)b.sort_blocks), dim3(64), 0, s, b.tpl, b.items, b.cnt, b.keys,
                       b.every, b.nonempty, b.hdr, b.recs, b.rec_cap, b.off, b.len, b.tx, b.ncell, plan.bp);
    HIP_TRY(hipGetLastError());
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
    int rc = bins_enqueue(sc, none, sc->stream);
    if (rc != CRT_OK) return rc;
    std::vector<int32_t> off((size_t)b.ncell), len((size_t)b.ncell);
    std::vector<CamCand> recs((size_t)b.rec_cap);
    HIP_TRY(hipMemcpyAsync(off.data(), b.off, off.size() * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipMemcpyAsync(len.data(), b.len, len.size() * sizeof(int32_t), hipMemcpyDeviceToHost, sc->stream));
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
