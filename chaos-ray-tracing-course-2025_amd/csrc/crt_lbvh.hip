/*
 * crt_lbvh.hip — device build of the secondary-ray BVH for large scenes
 * (crt_lbvh.h): the host SAH build (crt_bvh_build.cpp) takes seconds above
 * 2^18 triangles; this one takes milliseconds.
 *
 *   1. per triangle: its conservative hull (crt_device.h triangle_hull, the
 *      host build's), rounded outwards to floats, and its vertex-box centre;
 *      the centres' bounds (wave reductions + one atomic per wave);
 *   2. a 62-bit key per triangle: 30-bit Morton code of the quantised centre
 *      above the triangle id (unique keys), sorted (hipCUB radix sort);
 *   3. the triangles in key order (geometry as the BVH's triangle arrays hold
 *      it), and a segment tree of their hull boxes (one launch a level);
 *   4. the binary radix tree over the sorted keys (Karras 2012: internal node
 *      i, its key range by the common-prefix search, its split), parents;
 *   5. leaves: a node of at most kLbvhLeaf triangles is a leaf.  Its first
 *      triangle is marked; the marks' prefix sum gives any node's leaf count
 *      in its range, so its subtree's record count (2 leaves - 1) without a
 *      bottom-up pass;
 *   6. every kept node finds its preorder position in each of the 8 octant
 *      orders by walking up to the root (near child first: the right child
 *      holds the larger keys, so the larger coordinates along the axis of the
 *      split's highest differing Morton bit), its box by a segment-tree range
 *      union, and writes itself and its leaf children.
 *
 * Boxes are unions of rounded-out hulls, so every box holds the union of its
 * triangles' hulls (rounding is monotone): the walk's exactness argument
 * (crt_bvh.h) holds whatever the shape.
 */
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <limits>
#include <string>
#include <type_traits>
#include <vector>

#include "crt_device.h"
#include "crt_host.h"
#include "crt_lbvh.h"

#ifndef CRT_LBVH_LEAF
#define CRT_LBVH_LEAF 2
#endif

namespace crt_amd {

namespace {

#define LB_TRY(expr)                                                                                      \
    do {                                                                                                  \
        const hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                             \
            return set_error(CRT_E_HIP, std::string("bvh build: ") + #expr + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kLbvhLeaf = CRT_LBVH_LEAF;   /* triangles per leaf, at most (the host build's kLeafMax) */
static_assert(kLbvhLeaf >= 1 && kLbvhLeaf <= 15, "leaf count must fit BNode::leaf");
constexpr int kMaxSegLevels = 40;

struct LBox {
    float lo[3], hi[3];
};

struct SegLevels {
    int32_t n;                    /* levels */
    int64_t off[kMaxSegLevels];   /* first box of level k in the tree array */
};

/* internal node of the radix tree: children (>= 0 internal, < 0 leaf -(k + 1)),
 * its key range [lo, hi], the split's axis */
struct LInt {
    int32_t left, right;
    int32_t lo, hi;
    int32_t axis;
    int32_t pad;
};

__device__ __forceinline__ uint32_t f2o(float f) {   /* float order as unsigned order */
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__device__ __forceinline__ void box_grow(LBox &a, const LBox &b) {
    for (int k = 0; k < 3; ++k) {
        a.lo[k] = fminf(a.lo[k], b.lo[k]);
        a.hi[k] = fmaxf(a.hi[k], b.hi[k]);
    }
}
__device__ __forceinline__ LBox box_empty() {
    LBox b;
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = INFINITY;
        b.hi[k] = -INFINITY;
    }
    return b;
}

/* 1. hulls, centres and the centres' bounds (bounds: 3 mins then 3 maxes as f2o) */
__global__ __launch_bounds__(256) void k_lb_prims(const float *__restrict__ vpos, const DTriAttr *__restrict__ ta,
                                                  const float *__restrict__ fnorm, int32_t nt, double G,
                                                  LBox *__restrict__ hull, float4 *__restrict__ cen,
                                                  uint32_t *__restrict__ bounds) {
    const int32_t t = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
    if (t < nt) {
        const DTriAttr a = ta[t];
        float p0[3], p1[3], p2[3], fn[3];
        for (int k = 0; k < 3; ++k) {
            p0[k] = vpos[3 * (int64_t)a.i0 + k];
            p1[k] = vpos[3 * (int64_t)a.i1 + k];
            p2[k] = vpos[3 * (int64_t)a.i2 + k];
            fn[k] = fnorm[3 * (int64_t)t + k];
        }
        const HullD h = triangle_hull(p0, p1, p2, fn, G);
        LBox b;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = round_down(h.lo[k]);
            b.hi[k] = round_up(h.hi[k]);
        }
        hull[t] = b;
        float c[3];
        bool fin = true;
        for (int k = 0; k < 3; ++k) {
            c[k] = 0.5f * (fminf(p0[k], fminf(p1[k], p2[k])) + fmaxf(p0[k], fmaxf(p1[k], p2[k])));
            fin = fin && isfinite(c[k]);
        }
        if (!fin) c[0] = c[1] = c[2] = NAN;   /* quantised to 0: placed anywhere, its box holds it */
        cen[t] = make_float4(c[0], c[1], c[2], 0.f);
        if (fin)
            for (int k = 0; k < 3; ++k) mn[k] = mx[k] = f2o(c[k]);
    }
    for (int k = 0; k < 3; ++k) {
        for (int d = 32; d >= 1; d >>= 1) {
            mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], d));
            mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], d));
        }
    }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[k], mn[k]);
            atomicMax(&bounds[3 + k], mx[k]);
        }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {   /* bit i -> bit 3 i */
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

/* 2. keys: Morton code (x at bits 3k + 2, y 3k + 1, z 3k) << 32 | id */
__global__ __launch_bounds__(256) void k_lb_keys(const float4 *__restrict__ cen, const uint32_t *__restrict__ bounds,
                                                 int32_t nt, uint64_t *__restrict__ keys) {
    const int32_t t = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= nt) return;
    const float4 c4 = cen[t];
    const float c[3] = {c4.x, c4.y, c4.z};
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
        const float lo = o2f(bounds[k]), hi = o2f(bounds[3 + k]);
        const float ext = hi - lo;
        float u = ext > 0.f ? (c[k] - lo) / ext : 0.f;
        if (!(u >= 0.f)) u = 0.f;   /* NaN centre, or below */
        q[k] = (uint32_t)fminf(u * 1024.f, 1023.f);
    }
    const uint32_t m = (spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]);
    keys[t] = ((uint64_t)m << 32) | (uint32_t)t;
}

/* 3. triangles in key order, and the segment tree's level 0 */
__global__ __launch_bounds__(256) void k_lb_sorted(const uint64_t *__restrict__ keys, int32_t n,
                                                   const float *__restrict__ vpos, const DTriAttr *__restrict__ ta,
                                                   const float *__restrict__ fnorm, const uint8_t *__restrict__ cull,
                                                   const LBox *__restrict__ hull, DTriGeo *__restrict__ btri,
                                                   int32_t *__restrict__ btri_id, LBox *__restrict__ seg0) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int32_t t = (int32_t)(uint32_t)(keys[i] & 0xffffffffu);
    const DTriAttr a = ta[t];
    DTriGeo g;
    g.v0x = vpos[3 * (int64_t)a.i0]; g.v0y = vpos[3 * (int64_t)a.i0 + 1]; g.v0z = vpos[3 * (int64_t)a.i0 + 2];
    g.v1x = vpos[3 * (int64_t)a.i1]; g.v1y = vpos[3 * (int64_t)a.i1 + 1]; g.v1z = vpos[3 * (int64_t)a.i1 + 2];
    g.v2x = vpos[3 * (int64_t)a.i2]; g.v2y = vpos[3 * (int64_t)a.i2 + 1]; g.v2z = vpos[3 * (int64_t)a.i2 + 2];
    g.nx = fnorm[3 * (int64_t)t]; g.ny = fnorm[3 * (int64_t)t + 1]; g.nz = fnorm[3 * (int64_t)t + 2];
    btri[i] = g;
    btri_id[i] = t | (cull[t] ? (int32_t)0x80000000 : 0);
    seg0[i] = hull[t];
}

__global__ __launch_bounds__(256) void k_lb_seg(const LBox *__restrict__ prev, int64_t nprev, LBox *__restrict__ cur,
                                                int64_t ncur) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ncur) return;
    LBox b = prev[2 * j];
    if (2 * j + 1 < nprev) box_grow(b, prev[2 * j + 1]);
    cur[j] = b;
}

/* union of the sorted triangles' boxes lo .. hi (inclusive) */
__device__ LBox seg_union(const LBox *__restrict__ seg, const SegLevels &L, int32_t lo, int32_t hi) {
    LBox acc = box_empty();
    int64_t l = lo, r = (int64_t)hi + 1;
    for (int k = 0; k < L.n && l < r; ++k) {
        const LBox *lv = seg + L.off[k];
        if (l & 1) box_grow(acc, lv[l++]);
        if (r & 1) box_grow(acc, lv[--r]);
        l >>= 1;
        r >>= 1;
    }
    return acc;
}

/* 4. the radix tree (Karras 2012, keys unique) */
__device__ __forceinline__ int lb_delta(const uint64_t *__restrict__ keys, int32_t n, int32_t i, int64_t j) {
    if (j < 0 || j >= n) return -1;
    return __clzll((long long)(keys[i] ^ keys[j]));
}

__global__ __launch_bounds__(256) void k_lb_internal(const uint64_t *__restrict__ keys, int32_t n,
                                                     LInt *__restrict__ in, int32_t *__restrict__ parent) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n - 1) return;
    const int d = lb_delta(keys, n, i, (int64_t)i + 1) - lb_delta(keys, n, i, (int64_t)i - 1) >= 0 ? 1 : -1;
    const int dmin = lb_delta(keys, n, i, (int64_t)i - d);
    int64_t lmax = 2;
    while (lb_delta(keys, n, i, (int64_t)i + lmax * d) > dmin) lmax *= 2;
    int64_t l = 0;
    for (int64_t t = lmax / 2; t >= 1; t /= 2)
        if (lb_delta(keys, n, i, (int64_t)i + (l + t) * d) > dmin) l += t;
    const int64_t j = (int64_t)i + l * d;
    const int dnode = lb_delta(keys, n, i, j);
    int64_t s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (lb_delta(keys, n, i, (int64_t)i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int32_t gamma = (int32_t)((int64_t)i + s * d + min(d, 0));
    LInt nd;
    nd.lo = (int32_t)min<int64_t>(i, j);
    nd.hi = (int32_t)max<int64_t>(i, j);
    nd.left = nd.lo == gamma ? -(gamma + 1) : gamma;
    nd.right = nd.hi == gamma + 1 ? -(gamma + 2) : gamma + 1;
    /* the split's highest differing bit: a Morton bit gives its axis (x at
     * 3k + 2, y 3k + 1, z 3k); equal codes (an id bit) take x */
    const uint64_t x = keys[gamma] ^ keys[gamma + 1];
    const int b = 63 - __clzll((long long)x);
    nd.axis = b >= 32 ? 2 - (b - 32) % 3 : 0;
    nd.pad = 0;
    in[i] = nd;
    if (nd.left >= 0) parent[nd.left] = i;
    if (nd.right >= 0) parent[nd.right] = i;
    if (i == 0) parent[0] = -1;
}

__device__ __forceinline__ void child_range(const LInt *__restrict__ in, int32_t c, int32_t &lo, int32_t &hi) {
    if (c < 0) {
        lo = hi = -c - 1;
    } else {
        lo = in[c].lo;
        hi = in[c].hi;
    }
}

/* 5. a kept node (more than kLbvhLeaf triangles) marks the first triangle of
 * each of its leaf children */
__global__ __launch_bounds__(256) void k_lb_mark(const LInt *__restrict__ in, int32_t n, int32_t *__restrict__ mark) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n - 1) return;
    const LInt nd = in[i];
    if (nd.hi - nd.lo + 1 <= kLbvhLeaf) return;
    int32_t lo, hi;
    child_range(in, nd.left, lo, hi);
    if (hi - lo + 1 <= kLbvhLeaf) mark[lo] = 1;
    child_range(in, nd.right, lo, hi);
    if (hi - lo + 1 <= kLbvhLeaf) mark[lo] = 1;
}

/* records of a node's subtree: leaves in its range (marks' prefix F) */
__device__ __forceinline__ int32_t sub_count(const int32_t *__restrict__ F, int32_t lo, int32_t hi) {
    return hi - lo + 1 <= kLbvhLeaf ? 1 : 2 * (F[hi + 1] - F[lo]) - 1;
}

__device__ __forceinline__ BNode make_bnode(const LBox &b, int32_t skip, int32_t leaf) {
    BNode o;
    o.lo_x = b.lo[0]; o.hi_x = b.hi[0];
    o.lo_y = b.lo[1]; o.hi_y = b.hi[1];
    o.lo_z = b.lo[2]; o.hi_z = b.hi[2];
    o.skip = skip;
    o.leaf = leaf;
    return o;
}

/* 6. positions, boxes and records of every kept node and its leaf children */
__global__ __launch_bounds__(256) void k_lb_emit(const LInt *__restrict__ in, const int32_t *__restrict__ parent,
                                                 int32_t n, const int32_t *__restrict__ F, const LBox *__restrict__ seg,
                                                 SegLevels L, BNode *__restrict__ out, int32_t N,
                                                 int32_t *__restrict__ stats) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n - 1) return;
    const LInt nd = in[i];
    if (nd.hi - nd.lo + 1 <= kLbvhLeaf) return;   /* inside a leaf */
    int32_t pos[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t c = i, depth = 0;
    while (c != 0) {
        const int32_t p = parent[c];
        const LInt P = in[p];
        int32_t llo, lhi, rlo, rhi;
        child_range(in, P.left, llo, lhi);
        child_range(in, P.right, rlo, rhi);
        const int32_t cl = sub_count(F, llo, lhi), cr = sub_count(F, rlo, rhi);
        const bool is_left = P.left == c;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
            const bool neg = ((o >> P.axis) & 1) != 0;   /* right (larger) child first */
            const bool first = neg ? !is_left : is_left;
            pos[o] += first ? 1 : 1 + (neg ? cr : cl);
        }
        c = p;
        ++depth;
    }
    const int32_t cnt = sub_count(F, nd.lo, nd.hi);
    const LBox box = seg_union(seg, L, nd.lo, nd.hi);
    int32_t llo, lhi, rlo, rhi;
    child_range(in, nd.left, llo, lhi);
    child_range(in, nd.right, rlo, rhi);
    const bool lleaf = lhi - llo + 1 <= kLbvhLeaf, rleaf = rhi - rlo + 1 <= kLbvhLeaf;
    const int32_t cl = sub_count(F, llo, lhi);
    const int32_t cr = sub_count(F, rlo, rhi);
    LBox lb = box, rb = box;
    if (lleaf) lb = seg_union(seg, L, llo, lhi);
    if (rleaf) rb = seg_union(seg, L, rlo, rhi);
    for (int o = 0; o < 8; ++o) {
        BNode *ord = out + (size_t)o * (N + 1);
        ord[pos[o]] = make_bnode(box, pos[o] + cnt, 0);
        const bool neg = ((o >> nd.axis) & 1) != 0;
        const int32_t lpos = neg ? pos[o] + 1 + cr : pos[o] + 1;
        const int32_t rpos = neg ? pos[o] + 1 : pos[o] + 1 + cl;
        if (lleaf) ord[lpos] = make_bnode(lb, lpos + 1, llo * 16 + (lhi - llo + 1));
        if (rleaf) ord[rpos] = make_bnode(rb, rpos + 1, rlo * 16 + (rhi - rlo + 1));
    }
    atomicMax(&stats[0], depth + 1);
}

inline unsigned grid_for(int64_t n, int block = 256) { return (unsigned)std::max<int64_t>(1, (n + block - 1) / block); }

struct Scratch {
    std::vector<void *> ptrs;
    ~Scratch() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T>
    int alloc(T **p, size_t count) {
        void *q = nullptr;
        LB_TRY(hipMalloc(&q, std::max<size_t>(1, count) * sizeof(T)));
        ptrs.push_back(q);
        *p = static_cast<T *>(q);
        return CRT_OK;
    }
};

}  // namespace

int build_bvh_device(const HostScene &hs, void *stream_v, DeviceBvh &out) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = static_cast<hipStream_t>(stream_v);
    const int64_t nt64 = (int64_t)hs.tri_attr.size();
    if (nt64 <= kLbvhLeaf) return set_error(CRT_E_UNSUPPORTED, "bvh build: too few triangles for the device build");
    if (nt64 * 16 >= (int64_t)std::numeric_limits<int32_t>::max())
        return set_error(CRT_E_UNSUPPORTED, "too many triangles for the BVH leaf record");
    const int32_t n = (int32_t)nt64;
    Scratch tmp;
    int rc;
    float *d_vpos = nullptr, *d_fn = nullptr;
    DTriAttr *d_ta = nullptr;
    uint8_t *d_cull = nullptr;
    auto upload = [&](const auto &v, auto **dst) -> int {
        int r = tmp.alloc(dst, v.size());
        if (r != CRT_OK) return r;
        if (!v.empty()) LB_TRY(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice, st));
        return CRT_OK;
    };
    if ((rc = upload(hs.vpos, &d_vpos)) != CRT_OK) return rc;
    if ((rc = upload(hs.tri_attr, &d_ta)) != CRT_OK) return rc;
    if ((rc = upload(hs.face_normal, &d_fn)) != CRT_OK) return rc;
    if ((rc = upload(hs.tri_cull, &d_cull)) != CRT_OK) return rc;

    LBox *d_hull = nullptr;
    float4 *d_cen = nullptr;
    uint32_t *d_bounds = nullptr;
    uint64_t *d_keys = nullptr, *d_sorted = nullptr;
    if ((rc = tmp.alloc(&d_hull, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_cen, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_bounds, 6)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_keys, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_sorted, (size_t)n)) != CRT_OK) return rc;
    const uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    LB_TRY(hipMemcpyAsync(d_bounds, init, sizeof init, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_lb_prims, dim3(grid_for(n)), dim3(256), 0, st, d_vpos, d_ta, d_fn, n, hs.prune_G, d_hull,
                       d_cen, d_bounds);
    LB_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_lb_keys, dim3(grid_for(n)), dim3(256), 0, st, d_cen, d_bounds, n, d_keys);
    LB_TRY(hipGetLastError());
    {
        size_t bytes = 0;
        LB_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, d_keys, d_sorted, n, 0, 62, st));
        void *work = nullptr;
        if ((rc = tmp.alloc(reinterpret_cast<uint8_t **>(&work), bytes)) != CRT_OK) return rc;
        LB_TRY(hipcub::DeviceRadixSort::SortKeys(work, bytes, d_keys, d_sorted, n, 0, 62, st));
    }

    /* outputs (owned by the caller) */
    auto keep = [&](auto **p, size_t count) -> int {
        void *q = nullptr;
        LB_TRY(hipMalloc(&q, std::max<size_t>(1, count) * sizeof(**p)));
        out.allocs.push_back(q);
        *p = static_cast<std::remove_reference_t<decltype(*p)>>(q);
        return CRT_OK;
    };
    if ((rc = keep(&out.btri, (size_t)n)) != CRT_OK) return rc;
    if ((rc = keep(&out.btri_id, (size_t)n)) != CRT_OK) return rc;

    /* segment tree of the sorted hull boxes */
    SegLevels L{};
    std::vector<int64_t> size;
    {
        int64_t off = 0, s = n;
        for (;;) {
            if (L.n >= kMaxSegLevels) return set_error(CRT_E_UNSUPPORTED, "bvh build: too many triangles");
            L.off[L.n++] = off;
            size.push_back(s);
            off += s;
            if (s == 1) break;
            s = (s + 1) / 2;
        }
        LBox *d_seg = nullptr;
        if ((rc = tmp.alloc(&d_seg, (size_t)off)) != CRT_OK) return rc;
        hipLaunchKernelGGL(k_lb_sorted, dim3(grid_for(n)), dim3(256), 0, st, d_sorted, n, d_vpos, d_ta, d_fn, d_cull,
                           d_hull, out.btri, out.btri_id, d_seg);
        LB_TRY(hipGetLastError());
        for (int k = 1; k < L.n; ++k)
            hipLaunchKernelGGL(k_lb_seg, dim3(grid_for(size[k])), dim3(256), 0, st, d_seg + L.off[k - 1], size[k - 1],
                               d_seg + L.off[k], size[k]);
        LB_TRY(hipGetLastError());

        /* radix tree, leaves, record counts */
        LInt *d_in = nullptr;
        int32_t *d_par = nullptr, *d_mark = nullptr, *d_F = nullptr, *d_stats = nullptr;
        if ((rc = tmp.alloc(&d_in, (size_t)n - 1)) != CRT_OK) return rc;
        if ((rc = tmp.alloc(&d_par, (size_t)n - 1)) != CRT_OK) return rc;
        if ((rc = tmp.alloc(&d_mark, (size_t)n + 1)) != CRT_OK) return rc;
        if ((rc = tmp.alloc(&d_F, (size_t)n + 1)) != CRT_OK) return rc;
        if ((rc = tmp.alloc(&d_stats, 4)) != CRT_OK) return rc;
        LB_TRY(hipMemsetAsync(d_mark, 0, ((size_t)n + 1) * sizeof(int32_t), st));
        LB_TRY(hipMemsetAsync(d_stats, 0, 4 * sizeof(int32_t), st));
        hipLaunchKernelGGL(k_lb_internal, dim3(grid_for(n - 1)), dim3(256), 0, st, d_sorted, n, d_in, d_par);
        LB_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_lb_mark, dim3(grid_for(n - 1)), dim3(256), 0, st, d_in, n, d_mark);
        LB_TRY(hipGetLastError());
        {
            size_t bytes = 0;
            LB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, d_mark, d_F, n + 1, st));
            void *work = nullptr;
            if ((rc = tmp.alloc(reinterpret_cast<uint8_t **>(&work), bytes)) != CRT_OK) return rc;
            LB_TRY(hipcub::DeviceScan::ExclusiveSum(work, bytes, d_mark, d_F, n + 1, st));
        }
        int32_t leaves = 0;
        LB_TRY(hipMemcpyAsync(&leaves, d_F + n, sizeof leaves, hipMemcpyDeviceToHost, st));
        LB_TRY(hipStreamSynchronize(st));
        const int64_t N = 2 * (int64_t)leaves - 1;
        if (leaves < 2 || N >= (int64_t)std::numeric_limits<int32_t>::max() / 8)
            return set_error(CRT_E_STATE, "bvh build: bad leaf count " + std::to_string(leaves));
        if ((rc = keep(&out.bnodes, (size_t)8 * (N + 1))) != CRT_OK) return rc;
        LB_TRY(hipMemsetAsync(out.bnodes, 0, (size_t)8 * (N + 1) * sizeof(BNode), st));   /* + a zero record per order */
        hipLaunchKernelGGL(k_lb_emit, dim3(grid_for(n - 1)), dim3(256), 0, st, d_in, d_par, n, d_F, d_seg, L,
                           out.bnodes, (int32_t)N, d_stats);
        LB_TRY(hipGetLastError());
        int32_t stats[4] = {0, 0, 0, 0};
        LB_TRY(hipMemcpyAsync(stats, d_stats, sizeof stats, hipMemcpyDeviceToHost, st));
        LB_TRY(hipStreamSynchronize(st));
        out.node_count = (int32_t)N;
        out.max_depth = stats[0];
    }
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

}  // namespace crt_amd
