/*
 * crt_tree_build.hip — exact device-side build of the reference's acceleration
 * tree (acceleration_tree::build / build_branch, crt_acceleration_tree.cpp:13-106;
 * AABB::split / intersects, crt_aabb.h:24-45) and of every layout the walks
 * read (crt_layout.h): the DNode array in the reference's LIFO visit order,
 * the 8 octant-ordered PNode arrays with their triangle hulls, the leaf slots.
 *
 * The reference recursion is depth first; here the tree is built breadth
 * first, one launch sequence per tree level:
 *   1. every entry (node, triangle id) of the level tests its triangle's box
 *      against both child cells of its node — the reference's midpoint split
 *      on axis depth % 3 and its inclusive overlap test, same float operations;
 *   2. an exclusive scan of the packed flags (left | right << 32) places each
 *      entry that survives in its child's segment of the next level, keeping
 *      the input order (the reference keeps it too: in-place compaction of
 *      child0, push_back into child1);
 *   3. children are numbered level by level; leaves (depth > 39 or <= 16
 *      triangles, crt_acceleration_tree.cpp:32) keep their segment.
 * The reference's node numbers (preorder, child0's subtree first), the
 * traversal order (child1 first) and the 8 octant orders (near child first)
 * come afterwards from subtree sizes: a node's first child is at its index + 1,
 * its second at index + 1 + size(first).  Leaf slots are numbered in the
 * traversal order, as in crt_scene_build.cpp.  Every float the tree depends on
 * uses the reference's operations (-ffp-contract=off), so bounds, topology and
 * leaf contents are bit-identical to the host build, which is pinned to the
 * reference's own compiled build (tests/test_oracle_ref.py); the hulls use the
 * same double arithmetic as the host (crt_device.h triangle_hull).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <limits>
#include <string>
#include <type_traits>
#include <vector>

#include "crt_device.h"
#include "crt_host.h"
#include "crt_tree_build.h"

namespace crt_amd {
namespace {

#define TB_TRY(expr)                                                                                      \
    do {                                                                                                  \
        const hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                             \
            return set_error(CRT_E_HIP, std::string("tree build: ") + #expr + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kMaxTreeDepth = 39;   /* crt_acceleration_tree.h:12 */
constexpr int kMaxLeafTris = 16;    /* crt_acceleration_tree.h:13 */
constexpr int kOrders = 9;          /* 0: reference numbering, 1 + o: octant o (octant 7 = traversal order) */

struct Box6 { float lo[3], hi[3]; };

/* A node while the tree is built (global id = level offset + index). */
struct LNode {
    float lo[3], hi[3];   /* cell */
    int64_t begin;        /* first entry in the entry pool */
    int32_t count, depth;
    int32_t child[2];     /* global ids, -1 = none */
    int32_t leaf;         /* 1: leaf (entries are its triangles) */
    int32_t pad;
};

__device__ __forceinline__ bool overlap(const float clo[3], const float chi[3], const Box6 &b) {   /* crt_aabb.h:37-45 */
    for (int k = 0; k < 3; ++k) {
        if (b.lo[k] > chi[k]) return false;
        if (b.hi[k] < clo[k]) return false;
    }
    return true;
}

/* child cell c (0 = lower half) of a node (crt_aabb.h:24-35) */
__device__ __forceinline__ void child_cell(const LNode &n, int c, float lo[3], float hi[3]) {
    for (int k = 0; k < 3; ++k) { lo[k] = n.lo[k]; hi[k] = n.hi[k]; }
    const int axis = n.depth % 3;
    const float mid = (n.lo[axis] + n.hi[axis]) * 0.5f;
    if (c == 0) hi[axis] = mid; else lo[axis] = mid;
}

__device__ __forceinline__ uint32_t lo32(uint64_t v) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }

/* ---- exclusive scan (out has n + 1 entries, out[n] = total) ------------- */
template <class T>
__global__ __launch_bounds__(256) void k_scan_local(const T *__restrict__ in, T *__restrict__ out,
                                                    T *__restrict__ sums, int64_t n) {
    __shared__ T sh[256];
    const int64_t base = (int64_t)blockIdx.x * 1024 + (int64_t)threadIdx.x * 4;
    T v[4];
    T acc = 0;
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j;
        const T x = i < n ? in[i] : T(0);
        v[j] = acc;
        acc += x;
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const T t = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : T(0);
        __syncthreads();
        sh[threadIdx.x] += t;
        __syncthreads();
    }
    const T excl = sh[threadIdx.x] - acc;
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j;
        if (i < n) out[i] = v[j] + excl;
    }
    if (threadIdx.x == 255) sums[blockIdx.x] = sh[255];
}

template <class T>
__global__ __launch_bounds__(256) void k_scan_add(T *__restrict__ out, const T *__restrict__ offs, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 1024 + (int64_t)threadIdx.x * 4;
    const T o = offs[blockIdx.x];
    for (int j = 0; j < 4; ++j)
        if (base + j < n) out[base + j] += o;
}

template <class T>
__global__ void k_scan_total(const T *__restrict__ in, T *__restrict__ out, int64_t n) {
    out[n] = n > 0 ? out[n - 1] + in[n - 1] : T(0);
}

struct Scratch {
    std::vector<void *> ptrs;
    ~Scratch() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T>
    int alloc(T **p, size_t count) {
        void *q = nullptr;
        TB_TRY(hipMalloc(&q, std::max<size_t>(1, count) * sizeof(T)));
        ptrs.push_back(q);
        *p = static_cast<T *>(q);
        return CRT_OK;
    }
};

template <class T>
int scan_exclusive(const T *in, T *out, int64_t n, hipStream_t st, Scratch &tmp) {
    if (n > 0) {
        const int64_t nb = (n + 1023) / 1024;
        T *sums = nullptr, *sums_scan = nullptr;
        int rc;
        if ((rc = tmp.alloc(&sums, (size_t)nb)) != CRT_OK) return rc;
        hipLaunchKernelGGL(k_scan_local<T>, dim3((unsigned)nb), dim3(256), 0, st, in, out, sums, n);
        TB_TRY(hipGetLastError());
        if (nb > 1) {
            if ((rc = tmp.alloc(&sums_scan, (size_t)nb + 1)) != CRT_OK) return rc;
            if ((rc = scan_exclusive(sums, sums_scan, nb, st, tmp)) != CRT_OK) return rc;
            hipLaunchKernelGGL(k_scan_add<T>, dim3((unsigned)nb), dim3(256), 0, st, out, sums_scan, n);
            TB_TRY(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(k_scan_total<T>, dim3(1), dim3(1), 0, st, in, out, n);
    TB_TRY(hipGetLastError());
    return CRT_OK;
}

/* ---- level build ------------------------------------------------------- */
__global__ __launch_bounds__(256) void k_tri_boxes(const float *__restrict__ vpos, const DTriAttr *__restrict__ ta,
                                                   int64_t nt, Box6 *__restrict__ tb, int32_t *__restrict__ ids) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    Box6 b;
    for (int k = 0; k < 3; ++k) { b.lo[k] = INFINITY; b.hi[k] = -INFINITY; }
    const int32_t vs[3] = {ta[t].i0, ta[t].i1, ta[t].i2};
    for (int v = 0; v < 3; ++v)
        for (int k = 0; k < 3; ++k) {
            const float p = vpos[3 * (int64_t)vs[v] + k];
            b.lo[k] = (p < b.lo[k]) ? p : b.lo[k];   /* std::min(lo, p) */
            b.hi[k] = (b.hi[k] < p) ? p : b.hi[k];   /* std::max(hi, p) */
        }
    tb[t] = b;
    ids[t] = (int32_t)t;
}

__global__ __launch_bounds__(256) void k_classify(LNode *__restrict__ nodes, int32_t nn) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    LNode &n = nodes[k];
    n.leaf = (n.depth > kMaxTreeDepth || n.count <= kMaxLeafTris) ? 1 : 0;   /* :32 */
}

/* entry j of the level: its node (binary search on segment begins) and the
 * two overlap flags against the node's child cells */
__global__ __launch_bounds__(256) void k_entry_flags(const LNode *__restrict__ nodes, int32_t nn,
                                                     const int32_t *__restrict__ ids, int64_t ids_base, int64_t nids,
                                                     const Box6 *__restrict__ tb, uint64_t *__restrict__ flags,
                                                     int32_t *__restrict__ node_of) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nids) return;
    const int64_t pos = ids_base + j;
    int32_t lo = 0, hi = nn - 1;
    while (lo < hi) {   /* last node with begin <= pos */
        const int32_t mid = (lo + hi + 1) >> 1;
        if (nodes[mid].begin <= pos) lo = mid; else hi = mid - 1;
    }
    node_of[j] = lo;
    const LNode n = nodes[lo];
    uint64_t f = 0;
    if (!n.leaf) {
        const Box6 b = tb[ids[pos]];
        float c0lo[3], c0hi[3], c1lo[3], c1hi[3];
        child_cell(n, 0, c0lo, c0hi);
        child_cell(n, 1, c1lo, c1hi);
        f = (uint64_t)(overlap(c0lo, c0hi, b) ? 1u : 0u) | ((uint64_t)(overlap(c1lo, c1hi, b) ? 1u : 0u) << 32);
    }
    flags[j] = f;
}

__global__ __launch_bounds__(256) void k_node_children(const LNode *__restrict__ nodes, int32_t nn,
                                                       const uint64_t *__restrict__ S, int64_t ids_base,
                                                       int64_t *__restrict__ nbase, int32_t *__restrict__ nl,
                                                       int32_t *__restrict__ nr, int32_t *__restrict__ ccount) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    const LNode n = nodes[k];
    const int64_t b = n.begin - ids_base, e = b + n.count;
    const uint64_t sb = S[b], se = S[e];
    nbase[k] = (int64_t)lo32(sb) + (int64_t)hi32(sb);
    const int32_t l = n.leaf ? 0 : (int32_t)(lo32(se) - lo32(sb));
    const int32_t r = n.leaf ? 0 : (int32_t)(hi32(se) - hi32(sb));
    nl[k] = l;
    nr[k] = r;
    ccount[k] = (l > 0 ? 1 : 0) + (r > 0 ? 1 : 0);
}

__global__ __launch_bounds__(256) void k_make_children(LNode *__restrict__ nodes, int32_t nn,
                                                       const int64_t *__restrict__ nbase, const int32_t *__restrict__ nl,
                                                       const int32_t *__restrict__ nr, const int32_t *__restrict__ cpos,
                                                       LNode *__restrict__ next, int32_t next_gid0, int64_t next_ids_base) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    LNode &n = nodes[k];
    n.child[0] = n.child[1] = -1;
    if (n.leaf) return;
    int32_t idx = cpos[k];
    const int32_t cnt[2] = {nl[k], nr[k]};
    int64_t begin = next_ids_base + nbase[k];
    for (int c = 0; c < 2; ++c) {
        if (cnt[c] == 0) continue;
        LNode ch;
        child_cell(n, c, ch.lo, ch.hi);
        ch.begin = begin;
        ch.count = cnt[c];
        ch.depth = n.depth + 1;
        ch.child[0] = ch.child[1] = -1;
        ch.leaf = 0;
        ch.pad = 0;
        next[idx] = ch;
        n.child[c] = next_gid0 + idx;
        ++idx;
        begin += cnt[c];
    }
}

__global__ __launch_bounds__(256) void k_scatter(const LNode *__restrict__ nodes, const int32_t *__restrict__ node_of,
                                                 const uint64_t *__restrict__ flags, const uint64_t *__restrict__ S,
                                                 const int32_t *__restrict__ ids, int64_t ids_base, int64_t nids,
                                                 const int64_t *__restrict__ nbase, const int32_t *__restrict__ nl,
                                                 int32_t *__restrict__ next_ids) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nids) return;
    const uint64_t f = flags[j];
    if (f == 0) return;
    const int32_t k = node_of[j];
    const int64_t b = nodes[k].begin - ids_base;
    const uint64_t sb = S[b], sj = S[j];
    const int32_t id = ids[ids_base + j];
    if (lo32(f)) next_ids[nbase[k] + (int64_t)(lo32(sj) - lo32(sb))] = id;
    if (hi32(f)) next_ids[nbase[k] + nl[k] + (int64_t)(hi32(sj) - hi32(sb))] = id;
}

/* ---- numbering --------------------------------------------------------- */
__global__ __launch_bounds__(256) void k_sizes(const LNode *__restrict__ nodes, int32_t g0, int32_t nn,
                                               int32_t *__restrict__ size) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    const LNode n = nodes[g0 + k];
    int32_t sz = 1;
    for (int c = 0; c < 2; ++c)
        if (n.child[c] >= 0) sz += size[n.child[c]];
    size[g0 + k] = sz;
}

/* order o: 0 = reference numbering (child0 first); 1 + oct = octant oct
 * (near child first: on a negative direction along the split axis the upper
 * half, child1, is entered first — octant 7 is the reference's LIFO visit) */
__global__ __launch_bounds__(256) void k_orders(const LNode *__restrict__ nodes, int32_t g0, int32_t nn,
                                                const int32_t *__restrict__ size, int32_t *__restrict__ idx, int32_t n) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    const LNode nd = nodes[g0 + k];
    if (nd.child[0] < 0 && nd.child[1] < 0) return;
    for (int o = 0; o < kOrders; ++o) {
        const bool upper_first = o > 0 && (((o - 1) >> (nd.depth % 3)) & 1) != 0;
        const int32_t first = nd.child[upper_first ? 1 : 0], second = nd.child[upper_first ? 0 : 1];
        const int32_t me = idx[(int64_t)o * n + g0 + k];
        if (first >= 0) idx[(int64_t)o * n + first] = me + 1;
        if (second >= 0) idx[(int64_t)o * n + second] = me + 1 + (first >= 0 ? size[first] : 0);
    }
}

__global__ __launch_bounds__(256) void k_leaf_counts(const LNode *__restrict__ nodes, int32_t n,
                                                     const int32_t *__restrict__ idx_trav, const int32_t *__restrict__ idx_ref,
                                                     int32_t *__restrict__ cnt_trav, int64_t *__restrict__ cnt_ref,
                                                     int32_t *__restrict__ stats) {
    const int32_t x = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (x >= n) return;
    const LNode nd = nodes[x];
    const int32_t c = (nd.leaf && nd.count > 0) ? nd.count : 0;
    cnt_trav[idx_trav[x]] = c;
    cnt_ref[idx_ref[x]] = c;
    atomicMax(&stats[0], nd.depth);
    if (c > 0) {
        atomicAdd(&stats[1], 1);
        atomicMax(&stats[2], c);
    }
}

/* ---- hulls -------------------------------------------------------------- */
__global__ __launch_bounds__(256) void k_tri_hulls(const float *__restrict__ vpos, const DTriAttr *__restrict__ ta,
                                                   const float *__restrict__ fnorm, int64_t nt, double G,
                                                   HullD *__restrict__ th) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    const DTriAttr a = ta[t];
    float p0[3], p1[3], p2[3], fn[3];
    for (int k = 0; k < 3; ++k) {
        p0[k] = vpos[3 * (int64_t)a.i0 + k];
        p1[k] = vpos[3 * (int64_t)a.i1 + k];
        p2[k] = vpos[3 * (int64_t)a.i2 + k];
        fn[k] = fnorm[3 * t + k];
    }
    th[t] = triangle_hull(p0, p1, p2, fn, G);
}

__global__ __launch_bounds__(256) void k_node_hulls(const LNode *__restrict__ nodes, int32_t g0, int32_t nn,
                                                    const int32_t *__restrict__ pool, const HullD *__restrict__ th,
                                                    HullD *__restrict__ hull) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= nn) return;
    const LNode nd = nodes[g0 + k];
    HullD h;
    for (int a = 0; a < 3; ++a) { h.lo[a] = (double)INFINITY; h.hi[a] = -(double)INFINITY; }
    auto merge = [&](const HullD &o) {   /* std::min / std::max, as the host build */
        for (int a = 0; a < 3; ++a) {
            h.lo[a] = (o.lo[a] < h.lo[a]) ? o.lo[a] : h.lo[a];
            h.hi[a] = (h.hi[a] < o.hi[a]) ? o.hi[a] : h.hi[a];
        }
    };
    if (nd.leaf) {
        for (int32_t j = 0; j < nd.count; ++j) merge(th[pool[nd.begin + j]]);
    } else {
        for (int c = 0; c < 2; ++c)
            if (nd.child[c] >= 0) merge(hull[nd.child[c]]);
    }
    hull[g0 + k] = h;
}

/* ---- emission ----------------------------------------------------------- */
struct EmitArgs {
    const LNode *nodes;
    int32_t n;
    const int32_t *size, *idx;       /* idx: kOrders x n */
    const int32_t *slot_first_trav;  /* by traversal index */
    const int64_t *leaf_off_ref;     /* by reference index */
    const int32_t *pool;
    const HullD *hull;
    const float *vpos;
    const DTriAttr *ta;
    const float *fnorm;
    const uint8_t *tri_cull;
    DNode *dn;
    PNode *pn;
    DTriGeo *slots;
    int32_t *slot_tri;
    uint8_t *slot_cull;
    float *ref_bounds;
    int32_t *ref_children;
    int32_t *ref_leaf_tris;
    int32_t *planes_ok;
};

__global__ __launch_bounds__(256) void k_emit(EmitArgs A) {
    const int32_t x = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (x >= A.n) return;
    const LNode nd = A.nodes[x];
    const bool leaf = nd.leaf && nd.count > 0;
    const int32_t it = A.idx[(int64_t)8 * A.n + x];   /* traversal = octant 7 */
    const int32_t ir = A.idx[x];
    const int32_t first = leaf ? A.slot_first_trav[it] : 0;
    DNode d;
    d.lo_x = nd.lo[0]; d.lo_y = nd.lo[1]; d.lo_z = nd.lo[2];
    d.hi_x = nd.hi[0]; d.hi_y = nd.hi[1]; d.hi_z = nd.hi[2];
    if (leaf) {
        d.a = nd.count | (nd.depth << 24);
        d.b = first;
    } else {
        d.a = it + A.size[x];
        d.b = -(nd.depth + 1);
    }
    A.dn[it] = d;
    const HullD h = A.hull[x];
    for (int o = 0; o < 8; ++o) {
        const int32_t io = A.idx[(int64_t)(1 + o) * A.n + x];
        PNode p;
        p.lo_x = d.lo_x; p.lo_y = d.lo_y; p.lo_z = d.lo_z;
        p.hi_x = d.hi_x; p.hi_y = d.hi_y; p.hi_z = d.hi_z;
        p.a = leaf ? d.a : io + A.size[x];
        p.b = d.b;
        p.tlo_x = round_down(h.lo[0]); p.tlo_y = round_down(h.lo[1]); p.tlo_z = round_down(h.lo[2]);
        p.thi_x = round_up(h.hi[0]); p.thi_y = round_up(h.hi[1]); p.thi_z = round_up(h.hi[2]);
        p.depth = nd.depth;
        p.count = nd.leaf ? nd.count : 0;
        A.pn[(size_t)o * (size_t)(A.n + 1) + io] = p;
    }
    /* reference numbering */
    for (int k = 0; k < 3; ++k) {
        A.ref_bounds[6 * (int64_t)ir + k] = nd.lo[k];
        A.ref_bounds[6 * (int64_t)ir + 3 + k] = nd.hi[k];
    }
    for (int c = 0; c < 2; ++c)
        A.ref_children[2 * (int64_t)ir + c] = nd.child[c] >= 0 ? A.idx[nd.child[c]] : -1;
    if (leaf) {
        const int64_t ro = A.leaf_off_ref[ir];
        for (int32_t j = 0; j < nd.count; ++j) {
            const int32_t t = A.pool[nd.begin + j];
            const DTriAttr a = A.ta[t];
            DTriGeo g;
            g.v0x = A.vpos[3 * (int64_t)a.i0]; g.v0y = A.vpos[3 * (int64_t)a.i0 + 1]; g.v0z = A.vpos[3 * (int64_t)a.i0 + 2];
            g.v1x = A.vpos[3 * (int64_t)a.i1]; g.v1y = A.vpos[3 * (int64_t)a.i1 + 1]; g.v1z = A.vpos[3 * (int64_t)a.i1 + 2];
            g.v2x = A.vpos[3 * (int64_t)a.i2]; g.v2y = A.vpos[3 * (int64_t)a.i2 + 1]; g.v2z = A.vpos[3 * (int64_t)a.i2 + 2];
            g.nx = A.fnorm[3 * (int64_t)t]; g.ny = A.fnorm[3 * (int64_t)t + 1]; g.nz = A.fnorm[3 * (int64_t)t + 2];
            A.slots[first + j] = g;
            A.slot_tri[first + j] = t;
            A.slot_cull[first + j] = A.tri_cull[t];
            A.ref_leaf_tris[ro + j] = t;
        }
    }
    const float cs[6] = {d.lo_x, d.lo_y, d.lo_z, d.hi_x, d.hi_y, d.hi_z};
    bool ok = true;
    for (int k = 0; k < 6; ++k) ok = ok && coord_ok(cs[k]);
    ok = ok && d.lo_x <= d.hi_x && d.lo_y <= d.hi_y && d.lo_z <= d.hi_z;   /* ordered: crt_device.h in_slab */
    if (!ok) atomicAnd(A.planes_ok, 0);
}

__global__ __launch_bounds__(256) void k_cull_bits(const uint8_t *__restrict__ cull, int64_t m, uint32_t *__restrict__ bits,
                                                   int64_t words) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint32_t v = 0;
    for (int b = 0; b < 32; ++b) {
        const int64_t k = w * 32 + b;
        if (k < m && cull[k]) v |= 1u << b;
    }
    bits[w] = v;
}

inline unsigned grid_for(int64_t n, int block = 256) { return (unsigned)std::max<int64_t>(1, (n + block - 1) / block); }

template <class T>
int upload_vec(const std::vector<T> &v, T **dst, Scratch &tmp, hipStream_t st) {
    int rc = tmp.alloc(dst, v.size());
    if (rc != CRT_OK) return rc;
    if (!v.empty()) TB_TRY(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
    return CRT_OK;
}

/* device buffer that grows (copying its used prefix) */
template <class T>
struct Grow {
    T *p = nullptr;
    size_t cap = 0;
    ~Grow() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t need, size_t used, hipStream_t st) {
        if (need <= cap) return CRT_OK;
        const size_t nc = std::max(need, cap * 2);
        T *q = nullptr;
        TB_TRY(hipMalloc(&q, nc * sizeof(T)));
        if (used) TB_TRY(hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, st));
        TB_TRY(hipStreamSynchronize(st));
        if (p) (void)hipFree(p);
        p = q;
        cap = nc;
        return CRT_OK;
    }
};

}  // namespace

int build_tree_device(const HostScene &hs, void *stream_v, DeviceTree &out) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = static_cast<hipStream_t>(stream_v);
    const int64_t nt = (int64_t)hs.tri_attr.size();
    if (nt > (int64_t)std::numeric_limits<int32_t>::max() / 2) return set_error(CRT_E_UNSUPPORTED, "too many triangles");
    Scratch tmp;
    int rc;
    float *d_vpos = nullptr, *d_fn = nullptr;
    DTriAttr *d_ta = nullptr;
    uint8_t *d_cull = nullptr;
    if ((rc = upload_vec(hs.vpos, &d_vpos, tmp, st)) != CRT_OK) return rc;
    if ((rc = upload_vec(hs.tri_attr, &d_ta, tmp, st)) != CRT_OK) return rc;
    if ((rc = upload_vec(hs.face_normal, &d_fn, tmp, st)) != CRT_OK) return rc;
    if ((rc = upload_vec(hs.tri_cull, &d_cull, tmp, st)) != CRT_OK) return rc;

    Box6 *d_tb = nullptr;
    if ((rc = tmp.alloc(&d_tb, (size_t)nt)) != CRT_OK) return rc;
    Grow<LNode> nodes;
    Grow<int32_t> pool;
    if ((rc = nodes.reserve(1024, 0, st)) != CRT_OK) return rc;
    if ((rc = pool.reserve((size_t)std::max<int64_t>(nt, 1) * 4, 0, st)) != CRT_OK) return rc;
    if (nt > 0)
        hipLaunchKernelGGL(k_tri_boxes, dim3(grid_for(nt)), dim3(256), 0, st, d_vpos, d_ta, nt, d_tb, pool.p);
    TB_TRY(hipGetLastError());
    {
        LNode root;
        for (int k = 0; k < 3; ++k) { root.lo[k] = hs.root_box[k]; root.hi[k] = hs.root_box[3 + k]; }
        root.begin = 0;
        root.count = (int32_t)nt;
        root.depth = 0;
        root.child[0] = root.child[1] = -1;
        root.leaf = 0;
        root.pad = 0;
        TB_TRY(hipMemcpyAsync(nodes.p, &root, sizeof root, hipMemcpyHostToDevice, st));
    }
    std::vector<int32_t> lvl_off{0}, lvl_n{1};
    std::vector<int64_t> ids_off{0}, ids_n{nt};
    /* per-level scratch, grown to the largest level */
    Grow<uint64_t> flags, S;
    Grow<int32_t> node_of, nl, nr, ccount, cpos;
    Grow<int64_t> nbase;
    for (int L = 0;; ++L) {
        const int32_t nn = lvl_n[L], g0 = lvl_off[L];
        const int64_t nids = ids_n[L], ib = ids_off[L];
        LNode *lv = nodes.p + g0;
        hipLaunchKernelGGL(k_classify, dim3(grid_for(nn)), dim3(256), 0, st, lv, nn);
        if ((rc = flags.reserve((size_t)nids + 1, 0, st)) != CRT_OK) return rc;
        if ((rc = S.reserve((size_t)nids + 1, 0, st)) != CRT_OK) return rc;
        if ((rc = node_of.reserve((size_t)nids + 1, 0, st)) != CRT_OK) return rc;
        for (Grow<int32_t> *g : {&nl, &nr, &ccount, &cpos})
            if ((rc = g->reserve((size_t)nn + 1, 0, st)) != CRT_OK) return rc;
        if ((rc = nbase.reserve((size_t)nn + 1, 0, st)) != CRT_OK) return rc;
        if (nids > 0)
            hipLaunchKernelGGL(k_entry_flags, dim3(grid_for(nids)), dim3(256), 0, st, lv, nn, pool.p, ib, nids, d_tb,
                               flags.p, node_of.p);
        TB_TRY(hipGetLastError());
        if ((rc = scan_exclusive<uint64_t>(flags.p, S.p, nids, st, tmp)) != CRT_OK) return rc;
        hipLaunchKernelGGL(k_node_children, dim3(grid_for(nn)), dim3(256), 0, st, lv, nn, S.p, ib, nbase.p, nl.p, nr.p,
                           ccount.p);
        TB_TRY(hipGetLastError());
        if ((rc = scan_exclusive<int32_t>(ccount.p, cpos.p, nn, st, tmp)) != CRT_OK) return rc;
        int32_t nchild = 0;
        uint64_t stot = 0;
        TB_TRY(hipMemcpyAsync(&nchild, cpos.p + nn, sizeof nchild, hipMemcpyDeviceToHost, st));
        TB_TRY(hipMemcpyAsync(&stot, S.p + nids, sizeof stot, hipMemcpyDeviceToHost, st));
        TB_TRY(hipStreamSynchronize(st));
        const int64_t next_ids = (int64_t)(stot & 0xffffffffu) + (int64_t)(stot >> 32);
        if (nchild == 0) break;   /* every node of the level is a leaf; child links stay -1 */
        if ((int64_t)g0 + nn + nchild > (int64_t)std::numeric_limits<int32_t>::max())
            return set_error(CRT_E_UNSUPPORTED, "tree has too many nodes");
        if ((rc = nodes.reserve((size_t)g0 + nn + nchild, (size_t)g0 + nn, st)) != CRT_OK) return rc;
        if ((rc = pool.reserve((size_t)(ib + nids + next_ids), (size_t)(ib + nids), st)) != CRT_OK) return rc;
        lv = nodes.p + g0;
        hipLaunchKernelGGL(k_make_children, dim3(grid_for(nn)), dim3(256), 0, st, lv, nn, nbase.p, nl.p, nr.p, cpos.p,
                           nodes.p + g0 + nn, g0 + nn, ib + nids);
        TB_TRY(hipGetLastError());
        if (nids > 0)
            hipLaunchKernelGGL(k_scatter, dim3(grid_for(nids)), dim3(256), 0, st, lv, node_of.p, flags.p, S.p, pool.p, ib,
                               nids, nbase.p, nl.p, pool.p + ib + nids);
        TB_TRY(hipGetLastError());
        lvl_off.push_back(g0 + nn);
        lvl_n.push_back(nchild);
        ids_off.push_back(ib + nids);
        ids_n.push_back(next_ids);
    }
    const int levels = (int)lvl_n.size();
    const int32_t n = lvl_off.back() + lvl_n.back();

    /* subtree sizes (bottom up), the nine orders (top down) */
    int32_t *d_size = nullptr, *d_idx = nullptr;
    if ((rc = tmp.alloc(&d_size, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_idx, (size_t)kOrders * n)) != CRT_OK) return rc;
    for (int L = levels - 1; L >= 0; --L)
        hipLaunchKernelGGL(k_sizes, dim3(grid_for(lvl_n[L])), dim3(256), 0, st, nodes.p, lvl_off[L], lvl_n[L], d_size);
    TB_TRY(hipGetLastError());
    for (int o = 0; o < kOrders; ++o) TB_TRY(hipMemsetAsync(d_idx + (size_t)o * n, 0, sizeof(int32_t), st));   /* root = 0 */
    for (int L = 0; L < levels; ++L)
        hipLaunchKernelGGL(k_orders, dim3(grid_for(lvl_n[L])), dim3(256), 0, st, nodes.p, lvl_off[L], lvl_n[L], d_size,
                           d_idx, n);
    TB_TRY(hipGetLastError());

    /* leaf slot offsets (traversal order) and reference leaf offsets */
    int32_t *d_cnt_trav = nullptr, *d_first_trav = nullptr, *d_stats = nullptr;
    int64_t *d_cnt_ref = nullptr;
    if ((rc = tmp.alloc(&d_cnt_trav, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_first_trav, (size_t)n + 1)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_cnt_ref, (size_t)n)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_stats, 4)) != CRT_OK) return rc;
    TB_TRY(hipMemsetAsync(d_stats, 0, 4 * sizeof(int32_t), st));
    hipLaunchKernelGGL(k_leaf_counts, dim3(grid_for(n)), dim3(256), 0, st, nodes.p, n, d_idx + (size_t)8 * n, d_idx,
                       d_cnt_trav, d_cnt_ref, d_stats);
    TB_TRY(hipGetLastError());
    if ((rc = scan_exclusive<int32_t>(d_cnt_trav, d_first_trav, n, st, tmp)) != CRT_OK) return rc;

    /* outputs (owned by the caller) */
    auto keep = [&](auto **p, size_t count) -> int {
        void *q = nullptr;
        TB_TRY(hipMalloc(&q, std::max<size_t>(1, count) * sizeof(**p)));
        out.allocs.push_back(q);
        *p = static_cast<std::remove_reference_t<decltype(*p)>>(q);
        return CRT_OK;
    };
    int32_t stats[4] = {0, 0, 0, 0}, slots_total = 0;
    TB_TRY(hipMemcpyAsync(stats, d_stats, sizeof stats, hipMemcpyDeviceToHost, st));
    TB_TRY(hipMemcpyAsync(&slots_total, d_first_trav + n, sizeof slots_total, hipMemcpyDeviceToHost, st));
    TB_TRY(hipStreamSynchronize(st));
    if (stats[2] >= (1 << 24) || stats[0] > 127) return set_error(CRT_E_UNSUPPORTED, "leaf too large for the node record");
    const int64_t m = slots_total;
    if ((rc = keep(&out.ref_leaf_off, (size_t)n + 1)) != CRT_OK) return rc;
    if ((rc = scan_exclusive<int64_t>(d_cnt_ref, out.ref_leaf_off, n, st, tmp)) != CRT_OK) return rc;

    HullD *d_th = nullptr, *d_hull = nullptr;
    if ((rc = tmp.alloc(&d_th, (size_t)nt)) != CRT_OK) return rc;
    if ((rc = tmp.alloc(&d_hull, (size_t)n)) != CRT_OK) return rc;
    if (nt > 0)
        hipLaunchKernelGGL(k_tri_hulls, dim3(grid_for(nt)), dim3(256), 0, st, d_vpos, d_ta, d_fn, nt, hs.prune_G, d_th);
    for (int L = levels - 1; L >= 0; --L)
        hipLaunchKernelGGL(k_node_hulls, dim3(grid_for(lvl_n[L])), dim3(256), 0, st, nodes.p, lvl_off[L], lvl_n[L],
                           pool.p, d_th, d_hull);
    TB_TRY(hipGetLastError());

    if ((rc = keep(&out.nodes, (size_t)n)) != CRT_OK) return rc;
    if ((rc = keep(&out.pnodes, (size_t)8 * (n + 1))) != CRT_OK) return rc;
    TB_TRY(hipMemsetAsync(out.pnodes, 0, (size_t)8 * (n + 1) * sizeof(PNode), st));
    if ((rc = keep(&out.slots, (size_t)m)) != CRT_OK) return rc;
    if ((rc = keep(&out.slot_tri, (size_t)m)) != CRT_OK) return rc;
    if ((rc = keep(&out.slot_cull, (size_t)m)) != CRT_OK) return rc;
    const int64_t words = (m + 31) / 32 + 1;
    if ((rc = keep(&out.slot_cull_bits, (size_t)words)) != CRT_OK) return rc;
    if ((rc = keep(&out.ref_bounds, (size_t)n * 6)) != CRT_OK) return rc;
    if ((rc = keep(&out.ref_children, (size_t)n * 2)) != CRT_OK) return rc;
    if ((rc = keep(&out.ref_leaf_tris, (size_t)m)) != CRT_OK) return rc;
    int32_t *d_planes = nullptr;
    if ((rc = tmp.alloc(&d_planes, 1)) != CRT_OK) return rc;
    const int32_t one = 1;
    TB_TRY(hipMemcpyAsync(d_planes, &one, sizeof one, hipMemcpyHostToDevice, st));
    EmitArgs A;
    A.nodes = nodes.p; A.n = n; A.size = d_size; A.idx = d_idx; A.slot_first_trav = d_first_trav;
    A.leaf_off_ref = out.ref_leaf_off; A.pool = pool.p; A.hull = d_hull; A.vpos = d_vpos; A.ta = d_ta; A.fnorm = d_fn;
    A.tri_cull = d_cull; A.dn = out.nodes; A.pn = out.pnodes; A.slots = out.slots; A.slot_tri = out.slot_tri;
    A.slot_cull = out.slot_cull; A.ref_bounds = out.ref_bounds; A.ref_children = out.ref_children;
    A.ref_leaf_tris = out.ref_leaf_tris; A.planes_ok = d_planes;
    hipLaunchKernelGGL(k_emit, dim3(grid_for(n)), dim3(256), 0, st, A);
    TB_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_cull_bits, dim3(grid_for(words)), dim3(256), 0, st, out.slot_cull, m, out.slot_cull_bits, words);
    TB_TRY(hipGetLastError());
    int32_t planes = 1;
    TB_TRY(hipMemcpyAsync(&planes, d_planes, sizeof planes, hipMemcpyDeviceToHost, st));
    TB_TRY(hipStreamSynchronize(st));
    out.node_count = n;
    out.slot_count = m;
    out.max_depth = stats[0];
    out.leaf_count = stats[1];
    out.max_leaf_size = stats[2];
    out.planes_ok = planes;
    out.levels = levels;
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

}  // namespace crt_amd
