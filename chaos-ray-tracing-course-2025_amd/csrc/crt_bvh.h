/*
 * crt_bvh.h — exact closest hit of one scattered ray through a BVH over the
 * scene's triangles, checked against the reference's tree (host and device).
 *
 * What the reference computes (crt_intersection.cpp:109-136): among the leaf
 * copies of triangles whose leaf is reached — every node on the path from the
 * root passes the six-face test (ray_intersect_aabb_p, :14-45) — the hit with
 * the smallest t, ties going to the first copy in visit order.  Copies of one
 * triangle hold the same vertices, normal and flags (crt_acceleration_tree.cpp
 * :44-58 copies the Triangle), so they hit at the same t with the same record;
 * the copy only matters between *different* triangles hitting at equal t.
 *
 * Scattered rays (GI bounces, reflections, refractions) cross many cells of
 * the median-split tree and test the big triangles its leaves duplicate again
 * and again (15-01/scene2: 30,572 copies of 2,012 triangles; a GI ray tests
 * ~32 nodes and ~38 copies in the reference's order).  Here:
 *
 *   1. walk_bvh: closest hit over ALL triangles, each once, through a BVH
 *      whose boxes are unions of the triangles' conservative hulls (the hulls
 *      of the pruned kd walks, crt_scene_build.cpp: a box misses the ray
 *      before `lim` only if no triangle inside can produce a reference hit
 *      with t <= lim).  Result: t* = the smallest t the reference's triangle
 *      test accepts for any triangle, the triangle T* that gives it, and
 *      whether another triangle gives the same t (a tie);
 *   2. verify_kd: T* must have a copy the reference reaches.  The walk
 *      descends the reference tree from the root towards the hit point
 *      p = o + d t* (the child whose cell holds p), running the reference's
 *      six-face test on every node of the path; it succeeds when every test
 *      passes and the leaf holds a copy of T*.  Then that copy is eligible
 *      and no eligible copy can hit nearer (t* is the minimum over all
 *      triangles), and no other triangle ties: the reference's answer is T*
 *      at t*, bit for bit (same record from any copy);
 *   3. otherwise (a tie, or a path test failing — rounding at cell edges)
 *      the exact pruned kd walk (crt_device.h walk_pruned) decides.
 *
 * All loads go through CRT_LDG (global loads on the device). */
#pragma once
#include "crt_device.h"

#ifndef CRT_PROOF_TOPO
#define CRT_PROOF_TOPO 1     /* 0: the proof descends the 32-B nodes (verify_kd) even where KTopo exists */
#endif
#ifndef CRT_BVH_PREFETCH
#define CRT_BVH_PREFETCH 1   /* walk_bvh: 0 none, 1 both successor nodes, 2 + the node's first triangle, 3 + its second */
#endif
#ifndef CRT_WALK_HOOK
#define CRT_WALK_HOOK()        /* diagnostic builds: after step 1 (crt_render_wf.hip CRT_WF_STAMPS) */
#endif
#ifndef CRT_FALLBACK_HOOK
#define CRT_FALLBACK_HOOK()    /* diagnostic builds: when step 3 runs */
#endif
#ifndef CRT_PROOF_TOPO2
#define CRT_PROOF_TOPO2 1    /* 0: the proof's descent loads one KTopo a level even where KTopo2 exists */
#endif

namespace crt_amd {

#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
__device__ __forceinline__ T crt_ldg(const T *p, int64_t i) {
    using GT = const __attribute__((address_space(1))) T;
    return ((GT *)p)[i];
}
#define CRT_LDG(p, i) crt_ldg((p), (int64_t)(i))
#else
#define CRT_LDG(p, i) ((p)[i])
#endif

CRT_HD const BNode *bnode_order(const BNode *base, int node_count, int oct) {
    return base + (size_t)oct * (size_t)(node_count + 1);
}

/* hull_alive (crt_device.h) on a BVH box: false only when the ray cannot hit
 * any triangle inside at t <= lim (NaN bounds keep the box) */
CRT_HD bool bnode_alive(const BNode &n, const PruneRay &p, float lim) {
    const float t0x = fmaf(n.lo_x, p.ix, p.cx), t1x = fmaf(n.hi_x, p.ix, p.cx);
    const float t0y = fmaf(n.lo_y, p.iy, p.cy), t1y = fmaf(n.hi_y, p.iy, p.cy);
    const float t0z = fmaf(n.lo_z, p.iz, p.cz), t1z = fmaf(n.hi_z, p.iz, p.cz);
    const float tin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tout = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return !p.on || (!(tin > lim) && !(tin > tout) && !(tout < 0.0f));
}

/* Step 1: closest reference hit over all triangles.  Returns the triangle id
 * (-1: no triangle is hit), its t, and tie = another triangle hits at the
 * same t (each triangle is in the BVH once, so an equal t is another one). */
template <bool COUNT, int PF = CRT_BVH_PREFETCH>
CRT_HD int walk_bvh(const BNode *nodes, int n, const DTriGeo *geo, const int32_t *tid, Vec o, Vec d,
                    const PruneRay &pr, float &best_t, bool &tie, WalkCounts &c) {
    int best = -1;
    float lim = INFINITY;
    best_t = 0.0f;
    tie = false;
    int i = 0;
    /* PF: both possible successors (i + 1, skip) are loaded before the node is
     * tested: the walk is a chain of dependent loads, and each step's test
     * then overlaps the next step's load (every order ends with a zero
     * record, so i + 1 <= n and skip <= n are always in bounds).  Pays on
     * scattered rays (C3); the coherent camera rays of C2 walk without it.
     * PF 2: the node's first triangle too (an interior node's leaf field is 0:
     * triangle 0, a valid address), so an alive leaf costs no extra load. */
    BNode cur, n1, n2;
    DTriGeo g0, g1;
    int32_t id0 = 0, id1 = 0;
    if constexpr (PF > 0) cur = CRT_LDG(nodes, 0);
    while (i < n) {
        BNode nd;
        if constexpr (PF > 0) {
            nd = cur;
            n1 = CRT_LDG(nodes, i + 1);
            n2 = CRT_LDG(nodes, nd.skip);
            if constexpr (PF > 1) {
                g0 = CRT_LDG(geo, nd.leaf >> 4);
                id0 = CRT_LDG(tid, nd.leaf >> 4);
            }
            if constexpr (PF > 2) {   /* and its second (a one-triangle leaf: the next leaf's first, in bounds) */
                const int f1 = (nd.leaf >> 4) + ((nd.leaf & 15) > 1 ? 1 : 0);
                g1 = CRT_LDG(geo, f1);
                id1 = CRT_LDG(tid, f1);
            }
        } else {
            nd = CRT_LDG(nodes, i);
        }
        if (COUNT) ++c.nodes;
        if (!bnode_alive(nd, pr, lim)) {
            i = nd.skip;
            if constexpr (PF > 0) cur = n2;
            continue;
        }
        ++i;                                   /* interior: first child; leaf: next in preorder */
        if constexpr (PF > 0) cur = n1;
        const int cnt = nd.leaf & 15;
        const int first = nd.leaf >> 4;
        for (int k = 0; k < cnt; ++k) {
            DTriGeo g;
            int32_t id;
            if (PF > 1 && k == 0) {
                g = g0;
                id = id0;
            } else if (PF > 2 && k == 1) {
                g = g1;
                id = id1;
            } else {
                g = CRT_LDG(geo, first + k);
                id = CRT_LDG(tid, first + k);
            }
            const uint8_t cull = (uint8_t)((uint32_t)id >> 31);
            float t;
            if (COUNT) ++c.tris;
            if (tri_hit(o, d, g, &cull, t)) {
                if (best < 0 || t < best_t) {
                    best_t = t;
                    best = id & 0x7fffffff;
                    tie = false;
                    lim = t;
                } else if (t == best_t) {
                    tie = true;
                }
            }
        }
    }
    return best;
}

/* p inside the cell, inclusive (the reference's cell bounds) */
CRT_HD bool cell_holds(const DNode &nd, Vec p) {
    return p.x >= nd.lo_x && p.x <= nd.hi_x && p.y >= nd.lo_y && p.y <= nd.hi_y && p.z >= nd.lo_z && p.z <= nd.hi_z;
}

/* How far p lies outside the cell (max over axes; 0 inside, NaN-free for a
 * finite p): the descent's choice between two children when rounding put p
 * in neither (a hit on a wall that is also the root cell's face). */
CRT_HD float cell_excess(const DNode &nd, Vec p) {
    const float ex = fmaxf(nd.lo_x - p.x, p.x - nd.hi_x), ey = fmaxf(nd.lo_y - p.y, p.y - nd.hi_y);
    const float ez = fmaxf(nd.lo_z - p.z, p.z - nd.hi_z);
    return fmaxf(fmaxf(ex, ey), fmaxf(ez, 0.0f));
}

/* The six face predicates of ray_intersect_aabb_p (crt_intersection.cpp:
 * 14-45) as bits (lo x, lo y, lo z, hi x, hi y, hi z): their OR is
 * box_hit_r — the same arithmetic, face by face. */
CRT_HD unsigned box_faces(Vec o, Vec d, const RayRcp &r, const DNode &n) {
    if (r.fast) {
        f2 px, qx, py, qy, pz, qz;
        axis_points((f2){n.lo_x, n.hi_x}, o.x, d.x, r.y1[0], o.y, d.y, o.z, d.z, px, qx);
        axis_points((f2){n.lo_y, n.hi_y}, o.y, d.y, r.y1[1], o.z, d.z, o.x, d.x, py, qy);
        axis_points((f2){n.lo_z, n.hi_z}, o.z, d.z, r.y1[2], o.x, d.x, o.y, d.y, pz, qz);
        unsigned m = 0u;
        m |= (in_slab(px.x, n.lo_y, n.hi_y) && in_slab(qx.x, n.lo_z, n.hi_z)) ? 1u : 0u;
        m |= (in_slab(py.x, n.lo_z, n.hi_z) && in_slab(qy.x, n.lo_x, n.hi_x)) ? 2u : 0u;
        m |= (in_slab(pz.x, n.lo_x, n.hi_x) && in_slab(qz.x, n.lo_y, n.hi_y)) ? 4u : 0u;
        m |= (in_slab(px.y, n.lo_y, n.hi_y) && in_slab(qx.y, n.lo_z, n.hi_z)) ? 8u : 0u;
        m |= (in_slab(py.y, n.lo_z, n.hi_z) && in_slab(qy.y, n.lo_x, n.hi_x)) ? 16u : 0u;
        m |= (in_slab(pz.y, n.lo_x, n.hi_x) && in_slab(qz.y, n.lo_y, n.hi_y)) ? 32u : 0u;
        return m;
    }
    const float t0 = (n.lo_x - o.x) / d.x, t1 = (n.lo_y - o.y) / d.y, t2 = (n.lo_z - o.z) / d.z;
    const float t3 = (n.hi_x - o.x) / d.x, t4 = (n.hi_y - o.y) / d.y, t5 = (n.hi_z - o.z) / d.z;
    return (face_ok(t0, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) ? 1u : 0u) |
           (face_ok(t1, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) ? 2u : 0u) |
           (face_ok(t2, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y) ? 4u : 0u) |
           (face_ok(t3, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) ? 8u : 0u) |
           (face_ok(t4, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) ? 16u : 0u) |
           (face_ok(t5, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y) ? 32u : 0u);
}

CRT_HD float cell_plane(const DNode &n, int f) {
    switch (f) {
    case 0: return n.lo_x;
    case 1: return n.lo_y;
    case 2: return n.lo_z;
    case 3: return n.hi_x;
    case 4: return n.hi_y;
    default: return n.hi_z;
    }
}

/* Step 2: a copy of triangle `tri` the reference reaches, on the path towards
 * p through the reference-order DNode array (crt_layout.h: interior node i's
 * first child is i + 1, its second child, if any, starts where the first
 * one's subtree ends, before skip(i)).  Returns its slot, or -1.
 *
 * Every node on the path must pass the six-face test.  A node's cell holds
 * its descendants' cells, so when the leaf L passes through face f and an
 * ancestor A has the same plane on f, A's face f computes the same t and hit
 * point and checks it against a larger rectangle: A passes.  A child differs
 * from its parent in one plane, so face f's plane is shared by L and every
 * ancestor at or below the depth D_f where it was last set; the ancestors
 * above min D_f over L's passing faces are tested in full (usually the root
 * at most). */
template <bool COUNT>
CRT_HD int verify_kd(const DNode *nodes, const int32_t *slot_tri, int tri, Vec o, Vec d, const RayRcp &rr,
                     Vec p, WalkCounts &c) {
    int i = 0, depth = 0;
    uint64_t choice = 0;                       /* bit k: level k took the second child */
    int df[6] = {0, 0, 0, 0, 0, 0};            /* depth where each face's plane was last set */
    DNode nd = CRT_LDG(nodes, 0);
    while (nd.b < 0) {
        const int c1 = i + 1;
        const DNode n1 = CRT_LDG(nodes, c1);
        const int c2 = n1.b < 0 ? n1.a : c1 + 1;
        int ci = c1;
        DNode ch = n1;
        if (c2 < nd.a && !cell_holds(n1, p)) {   /* two children, p not in the first */
            const DNode n2 = CRT_LDG(nodes, c2);
            if (cell_holds(n2, p) || cell_excess(n2, p) < cell_excess(n1, p)) {
                ci = c2;
                ch = n2;
                choice |= 1ull << depth;
            }
        }
        ++depth;
        if (depth > 62) return -1;
        for (int f = 0; f < 6; ++f)
            if (!(cell_plane(ch, f) == cell_plane(nd, f))) df[f] = depth;
        i = ci;
        nd = ch;
    }
    int slot = -1;
    const int cnt = node_leaf_count(nd);
    for (int k = 0; k < cnt && slot < 0; ++k)
        if (CRT_LDG(slot_tri, nd.b + k) == tri) slot = nd.b + k;
    if (slot < 0) return -1;
    if (COUNT) ++c.nodes;
    const unsigned m = box_faces(o, d, rr, nd);
    if (m == 0u) return -1;
    int dmin = depth;
    for (int f = 0; f < 6; ++f)
        if ((m >> f) & 1u) dmin = df[f] < dmin ? df[f] : dmin;
    /* ancestors above dmin: full tests, replaying the descent's choices */
    i = 0;
    nd = CRT_LDG(nodes, 0);
    for (int k = 0; k < dmin; ++k) {
        if (COUNT) ++c.nodes;
        if (!box_hit_r(o, d, rr, nd)) return -1;
        const int c1 = i + 1;
        const DNode n1 = CRT_LDG(nodes, c1);
        if ((choice >> k) & 1ull) {
            i = n1.b < 0 ? n1.a : c1 + 1;
            nd = CRT_LDG(nodes, i);
        } else {
            i = c1;
            nd = n1;
        }
    }
    return slot;
}

/* The two halves of a cell on axis AX (AX = depth % 3, a template
 * parameter so no field is selected by a run-time index; AABB::split,
 * crt_aabb.h:24-35: the reference's child cells, the same fp32 operations,
 * so the same bits). */
template <int AX>
CRT_HD void topo_halves(const DNode &c, DNode &lo, DNode &hi) {
    lo = c;
    hi = c;
    if constexpr (AX == 0) {
        const float m = (c.lo_x + c.hi_x) * 0.5f;
        lo.hi_x = m;
        hi.lo_x = m;
    } else if constexpr (AX == 1) {
        const float m = (c.lo_y + c.hi_y) * 0.5f;
        lo.hi_y = m;
        hi.lo_y = m;
    } else {
        const float m = (c.lo_z + c.hi_z) * 0.5f;
        lo.hi_z = m;
        hi.lo_z = m;
    }
}

CRT_HD void topo_halves(const DNode &c, int axis, DNode &lo, DNode &hi) {   /* host build check */
    if (axis == 0) topo_halves<0>(c, lo, hi);
    else if (axis == 1) topo_halves<1>(c, lo, hi);
    else topo_halves<2>(c, lo, hi);
}

/* c ? a : b field by field (a struct-valued ?: can become a select of two
 * stack addresses) */
CRT_HD DNode cell_sel(bool c, const DNode &a, const DNode &b) {
    DNode r;
    r.lo_x = c ? a.lo_x : b.lo_x;
    r.hi_x = c ? a.hi_x : b.hi_x;
    r.lo_y = c ? a.lo_y : b.lo_y;
    r.hi_y = c ? a.hi_y : b.hi_y;
    r.lo_z = c ? a.lo_z : b.lo_z;
    r.hi_z = c ? a.hi_z : b.hi_z;
    r.a = c ? a.a : b.a;
    r.b = c ? a.b : b.b;
    return r;
}

/* bit-identical cells (build-time check of the halving) */
CRT_HD bool cell_equal(const DNode &a, const DNode &b) {
    return __builtin_bit_cast(uint32_t, a.lo_x) == __builtin_bit_cast(uint32_t, b.lo_x) &&
           __builtin_bit_cast(uint32_t, a.hi_x) == __builtin_bit_cast(uint32_t, b.hi_x) &&
           __builtin_bit_cast(uint32_t, a.lo_y) == __builtin_bit_cast(uint32_t, b.lo_y) &&
           __builtin_bit_cast(uint32_t, a.hi_y) == __builtin_bit_cast(uint32_t, b.hi_y) &&
           __builtin_bit_cast(uint32_t, a.lo_z) == __builtin_bit_cast(uint32_t, b.lo_z) &&
           __builtin_bit_cast(uint32_t, a.hi_z) == __builtin_bit_cast(uint32_t, b.hi_z);
}

/* One level of verify_topo's descent on axis AX: false at a leaf. */
struct TopoWalk {
    DNode cell;
    KTopo tp;
    int i, depth;
    uint64_t upper;   /* bit k: level k went to the upper half */
    uint64_t df;      /* byte f: depth where face f's plane was last set */
};

template <int AX>
CRT_HD bool topo_level(const KTopo *topo, Vec p, TopoWalk &w) {
    if (w.tp.b >= 0 || w.depth >= 62) return false;   /* verify_kd: no level below 62 */
    DNode lo, hi;
    topo_halves<AX>(w.cell, lo, hi);
    const bool first_up = w.tp.b == -2;        /* the first child (i + 1) is the upper half */
    const DNode n1 = cell_sel(first_up, hi, lo), n2 = cell_sel(first_up, lo, hi);
    int ci = w.i + 1;
    bool up = first_up;
    if (w.tp.a >= 0 && !cell_holds(n1, p)) {   /* two children, p not in the first */
        if (cell_holds(n2, p) || cell_excess(n2, p) < cell_excess(n1, p)) {
            ci = w.tp.a;
            up = !first_up;
        }
    }
    if (up) w.upper |= 1ull << w.depth;
    ++w.depth;
    /* only the split plane changes: lo[AX] (face AX) going up, hi[AX] (face 3 + AX) going down */
    const float old = up ? cell_plane(w.cell, AX) : cell_plane(w.cell, 3 + AX);
    const float mid = up ? cell_plane(hi, AX) : cell_plane(lo, 3 + AX);
    const int f = up ? AX : 3 + AX;
    if (!(mid == old)) w.df = (w.df & ~(0xffull << (8 * f))) | ((uint64_t)w.depth << (8 * f));
    w.cell = cell_sel(up, hi, lo);
    w.i = ci;
    w.tp = CRT_LDG(topo, ci);
    return true;
}

/* KTopo2 entry LO + k, k < N (N a power of two): a tree of selects on the
 * record's registers (a dynamic index would put the record in scratch) */
template <int LO, int N>
CRT_HD KTopo topo2_pick(const KTopo2 &r, int k) {
    if constexpr (N == 1) {
        (void)k;
        return r.t[LO];
    } else {
        const KTopo a = topo2_pick<LO, N / 2>(r, k), b = topo2_pick<LO + N / 2, N / 2>(r, k);
        const bool hi = (k & (N / 2)) != 0;
        return KTopo{hi ? b.a : a.a, hi ? b.b : a.b};
    }
}

/* topo_level with the child's record from the node's KTopo2 (r, loaded at
 * the treelet's root; q: the current node's heap position there, LV its
 * level below the root + 1) instead of a load */
template <int AX, int LV>
CRT_HD bool topo_level2(const KTopo2 &r, int &q, Vec p, TopoWalk &w) {
    if (w.tp.b >= 0 || w.depth >= 62) return false;
    DNode lo, hi;
    topo_halves<AX>(w.cell, lo, hi);
    const bool first_up = w.tp.b == -2;
    const DNode n1 = cell_sel(first_up, hi, lo), n2 = cell_sel(first_up, lo, hi);
    int ci = w.i + 1;
    bool up = first_up, second = false;
    if (w.tp.a >= 0 && !cell_holds(n1, p)) {
        if (cell_holds(n2, p) || cell_excess(n2, p) < cell_excess(n1, p)) {
            ci = w.tp.a;
            up = !first_up;
            second = true;
        }
    }
    if (up) w.upper |= 1ull << w.depth;
    ++w.depth;
    const float old = up ? cell_plane(w.cell, AX) : cell_plane(w.cell, 3 + AX);
    const float mid = up ? cell_plane(hi, AX) : cell_plane(lo, 3 + AX);
    const int f = up ? AX : 3 + AX;
    if (!(mid == old)) w.df = (w.df & ~(0xffull << (8 * f))) | ((uint64_t)w.depth << (8 * f));
    w.cell = cell_sel(up, hi, lo);
    w.i = ci;
    q = 2 * q + (second ? 1 : 0);
    /* level LV's entries: positions 2^LV .. 2^(LV+1) - 1, entries from 2^LV - 2 */
    w.tp = topo2_pick<(1 << LV) - 2, (1 << LV)>(r, q - (1 << LV));
    return true;
}

/* Step 2 on the topology records (crt_layout.h KTopo): verify_kd's descent
 * and proof with the cells computed in registers — one dependent 8-B load
 * per level (verify_kd: one or two 32-B loads), and the full tests of the
 * ancestors above dmin replay the path from the root cell with no load.
 * Levels go three at a time (axes 0, 1, 2). */
template <bool COUNT>
CRT_HD int verify_topo(const KTopo *topo, const DNode *nodes, const int32_t *slot_tri, int tri, Vec o, Vec d,
                       const RayRcp &rr, Vec p, WalkCounts &c, const KTopo2 *topo2 = nullptr) {
    TopoWalk w;
    w.cell = CRT_LDG(nodes, 0);                /* the root cell */
    w.tp = CRT_LDG(topo, 0);
    w.i = 0;
    w.depth = 0;
    w.upper = 0;
    w.df = 0;
    if (topo2) {   /* two levels a load (the axes cycle with depth: six levels a round) */
        for (;;) {
            KTopo2 r;
            int q;
#define CRT_TOPO2_PAIR(A0, A1)                                                                     \
    if (w.tp.b >= 0 || w.depth >= 62) break;                                                       \
    r = CRT_LDG(topo2, w.i);                                                                       \
    q = 1;                                                                                         \
    if (!(topo_level2<A0, 1>(r, q, p, w) && topo_level2<A1, 2>(r, q, p, w))) break;
            CRT_TOPO2_PAIR(0, 1)
            CRT_TOPO2_PAIR(2, 0)
            CRT_TOPO2_PAIR(1, 2)
#undef CRT_TOPO2_PAIR
        }
    } else {
        while (topo_level<0>(topo, p, w) && topo_level<1>(topo, p, w) && topo_level<2>(topo, p, w)) {
        }
    }
    if (w.tp.b < 0) return -1;                 /* an interior node at depth 62 */
    int slot = -1;
    for (int k = 0; k < w.tp.a && slot < 0; ++k)
        if (CRT_LDG(slot_tri, w.tp.b + k) == tri) slot = w.tp.b + k;
    if (slot < 0) return -1;
    if (COUNT) ++c.nodes;
    const unsigned m = box_faces(o, d, rr, w.cell);
    if (m == 0u) return -1;
    int dmin = w.depth;
#pragma unroll
    for (int f = 0; f < 6; ++f)
        if ((m >> f) & 1u) {
            const int df = (int)((w.df >> (8 * f)) & 0xffull);
            dmin = df < dmin ? df : dmin;
        }
    /* ancestors above dmin: full tests on the cells of the path, from the root */
    DNode a = CRT_LDG(nodes, 0);
    for (int k = 0; k < dmin; k += 3) {
        DNode lo, hi;
        if (COUNT) ++c.nodes;
        if (!box_hit_r(o, d, rr, a)) return -1;
        if (k + 1 >= dmin) break;
        topo_halves<0>(a, lo, hi);
        a = cell_sel(((w.upper >> k) & 1ull) != 0ull, hi, lo);
        if (COUNT) ++c.nodes;
        if (!box_hit_r(o, d, rr, a)) return -1;
        if (k + 2 >= dmin) break;
        topo_halves<1>(a, lo, hi);
        a = cell_sel(((w.upper >> (k + 1)) & 1ull) != 0ull, hi, lo);
        if (COUNT) ++c.nodes;
        if (!box_hit_r(o, d, rr, a)) return -1;
        topo_halves<2>(a, lo, hi);
        a = cell_sel(((w.upper >> (k + 2)) & 1ull) != 0ull, hi, lo);
    }
    return slot;
}

/* Step 1 over a camera cell's candidate list (crt_layout.h CamCand) instead
 * of the BVH: the same closest triangle, t and tie flag as walk_bvh for any
 * camera ray of the cell.  Every triangle the ray can hit is in the list
 * (crt_bvh_build.cpp build_camera_bins); a candidate whose hull the ray
 * misses before lim cannot hit at t <= lim (bnode_alive, as walk_bvh's
 * boxes); the list is sorted by dmin, a lower bound of any accepted t, so
 * once dmin > best t no later candidate can hit at t <= best t — not even
 * tie; a candidate whose pixel mask lacks the ray's pixel (bit = 8 y + x in
 * the cell) cannot be hit by it, and once no later one has the pixel
 * (rest) the walk is over. */
CRT_HD bool cand_alive(const CamCand &c, const PruneRay &p, float lim) {
    BNode n;
    n.lo_x = c.lo_x; n.hi_x = c.hi_x; n.lo_y = c.lo_y; n.hi_y = c.hi_y; n.lo_z = c.lo_z; n.hi_z = c.hi_z;
    n.skip = 0;
    n.leaf = 0;
    return bnode_alive(n, p, lim);
}

/* one candidate into the running (best, t, tie, lim) of walk_bvh; true when
 * the triangle test ran */
CRT_HD bool cand_test(const CamCand &c, Vec o, Vec d, const PruneRay &pr, int &best, float &best_t, bool &tie,
                      float &lim) {
    if (!cand_alive(c, pr, lim)) return false;
    const uint8_t cull = (uint8_t)((uint32_t)c.id >> 31);
    float t;
    if (tri_hit(o, d, c.g, &cull, t)) {
        if (best < 0 || t < best_t) {
            best_t = t;
            best = c.id & 0x7fffffff;
            tie = false;
            lim = t;
        } else if (t == best_t) {
            tie = true;
        }
    }
    return true;
}

/* cand_test's verdict without branches (for interleaved tests): the
 * triangle test's conjuncts exactly as tri_hit orders them (crt_device.h,
 * crt_intersection.cpp:47-93) and the hull against lim; t valid when true. */
CRT_HD bool cand_hit_bf(const CamCand &c, Vec o, Vec d, const PruneRay &pr, float lim, float &t) {
    const DTriGeo &g = c.g;
    const Vec N = vec(g.nx, g.ny, g.nz);
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z), v1 = vec(g.v1x, g.v1y, g.v1z), v2 = vec(g.v2x, g.v2y, g.v2z);
    const float rn = vdot(N, d);
    const float op = vdot(N, vsub(v0, o));
    const bool cull = ((uint32_t)c.id >> 31) != 0u;
    t = op / rn;
    const Vec e0 = vsub(v1, v0), e1 = vsub(v2, v1), e2 = vsub(v0, v2);
    const Vec p = vadd(o, vscale(d, t));
    const Vec v0p = vsub(p, v0), v1p = vsub(p, v1), v2p = vsub(p, v2);
    return (int)cand_alive(c, pr, lim) & (int)!(fabsf(rn) < 1e-6f) & (int)((op < 0.0f) | !cull) &
           (int)!(opposite_signs(op, rn) && fabsf(rn) < 2.0f) & (int)!(t < 0.0f) &
           (int)(vdot(N, vcross(e0, v0p)) >= 0.0f) & (int)(vdot(N, vcross(e1, v1p)) >= 0.0f) &
           (int)(vdot(N, vcross(e2, v2p)) >= 0.0f);
}

template <bool COUNT>
CRT_HD int walk_bins(const CamCand *cands, int beg, int end, int bit, Vec o, Vec d, const PruneRay &pr, float &best_t,
                     bool &tie, WalkCounts &c) {
    int best = -1;
    float lim = INFINITY;
    best_t = 0.0f;
    tie = false;
    for (int k = beg; k < end; ++k) {
        const CamCand cc = CRT_LDG(cands, k);
        if (((cc.rest >> bit) & 1ull) == 0ull) break;          /* no later candidate covers this pixel */
        if (best >= 0 && cc.dmin > best_t) break;
        if (((cc.mask >> bit) & 1ull) == 0ull) continue;       /* not this pixel's */
        if (COUNT) ++c.nodes;
        const bool tested = cand_test(cc, o, d, pr, best, best_t, tie, lim);
        if (COUNT && tested) ++c.tris;
    }
    return best;
}

/* Steps 2-3 for the closest triangle tri at t (tie: another triangle at the
 * same t) found by step 1: the reference's slot, or -1. */
template <bool COUNT>
CRT_HD int resolve_closest(const DNode *nodes, const PNode *pnodes, int n, const DTriGeo *slots,
                           const uint8_t *slot_cull, const int32_t *slot_tri, const KTopo *ktopo, bool planes_ok,
                           Vec o, Vec d, const PruneRay &pr, int tri, float t, bool tie, float &best_t, WalkCounts &c,
                           bool *fb = nullptr, const KTopo2 *ktopo2 = nullptr) {
    best_t = 0.0f;
    if (tri < 0) return -1;
    const RayRcp rr = make_ray_rcp(o, d, planes_ok);
    if (!tie) {
        const Vec p = vadd(o, vscale(d, t));
        const int slot = CRT_PROOF_TOPO && ktopo ? verify_topo<COUNT>(ktopo, nodes, slot_tri, tri, o, d, rr, p, c,
                                                                      CRT_PROOF_TOPO2 ? ktopo2 : nullptr)
                                                 : verify_kd<COUNT>(nodes, slot_tri, tri, o, d, rr, p, c);
        if (slot >= 0) {
            best_t = t;
            return slot;
        }
    }
    if (fb) *fb = true;
    CRT_FALLBACK_HOOK();
    return walk_pruned<COUNT>(pnode_order(pnodes, n, ray_octant(d)), n, slots, slot_cull, o, d, rr, pr, best_t, c);
}

/* The reference's closest hit of one ray (slot in reference visit-order
 * numbering, -1: miss) by steps 1-3.  fb (optional) is set when step 3 ran.
 * Rays with a NaN component miss every cell (each face test reads a NaN
 * coordinate), so they are answered without a walk. */
template <bool COUNT, int PF = CRT_BVH_PREFETCH>
CRT_HD int trace_bvh_exact(const BNode *bnodes, int bn, const DTriGeo *btri, const int32_t *btri_id,
                           const DNode *nodes, const PNode *pnodes, int n, const DTriGeo *slots,
                           const uint8_t *slot_cull, const int32_t *slot_tri, const KTopo *ktopo,
                           float prune_origin_max, bool planes_ok,
                           Vec o, Vec d, float &best_t, WalkCounts &c, bool *fb = nullptr,
                           const KTopo2 *ktopo2 = nullptr) {
    best_t = 0.0f;
    if (fb) *fb = false;
    if (isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z)) return -1;
    const int oct = ray_octant(d);
    const PruneRay pr = make_prune_ray(o, d, prune_origin_max);
    bool tie = false;
    float t = 0.0f;
    const int tri = walk_bvh<COUNT, PF>(bnode_order(bnodes, bn, oct), bn, btri, btri_id, o, d, pr, t, tie, c);
    CRT_WALK_HOOK();
    return resolve_closest<COUNT>(nodes, pnodes, n, slots, slot_cull, slot_tri, ktopo, planes_ok, o, d, pr, tri, t, tie,
                                  best_t, c, fb, ktopo2);
}

/* Shadow rays (option "shadows", the course's earlier renderer,
 * crt_renderer.cpp:90-92): whether the reference's closest hit of the ray
 * lies within the light, !(t * t > r2).  Any hit with !(fl(t * t) > r2)
 * decides it — the closest hit is no farther and rounding is monotone — so
 * the BVH walk stops at the first such hit whose triangle the reference
 * reaches (step 2's proof towards that hit's point), instead of walking to
 * the closest.  With lim = sqrt(r2) (1 + 2^-20) the walk drops every box that
 * cannot hold such a hit (fl(t * t) <= r2 implies t <= sqrt(r2) (1 + 2^-24)),
 * and a ray with no such hit among all triangles has none among the copies the
 * reference reaches.  Returns 1 (occluded), 0 (lit) or -1: the hit found
 * failed the proof (a cell edge) and the exact walk decides. */
template <bool COUNT>
CRT_HD int occluded_bvh(const BNode *bnodes, int bn, const DTriGeo *btri, const int32_t *btri_id, const DNode *nodes,
                        const int32_t *slot_tri, const KTopo *ktopo, const KTopo2 *ktopo2, float prune_origin_max,
                        bool planes_ok, Vec o, Vec d, float r2, WalkCounts &c) {
    if (isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z)) return 0;   /* misses every cell */
    const BNode *ord = bnode_order(bnodes, bn, ray_octant(d));
    const PruneRay pr = make_prune_ray(o, d, prune_origin_max);
    const float lim = sqrtf(r2) * (1.0f + 0x1p-20f);
    int i = 0;
    while (i < bn) {
        const BNode nd = CRT_LDG(ord, i);
        if (COUNT) ++c.nodes;
        if (!bnode_alive(nd, pr, lim)) {
            i = nd.skip;
            continue;
        }
        ++i;
        const int cnt = nd.leaf & 15, first = nd.leaf >> 4;
        for (int k = 0; k < cnt; ++k) {
            const DTriGeo g = CRT_LDG(btri, first + k);
            const int32_t id = CRT_LDG(btri_id, first + k);
            const uint8_t cull = (uint8_t)((uint32_t)id >> 31);
            float t;
            if (COUNT) ++c.tris;
            if (tri_hit(o, d, g, &cull, t) && !(t * t > r2)) {
                const RayRcp rr = make_ray_rcp(o, d, planes_ok);
                const Vec p = vadd(o, vscale(d, t));
                const int tri = id & 0x7fffffff;
                const int slot = CRT_PROOF_TOPO && ktopo
                                     ? verify_topo<COUNT>(ktopo, nodes, slot_tri, tri, o, d, rr, p, c,
                                                          CRT_PROOF_TOPO2 ? ktopo2 : nullptr)
                                     : verify_kd<COUNT>(nodes, slot_tri, tri, o, d, rr, p, c);
                return slot >= 0 ? 1 : -1;
            }
        }
    }
    return 0;
}

/* Step 1 of a shadow ray towards light P over its light bins (crt_layout.h
 * DLightBin; lists built by crt_light_bins.cpp, where the bound below is
 * derived): the first candidate with a hit the reference's triangle test
 * accepts within the light (fl(t * t) <= r2).  Returns 1 with (tri, t) set,
 * 0 when no triangle has such a hit, -1 when the bins do not decide this ray
 * (origin past the hull margins' bound, the line passes the light farther
 * than e_max, it ends farther than R0 past the light, or NaN) — the BVH
 * does.  With w = o - L, e the line's distance from L and the ray ending
 * within R0 of L: every hit point q the ray can reach lies in its
 * triangle's hull, either within R0 of L (the near list) or on the stretch
 * before the line's closest approach, where |q - L| <= |w| and the
 * direction of q - L is within asin(e_max / R0) of w's — in w's cell list,
 * whose candidates past dmin > |w| cannot hold it. */
/* One ray's part of the walk: ok = the bins decide it; its cell (-1: its
 * origin is within R0, the near list holds everything it can hit) and the
 * squared cut-offs of the near list and of the cell. */
struct LbinRay {
    double cut_near, cut_far;
    int cell;
    bool ok;
};

CRT_HD LbinRay lbin_setup(const DLightBin &P, int N, float prune_origin_max, Vec o, Vec d, float lim) {
    LbinRay r;
    r.cut_near = r.cut_far = 0.0;
    r.cell = -1;
    r.ok = false;
    if (!P.on) return r;
    if (!(fabsf(o.x) <= prune_origin_max && fabsf(o.y) <= prune_origin_max && fabsf(o.z) <= prune_origin_max))
        return r;   /* also NaN */
    const double dx = d.x, dy = d.y, dz = d.z;
    const double dd = dx * dx + dy * dy + dz * dz;
    if (!(dd > 0.0) || !(dd < 1e300)) return r;
    const double wx = (double)o.x - P.lx, wy = (double)o.y - P.ly, wz = (double)o.z - P.lz;
    const double cx = wy * dz - wz * dy, cy = wz * dx - wx * dz, cz = wx * dy - wy * dx;
    const double e2 = (cx * cx + cy * cy + cz * cz) / dd;
    if (!(e2 <= P.e_sq)) return r;
    const double l = lim;
    const double ex = wx + dx * l, ey = wy + dy * l, ez = wz + dz * l;
    const double end2 = ex * ex + ey * ey + ez * ez;
    if (!(end2 < 0.98 * P.r0_sq)) return r;
    const double w2 = wx * wx + wy * wy + wz * wz;
    r.ok = true;
    /* near list: points up to the closest approach are within |w|, past it within max(e, |end|) */
    r.cut_near = fmax(w2, fmax(e2, end2)) * (1.0 + 1e-9);
    /* a cell's triangles (hull >= R0 away) only before the closest approach, within |w| */
    r.cut_far = w2 * (1.0 + 1e-9);
    if (!(w2 >= 0.999 * P.r0_sq)) return r;   /* nearer origins: every point the ray reaches is within R0 */
    /* w's cell: face by the largest |w| component (ties: the lower axis), u, v = w_j / |w_k| */
    const double ax = fabs(wx), ay = fabs(wy), az = fabs(wz);
    int k;
    double m, a, b;
    if (ax >= ay && ax >= az) { k = 0; m = ax; a = wy; b = wz; }
    else if (ay >= az) { k = 1; m = ay; a = wx; b = wz; }
    else { k = 2; m = az; a = wx; b = wy; }
    const double wk = k == 0 ? wx : (k == 1 ? wy : wz);
    const int face = 2 * k + (wk < 0.0 ? 1 : 0);
    const double h = 0.5 * N;
    int cu = (int)floor((a / m + 1.0) * h), cv = (int)floor((b / m + 1.0) * h);
    cu = cu < 0 ? 0 : (cu > N - 1 ? N - 1 : cu);
    cv = cv < 0 ? 0 : (cv > N - 1 ? N - 1 : cv);
    r.cell = (face * N + cv) * N + cu;
    return r;
}

/* a candidate: a hit the reference's test accepts within the light */
CRT_HD bool lbin_test(const LightCand &cc, Vec o, Vec d, float r2, float &t) {
    const uint8_t cull = (uint8_t)((uint32_t)cc.id >> 31);
    return tri_hit(o, d, cc.g, &cull, t) && !(t * t > r2);
}

#ifndef CRT_LBINS_CAP
#define CRT_LBINS_CAP 96   /* candidates a shadow ray walks in its cell at most (more: undecided, the BVH decides; C2 with shadows: 24 0.42, 48 0.40, 96 0.37 ms) */
#endif

template <bool COUNT>
CRT_HD int lbin_first_hit(const LightCand *lb, const int32_t *off, const DLightBin &P, int N, float prune_origin_max,
                          Vec o, Vec d, float r2, int &tri, float &t_hit, WalkCounts &c) {
    tri = -1;
    t_hit = 0.0f;
    const float lim = sqrtf(r2) * (1.0f + 0x1p-20f);
    const LbinRay lr = lbin_setup(P, N, prune_origin_max, o, d, lim);
    if (!lr.ok) return -1;
    for (int phase = 0; phase < 2; ++phase) {
        if (phase == 1 && lr.cell < 0) break;
        const int beg = off[P.base + (phase ? 1 + lr.cell : 0)], end = off[P.base + (phase ? 2 + lr.cell : 1)];
        const double cut = phase ? lr.cut_far : lr.cut_near;
        for (int k = beg; k < end; ++k) {
            if (phase == 1 && k - beg >= CRT_LBINS_CAP) return -1;   /* a long walk: the BVH's */
            const LightCand cc = CRT_LDG(lb, k);
            if ((double)cc.dmin * (double)cc.dmin > cut) break;
            if (COUNT) ++c.tris;
            float t;
            if (lbin_test(cc, o, d, r2, t)) {
                tri = cc.id & 0x7fffffff;
                t_hit = t;
                return 1;
            }
        }
    }
    return 0;
}

/* lbin_first_hit with its hit proved on the reference's tree: 1 occluded,
 * 0 lit, -1 undecided (the BVH or the exact walk decides). */
template <bool COUNT>
CRT_HD int occluded_lbins(const LightCand *lb, const int32_t *off, const DLightBin &P, int N, float prune_origin_max,
                          const DNode *nodes, const int32_t *slot_tri, const KTopo *ktopo, const KTopo2 *ktopo2,
                          bool planes_ok, Vec o, Vec d, float r2, WalkCounts &c) {
    int tri;
    float t;
    const int r = lbin_first_hit<COUNT>(lb, off, P, N, prune_origin_max, o, d, r2, tri, t, c);
    if (r != 1) return r;
    const RayRcp rr = make_ray_rcp(o, d, planes_ok);
    const Vec p = vadd(o, vscale(d, t));
    const int slot = CRT_PROOF_TOPO && ktopo ? verify_topo<COUNT>(ktopo, nodes, slot_tri, tri, o, d, rr, p, c,
                                                                  CRT_PROOF_TOPO2 ? ktopo2 : nullptr)
                                             : verify_kd<COUNT>(nodes, slot_tri, tri, o, d, rr, p, c);
    return slot >= 0 ? 1 : -1;
}

/* The same answer for a camera ray of cell [beg, end) through the camera bins. */
template <bool COUNT>
CRT_HD int trace_bins_exact(const CamCand *cands, int beg, int end, int bit, const DNode *nodes, const PNode *pnodes, int n,
                            const DTriGeo *slots, const uint8_t *slot_cull, const int32_t *slot_tri,
                            const KTopo *ktopo, float prune_origin_max, bool planes_ok, Vec o, Vec d, float &best_t,
                            WalkCounts &c, bool *fb = nullptr, const KTopo2 *ktopo2 = nullptr) {
    best_t = 0.0f;
    if (fb) *fb = false;
    if (isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z)) return -1;
    const PruneRay pr = make_prune_ray(o, d, prune_origin_max);
    bool tie = false;
    float t = 0.0f;
    const int tri = walk_bins<COUNT>(cands, beg, end, bit, o, d, pr, t, tie, c);
    return resolve_closest<COUNT>(nodes, pnodes, n, slots, slot_cull, slot_tri, ktopo, planes_ok, o, d, pr, tri, t, tie,
                                  best_t, c, fb, ktopo2);
}

}  // namespace crt_amd
