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
template <bool COUNT>
CRT_HD int walk_bvh(const BNode *nodes, int n, const DTriGeo *geo, const int32_t *tid, Vec o, Vec d,
                    const PruneRay &pr, float &best_t, bool &tie, WalkCounts &c) {
    int best = -1;
    float lim = INFINITY;
    best_t = 0.0f;
    tie = false;
    int i = 0;
    while (i < n) {
        const BNode nd = CRT_LDG(nodes, i);
        if (COUNT) ++c.nodes;
        if (!bnode_alive(nd, pr, lim)) {
            i = nd.skip;
            continue;
        }
        ++i;                                   /* interior: first child; leaf: next in preorder */
        const int cnt = nd.leaf & 15;
        const int first = nd.leaf >> 4;
        for (int k = 0; k < cnt; ++k) {
            const DTriGeo g = CRT_LDG(geo, first + k);
            const int32_t id = CRT_LDG(tid, first + k);
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

/* The reference's closest hit of one ray (slot in reference visit-order
 * numbering, -1: miss) by steps 1-3.  fb (optional) is set when step 3 ran.
 * Rays with a NaN component miss every cell (each face test reads a NaN
 * coordinate), so they are answered without a walk. */
template <bool COUNT>
CRT_HD int trace_bvh_exact(const BNode *bnodes, int bn, const DTriGeo *btri, const int32_t *btri_id,
                           const DNode *nodes, const PNode *pnodes, int n, const DTriGeo *slots,
                           const uint8_t *slot_cull, const int32_t *slot_tri, float prune_origin_max, bool planes_ok,
                           Vec o, Vec d, float &best_t, WalkCounts &c, bool *fb = nullptr) {
    best_t = 0.0f;
    if (fb) *fb = false;
    if (isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z)) return -1;
    const int oct = ray_octant(d);
    const PruneRay pr = make_prune_ray(o, d, prune_origin_max);
    bool tie = false;
    float t = 0.0f;
    const int tri = walk_bvh<COUNT>(bnode_order(bnodes, bn, oct), bn, btri, btri_id, o, d, pr, t, tie, c);
    if (tri < 0) return -1;
    const RayRcp rr = make_ray_rcp(o, d, planes_ok);
    if (!tie) {
        const int slot = verify_kd<COUNT>(nodes, slot_tri, tri, o, d, rr, vadd(o, vscale(d, t)), c);
        if (slot >= 0) {
            best_t = t;
            return slot;
        }
    }
    if (fb) *fb = true;
    return walk_pruned<COUNT>(pnode_order(pnodes, n, oct), n, slots, slot_cull, o, d, rr, pr, best_t, c);
}

}  // namespace crt_amd
