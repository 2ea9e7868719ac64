/*
 * prune_sim.cpp — TEST TOOL (CPU only): runs the product's pruned walk
 * (crt_device.h walk_pruned over the octant-ordered PNode arrays built by
 * crt_scene_build.cpp) next to the unpruned reference-order walk on the host,
 * from the same sources the HIP library compiles, so the pruning rule can be
 * checked for exact (slot, t) agreement on many rays without a GPU and its
 * work reduction measured.  The unpruned walk here is the reference's visit
 * order (crt_intersection.cpp:109-136); tests/ also checks it against the
 * oracle.  Built by tests/tools/Makefile; loaded by tests/test_prune.py.
 */
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_host.h"
#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_device.h"

using namespace crt_amd;

namespace {

int walk_reference(const HostScene &hs, Vec o, Vec d, float &best_t, uint64_t &nodes, uint64_t &tris) {
    int best = -1;
    best_t = 0.0f;
    const int n = (int)hs.nodes.size();
    int i = 0;
    while (i < n) {
        const DNode nd = hs.nodes[i];
        const bool pass = box_hit(o, d, nd);
        ++nodes;
        if (nd.b < 0) {
            i = pass ? i + 1 : nd.a;
            continue;
        }
        if (pass) {
            for (int k = 0; k < node_leaf_count(nd); ++k) {
                const int slot = nd.b + k;
                float t;
                ++tris;
                if (tri_hit(o, d, hs.slots[slot], hs.slot_cull.data() + slot, t) && (best < 0 || t < best_t)) {
                    best_t = t;
                    best = slot;
                }
            }
        }
        ++i;
    }
    return best;
}

}  // namespace

extern "C" {

/* counts[0..3] = reference nodes, reference triangles, pruned nodes, pruned
 * triangles (summed over the batch).  Slots are reference visit-order slot
 * numbers (-1 = miss). */
int prune_sim_trace(const crt_scene_desc *desc, const float *rays, int64_t n, int32_t *ref_slot, float *ref_t,
                    int32_t *pr_slot, float *pr_t, uint64_t *counts) {
    HostScene hs;
    const int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    const int nn = (int)hs.nodes.size();
    uint64_t rn = 0, rt = 0, pn = 0, pt = 0;
    for (int64_t i = 0; i < n; ++i) {
        const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        float t = 0.f;
        ref_slot[i] = walk_reference(hs, o, d, t, rn, rt);
        ref_t[i] = t;
        const RayRcp rr = make_ray_rcp(o, d, false);
        const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
        WalkCounts c = {0u, 0u};
        pr_slot[i] = walk_pruned<true>(pnode_order(hs.pnodes.data(), nn, ray_octant(d)), nn, hs.slots.data(),
                                       hs.slot_cull.data(), o, d, rr, pr, t, c);
        pr_t[i] = t;
        pn += c.nodes;
        pt += c.tris;
    }
    counts[0] = rn;
    counts[1] = rt;
    counts[2] = pn;
    counts[3] = pt;
    return CRT_OK;
}

/* Hull containment check: every slot's triangle box lies inside the hull of
 * every PNode on its leaf's path, in all 8 orders.  Returns the number of
 * violations (0 expected). */
int64_t prune_sim_check_hulls(const crt_scene_desc *desc) {
    HostScene hs;
    if (prepare_scene(desc, hs) != CRT_OK) return -1;
    const int nn = (int)hs.nodes.size();
    int64_t bad = 0;
    for (int oct = 0; oct < 8; ++oct) {
        const PNode *p = pnode_order(hs.pnodes.data(), nn, oct);
        /* walk with an explicit path of open interior nodes */
        int path[128];
        int depth_top = 0;
        for (int i = 0; i < nn; ++i) {
            while (depth_top > 0 && p[path[depth_top - 1]].a <= i) --depth_top;
            if (p[i].b < 0) {
                path[depth_top++] = i;
                continue;
            }
            for (int k = 0; k < pnode_leaf_count(p[i]); ++k) {
                const DTriGeo &g = hs.slots[p[i].b + k];
                const float xs[3] = {g.v0x, g.v1x, g.v2x}, ys[3] = {g.v0y, g.v1y, g.v2y}, zs[3] = {g.v0z, g.v1z, g.v2z};
                for (int v = 0; v < 3; ++v) {
                    auto inside = [&](const PNode &q) {
                        return xs[v] >= q.tlo_x && xs[v] <= q.thi_x && ys[v] >= q.tlo_y && ys[v] <= q.thi_y &&
                               zs[v] >= q.tlo_z && zs[v] <= q.thi_z;
                    };
                    bool ok = inside(p[i]);
                    for (int u = 0; u < depth_top; ++u) ok = ok && inside(p[path[u]]);
                    if (!ok) ++bad;
                }
            }
        }
    }
    return bad;
}

}  // extern "C"
