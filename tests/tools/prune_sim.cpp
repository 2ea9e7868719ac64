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
#include <algorithm>
#include <array>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_host.h"
#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_device.h"
#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_bvh.h"
#include "../../chaos-ray-tracing-course-2025_amd/csrc/crt_bins.h"

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

/* The BVH walk with its kd verification (crt_bvh.h trace_bvh_exact), from
 * the product's sources, next to the reference-order walk.  A BVH answer is
 * equal to the reference's when its t bits match and its slot holds the same
 * triangle (copies of a triangle give the same record; the slot numbers may
 * differ).  counts[0..4] = reference nodes, reference triangles, BVH walk +
 * verification node tests, BVH triangle tests, rays that took the fallback. */
int bvh_sim_trace(const crt_scene_desc *desc, const float *rays, int64_t n, int32_t *ref_tri, float *ref_t,
                  int32_t *bvh_tri, float *bvh_t, uint64_t *counts) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK))
        return rc;   /* scenes without scattered rays */
    const int nn = (int)hs.nodes.size();
    uint64_t rn = 0, rt = 0, fbn = 0;
    WalkCounts c = {0u, 0u};
    for (int64_t i = 0; i < n; ++i) {
        const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        float t = 0.f;
        const int rs = walk_reference(hs, o, d, t, rn, rt);
        ref_tri[i] = rs >= 0 ? hs.slot_tri[rs] : -1;
        ref_t[i] = t;
        bool fb = false;
        const int bs = trace_bvh_exact<true>(hs.bnodes.data(), hs.bnode_count, hs.btri.data(), hs.btri_id.data(),
                                             hs.nodes.data(), hs.pnodes.data(), nn, hs.slots.data(),
                                             hs.slot_cull.data(), hs.slot_tri.data(), hs.ktopo.empty() ? nullptr : hs.ktopo.data(), hs.prune_origin_max, false, o,
                                             d, t, c, &fb);
        bvh_tri[i] = bs >= 0 ? hs.slot_tri[bs] : -1;
        bvh_t[i] = t;
        fbn += fb ? 1 : 0;
    }
    counts[0] = rn;
    counts[1] = rt;
    counts[2] = c.nodes;
    counts[3] = c.tris;
    counts[4] = fbn;
    return CRT_OK;
}

/* Shadow rays over the light bins (crt_light_bins.cpp, crt_bvh.h
 * occluded_lbins) next to the reference's closest hit: rays[8 i ..] =
 * {o, d, r2, light}; ref[i] = 1 when the reference's closest hit is within
 * the light (fl(t * t) <= r2), lb[i] = the bins' answer (1 / 0 / -1
 * undecided).  info[0..3] = records, lights on, near records of light 0,
 * candidate tests. */
int lbins_sim_check(const crt_scene_desc *desc, const float *rays, int64_t n, double e_max, int N, int8_t *ref,
                    int8_t *lb, int64_t *info) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK))
        return rc;
    std::vector<CamCand> tpl;
    bin_templates(hs, tpl);
    LightBinsHost L;
    build_light_bins(tpl.data(), (int)tpl.size(), hs.lights.data(), (int)hs.lights.size(), e_max, N, L);
    info[0] = (int64_t)L.recs.size();
    info[1] = 0;
    for (const DLightBin &p : L.par) info[1] += p.on;
    info[2] = L.par.empty() ? 0 : L.off[1] - L.off[0];
    WalkCounts c = {0u, 0u};
    uint64_t rn = 0, rt = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *r = rays + 8 * i;
        const Vec o = vec(r[0], r[1], r[2]), d = vec(r[3], r[4], r[5]);
        const float r2 = r[6];
        const int l = (int)r[7];
        float t = 0.f;
        const int rs = walk_reference(hs, o, d, t, rn, rt);
        ref[i] = (int8_t)(rs >= 0 && !(t * t > r2));
        lb[i] = L.par.empty() ? (int8_t)-1
                              : (int8_t)occluded_lbins<true>(L.recs.data(), L.off.data(), L.par[(size_t)l], L.n,
                                                             hs.prune_origin_max, hs.nodes.data(), hs.slot_tri.data(),
                                                             hs.ktopo.empty() ? nullptr : hs.ktopo.data(),
                                                             hs.ktopo2.empty() ? nullptr : hs.ktopo2.data(), false, o, d,
                                                             r2, c);
    }
    info[3] = (int64_t)c.tris;
    return CRT_OK;
}

/* Per shadow ray of the light bins: its cell (-1 near only, -2 undecided) and
 * the candidates its walk visits (near + cell), for wave-cost analysis
 * (scripts/lbins_wave_cost.py). */
int lbins_sim_steps(const crt_scene_desc *desc, const float *rays, int64_t n, double e_max, int N, int32_t *cell,
                    int32_t *steps) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    std::vector<CamCand> tpl;
    bin_templates(hs, tpl);
    LightBinsHost L;
    if (!build_light_bins(tpl.data(), (int)tpl.size(), hs.lights.data(), (int)hs.lights.size(), e_max, N, L)) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const float *r = rays + 8 * i;
        const Vec o = vec(r[0], r[1], r[2]), d = vec(r[3], r[4], r[5]);
        const float r2 = r[6];
        const DLightBin &P = L.par[(size_t)r[7]];
        const float lim = sqrtf(r2) * (1.0f + 0x1p-20f);
        const LbinRay lr = lbin_setup(P, L.n, hs.prune_origin_max, o, d, lim);
        cell[i] = lr.ok ? lr.cell : -2;
        steps[i] = 0;
        if (!lr.ok) continue;
        bool done = false;
        for (int phase = 0; phase < 2 && !done; ++phase) {
            if (phase == 1 && lr.cell < 0) break;
            const int beg = L.off[(size_t)P.base + (phase ? 1 + lr.cell : 0)];
            const int end = L.off[(size_t)P.base + (phase ? 2 + lr.cell : 1)];
            const double cut = phase ? lr.cut_far : lr.cut_near;
            for (int k = beg; k < end && !done; ++k) {
                const LightCand &cc = L.recs[(size_t)k];
                ++steps[i];
                if ((double)cc.dmin * (double)cc.dmin > cut) break;
                float t;
                if (lbin_test(cc, o, d, r2, t)) done = true;
            }
        }
    }
    return CRT_OK;
}

/* Per-ray work of trace_bvh_exact (for wave-cost analysis, scripts/bvh_wave_cost.py):
 * out[4 i ..] = {BVH walk nodes, BVH walk triangles, proof/fallback nodes +
 * triangles, fallback taken}. */
int bvh_sim_ray_stats(const crt_scene_desc *desc, const float *rays, int64_t n, int32_t *out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    const int nn = (int)hs.nodes.size();
    for (int64_t i = 0; i < n; ++i) {
        const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        WalkCounts w = {0u, 0u}, c = {0u, 0u};
        float t = 0.f;
        bool tie = false, fb = false;
        const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
        (void)walk_bvh<true>(bnode_order(hs.bnodes.data(), hs.bnode_count, ray_octant(d)), hs.bnode_count,
                             hs.btri.data(), hs.btri_id.data(), o, d, pr, t, tie, w);
        (void)trace_bvh_exact<true>(hs.bnodes.data(), hs.bnode_count, hs.btri.data(), hs.btri_id.data(),
                                    hs.nodes.data(), hs.pnodes.data(), nn, hs.slots.data(), hs.slot_cull.data(),
                                    hs.slot_tri.data(), hs.ktopo.empty() ? nullptr : hs.ktopo.data(), hs.prune_origin_max, false, o, d, t, c, &fb);
        out[4 * i] = (int32_t)w.nodes;
        out[4 * i + 1] = (int32_t)w.tris;
        out[4 * i + 2] = (int32_t)(c.nodes + c.tris - w.nodes - w.tris);
        out[4 * i + 3] = fb ? 1 : 0;
    }
    return CRT_OK;
}

/* The proof on the topology records against the descent of the 32-B nodes
 * (crt_bvh.h verify_topo / verify_kd) on every ray whose BVH hit has no tie,
 * with both division paths of the box test: the same algorithm, so the same
 * slot (or -1) and the same node-test count for every ray.
 * out = {proofs compared, proofs that differ, proofs that succeed}; -1: no KTopo. */
int bvh_sim_proof_check(const crt_scene_desc *desc, const float *rays, int64_t n, uint64_t *out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    if (hs.ktopo.empty()) return -1;
    for (int k = 0; k < 3; ++k) out[k] = 0;
    for (int64_t i = 0; i < n; ++i) {
        const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        WalkCounts w = {0u, 0u};
        float t = 0.f;
        bool tie = false;
        const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
        const int tri = walk_bvh<true>(bnode_order(hs.bnodes.data(), hs.bnode_count, ray_octant(d)), hs.bnode_count,
                                       hs.btri.data(), hs.btri_id.data(), o, d, pr, t, tie, w);
        if (tri < 0 || tie) continue;
        for (int fast = 0; fast < 2; ++fast) {
            WalkCounts ca = {0u, 0u}, cb = {0u, 0u};
            const RayRcp rr = make_ray_rcp(o, d, fast != 0);
            const Vec p = vadd(o, vscale(d, t));
            const int a = verify_topo<true>(hs.ktopo.data(), hs.nodes.data(), hs.slot_tri.data(), tri, o, d, rr, p, ca);
            const int b = verify_kd<true>(hs.nodes.data(), hs.slot_tri.data(), tri, o, d, rr, p, cb);
            ++out[0];
            out[1] += (a != b || ca.nodes != cb.nodes) ? 1 : 0;
            out[2] += a >= 0 ? 1 : 0;
        }
    }
    return CRT_OK;
}

/* BVH box containment: every triangle's vertices lie inside the box of every
 * BVH node above its leaf, in all 8 orders, and every order lists each
 * triangle exactly once.  Returns the number of violations (0 expected). */
int64_t bvh_sim_check(const crt_scene_desc *desc) {
    HostScene hs;
    if (prepare_scene(desc, hs) != CRT_OK) return -1;
    if (hs.bnode_count == 0 && build_bvh(hs) != CRT_OK) return -1;
    const int n = hs.bnode_count;
    const int nt = (int)hs.btri.size();
    int64_t bad = 0;
    for (int oct = 0; oct < 8; ++oct) {
        const BNode *p = bnode_order(hs.bnodes.data(), n, oct);
        std::vector<int> seen(nt, 0);
        int path[128];
        int top = 0;
        for (int i = 0; i < n; ++i) {
            while (top > 0 && p[path[top - 1]].skip <= i) --top;
            const int cnt = p[i].leaf & 15;
            if (cnt == 0) {
                if (top >= 128) return -2;
                path[top++] = i;
                continue;
            }
            if (p[i].skip != i + 1) ++bad;
            for (int k = 0; k < cnt; ++k) {
                const int j = (p[i].leaf >> 4) + k;
                if (j < 0 || j >= nt) { ++bad; continue; }
                ++seen[j];
                const DTriGeo &g = hs.btri[j];
                const float xs[3] = {g.v0x, g.v1x, g.v2x}, ys[3] = {g.v0y, g.v1y, g.v2y}, zs[3] = {g.v0z, g.v1z, g.v2z};
                for (int v = 0; v < 3; ++v) {
                    auto inside = [&](const BNode &q) {
                        return xs[v] >= q.lo_x && xs[v] <= q.hi_x && ys[v] >= q.lo_y && ys[v] <= q.hi_y &&
                               zs[v] >= q.lo_z && zs[v] <= q.hi_z;
                    };
                    bool ok = inside(p[i]);
                    for (int u = 0; u < top; ++u) ok = ok && inside(p[path[u]]);
                    if (!ok) ++bad;
                }
            }
        }
        for (int j = 0; j < nt; ++j) bad += seen[j] != 1;
    }
    return bad;
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

/* Lockstep coherence of the per-lane camera BVH walk (crt_bvh.h walk_bvh, no
 * prefetch) over the 8x8 tiles of a frame: the wave loop runs one node step
 * per active lane per iteration (a lane on a live leaf tests its triangles in
 * the same iteration).  rays: [h*w, 6] camera rays, row-major.
 * out[0] wave iterations, [1] iterations whose active lanes all stand on one
 * node, [2] sum over iterations of distinct nodes, [3] sum of active lanes,
 * [4] leaf rounds (max triangles of the iteration's leaf lanes),
 * [5] max iterations of a tile, [6] tiles. */
extern "C" int bvh_sim_tile_coherence(const crt_scene_desc *desc, const float *rays, int w, int h, uint64_t *out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    for (int k = 0; k < 7; ++k) out[k] = 0;
    const int n = hs.bnode_count;
    struct L { const BNode *nodes; PruneRay pr; Vec o, d; int i, best; float lim, bt; bool on; };
    for (int ty = 0; ty < h; ty += 8)
        for (int tx = 0; tx < w; tx += 8) {
            L ln[64];
            int nl = 0;
            for (int y = ty; y < std::min(h, ty + 8); ++y)
                for (int x = tx; x < std::min(w, tx + 8); ++x) {
                    const float *r = rays + 6 * ((int64_t)y * w + x);
                    L &l = ln[nl++];
                    l.o = vec(r[0], r[1], r[2]);
                    l.d = vec(r[3], r[4], r[5]);
                    l.nodes = bnode_order(hs.bnodes.data(), n, ray_octant(l.d));
                    l.pr = make_prune_ray(l.o, l.d, hs.prune_origin_max);
                    l.i = 0;
                    l.best = -1;
                    l.lim = INFINITY;
                    l.bt = 0.f;
                    l.on = true;
                }
            uint64_t it = 0;
            for (;;) {
                int act = 0, leafmax = 0;
                const BNode *addr[64];
                for (int k = 0; k < nl; ++k) {
                    L &l = ln[k];
                    if (!l.on || l.i >= n) { l.on = false; continue; }
                    addr[act++] = l.nodes + l.i;
                    const BNode nd = l.nodes[l.i];
                    if (!bnode_alive(nd, l.pr, l.lim)) { l.i = nd.skip; continue; }
                    ++l.i;
                    const int cnt = nd.leaf & 15, first = nd.leaf >> 4;
                    leafmax = std::max(leafmax, cnt);
                    for (int q = 0; q < cnt; ++q) {
                        const DTriGeo g = hs.btri[first + q];
                        const uint8_t cull = (uint8_t)((uint32_t)hs.btri_id[first + q] >> 31);
                        float t;
                        if (tri_hit(l.o, l.d, g, &cull, t) && (l.best < 0 || t < l.bt)) {
                            l.bt = t;
                            l.best = 1;
                            l.lim = t;
                        }
                    }
                }
                if (act == 0) break;
                ++it;
                std::sort(addr, addr + act);
                const int distinct = (int)(std::unique(addr, addr + act) - addr);
                out[1] += distinct == 1;
                out[2] += distinct;
                out[3] += act;
                out[4] += leafmax;
            }
            out[0] += it;
            out[5] = std::max<uint64_t>(out[5], it);
            ++out[6];
        }
    return CRT_OK;
}

/* Camera bins against the BVH walk (crt_bvh.h walk_bins vs walk_bvh) on every
 * camera ray of the frame at the scene's resolution: the same t bits and tie
 * flag, and the same closest triangle where there is no tie (with one, the
 * triangle is not used: crt_bvh.h resolve_closest takes the exact kd walk).  out: [0] rays, [1] rays that differ,
 * [2] candidates tested, [3] most candidates tested by one ray, [4] cells,
 * [5] listed candidates, [6] 1 if bins were built. */
extern "C" int bins_sim_check(const crt_scene_desc *desc, uint64_t *out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;   /* cells over the cap walk the BVH (crt_bins.h): no list to check */
    if ((rc = build_camera_bins(hs, bins, off, &over)) != CRT_OK) return rc;
    for (int k = 0; k < 7; ++k) out[k] = 0;
    if (bins.empty()) return CRT_OK;
    out[6] = 1;
    out[4] = off.size() - 1;
    out[5] = bins.size();
    DeviceScene ds{};
    const DCamera cam = host_camera(hs);
    const int tx = (hs.width + 7) / 8;
    for (int y = 0; y < hs.height; ++y)
        for (int x = 0; x < hs.width; ++x) {
            Vec o, d;
            camera_ray(cam, x, y, o, d);
            const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
            WalkCounts w = {0u, 0u}, wb = {0u, 0u};
            float t1 = 0.f, t2 = 0.f;
            bool tie1 = false, tie2 = false;
            const int a = walk_bvh<true>(bnode_order(hs.bnodes.data(), hs.bnode_count, ray_octant(d)), hs.bnode_count,
                                         hs.btri.data(), hs.btri_id.data(), o, d, pr, t1, tie1, w);
            const int cell = (y / 8) * tx + x / 8;
            if (over[(size_t)cell]) continue;
            const int b = walk_bins<true>(bins.data(), off[cell], off[cell + 1], 8 * (y % 8) + x % 8, o, d, pr, t2, tie2, wb);
            ++out[0];
            uint32_t u1, u2;
            std::memcpy(&u1, &t1, 4);
            std::memcpy(&u2, &t2, 4);
            /* with a tie the triangle is not used (the exact kd walk decides) */
            if ((a < 0) != (b < 0) || (a >= 0 && (u1 != u2 || tie1 != tie2 || (!tie1 && a != b)))) ++out[1];
            out[2] += wb.nodes;
            out[3] = std::max<uint64_t>(out[3], wb.nodes);
        }
    return CRT_OK;
}

/* Host restatement of crt_walks.h trace_bins_lanes' schedule (K lanes per
 * pixel: lane sl takes the covering records at chunk positions j = sl mod K,
 * one per round, the K share lim after every round; merged: smallest t, the
 * lowest lane holding it, tie when two lanes hold it or one saw two hits
 * there) against walk_bins on every camera ray of the frame.  out[0] rays,
 * out[1] rays whose (hit, t bits, tie, triangle when no tie) differ, out[2]
 * rays where some lane stopped on the shared bound (the sharing mattered). */
extern "C" int bins_sim_lanes_check(const crt_scene_desc *desc, int K, uint64_t *out) {
    if (K != 2 && K != 4) return -1;
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;   /* cells over the cap walk the BVH (crt_bins.h): no list to check */
    if ((rc = build_camera_bins(hs, bins, off, &over)) != CRT_OK) return rc;
    out[0] = out[1] = out[2] = 0;
    if (bins.empty()) return CRT_OK;
    DeviceScene ds{};
    const DCamera cam = host_camera(hs);
    const int tx = (hs.width + 7) / 8;
    constexpr int kChunk = 32;   /* crt_walks.h kBinChunk */
    for (int y = 0; y < hs.height; ++y)
        for (int x = 0; x < hs.width; ++x) {
            Vec o, d;
            camera_ray(cam, x, y, o, d);
            const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
            const int cell = (y / 8) * tx + x / 8, bit = 8 * (y % 8) + x % 8;
            if (over[(size_t)cell]) continue;
            WalkCounts wc = {0u, 0u};
            float ts = 0.f;
            bool ties = false;
            const int a = walk_bins<false>(bins.data(), off[cell], off[cell + 1], bit, o, d, pr, ts, ties, wc);
            int best[4] = {-1, -1, -1, -1};
            float bt[4] = {0.f, 0.f, 0.f, 0.f}, lim = INFINITY;
            bool tie[4] = {false, false, false, false}, live[4], shared_stop = false;
            for (int l = 0; l < K; ++l) live[l] = true;
            for (int k0 = off[cell]; k0 < off[cell + 1]; k0 += kChunk) {
                bool any = false;
                for (int l = 0; l < K; ++l) any = any || live[l];
                if (!any) break;
                const int n = std::min(kChunk, off[cell + 1] - k0);
                const bool rest = ((bins[k0].rest >> bit) & 1ull) != 0ull;
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                for (int l = 0; l < K; ++l) {
                    live[l] = live[l] && rest;
                    if (live[l])
                        for (int j = l; j < n; j += K) w[l] |= (uint32_t)((bins[k0 + j].mask >> bit) & 1ull) << j;
                }
                for (;;) {
                    bool busy = false;
                    for (int l = 0; l < K; ++l) busy = busy || w[l] != 0u;
                    if (!busy) break;
                    for (int l = 0; l < K; ++l) {
                        if (w[l] == 0u) continue;
                        const int j = __builtin_ctz(w[l]);
                        w[l] &= w[l] - 1u;
                        const CamCand &cc = bins[k0 + j];
                        if (cc.dmin > lim) {
                            if (best[l] < 0 || cc.dmin <= bt[l]) shared_stop = true;   /* alone it would go on */
                            live[l] = false;
                            w[l] = 0u;
                        } else if (cand_alive(cc, pr, lim)) {
                            const uint8_t cull = (uint8_t)((uint32_t)cc.id >> 31);
                            float t;
                            if (tri_hit(o, d, cc.g, &cull, t)) {
                                if (best[l] < 0 || t < bt[l]) {
                                    bt[l] = t;
                                    best[l] = cc.id & 0x7fffffff;
                                    tie[l] = false;
                                } else if (t == bt[l]) {
                                    tie[l] = true;
                                }
                            }
                        }
                    }
                    for (int l = 0; l < K; ++l)
                        if (best[l] >= 0) lim = std::min(lim, bt[l]);
                }
            }
            float g = INFINITY;
            for (int l = 0; l < K; ++l)
                if (best[l] >= 0) g = std::min(g, bt[l]);
            int holders = 0, b = -1;
            bool tg = false;
            for (int l = 0; l < K; ++l)
                if (best[l] >= 0 && bt[l] == g) {
                    if (b < 0) b = best[l];
                    ++holders;
                    tg = tg || tie[l];
                }
            tg = tg || holders > 1;
            ++out[0];
            out[2] += shared_stop;
            uint32_t u1, u2;
            std::memcpy(&u1, &ts, 4);
            std::memcpy(&u2, &g, 4);
            if ((a < 0) != (b < 0) || (a >= 0 && (u1 != u2 || ties != tg || (!ties && a != b)))) ++out[1];
        }
    return CRT_OK;
}

/* debugging aid: the first `cap` differing rays of bins_sim_check as
 * {x, y, bvh tri, bins tri, bvh t bits, bins t bits, tie bvh, tie bins, bvh tri listed in the cell} */
extern "C" int bins_sim_diffs(const crt_scene_desc *desc, int64_t *rows, int cap) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;   /* cells over the cap walk the BVH (crt_bins.h): no list to check */
    if ((rc = build_camera_bins(hs, bins, off, &over)) != CRT_OK) return rc;
    if (bins.empty()) return 0;
    DeviceScene ds{};
    const DCamera cam = host_camera(hs);
    const int tx = (hs.width + 7) / 8;
    int n = 0;
    for (int y = 0; y < hs.height && n < cap; ++y)
        for (int x = 0; x < hs.width && n < cap; ++x) {
            Vec o, d;
            camera_ray(cam, x, y, o, d);
            const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
            WalkCounts w = {0u, 0u};
            float t1 = 0.f, t2 = 0.f;
            bool tie1 = false, tie2 = false;
            const int a = walk_bvh<false>(bnode_order(hs.bnodes.data(), hs.bnode_count, ray_octant(d)), hs.bnode_count,
                                          hs.btri.data(), hs.btri_id.data(), o, d, pr, t1, tie1, w);
            const int cell = (y / 8) * tx + x / 8;
            if (over[(size_t)cell]) continue;
            const int b = walk_bins<false>(bins.data(), off[cell], off[cell + 1], 8 * (y % 8) + x % 8, o, d, pr, t2, tie2, w);
            uint32_t u1, u2;
            std::memcpy(&u1, &t1, 4);
            std::memcpy(&u2, &t2, 4);
            if ((a < 0) != (b < 0) || (a >= 0 && (u1 != u2 || tie1 != tie2 || (!tie1 && a != b)))) {
                int listed = 0;
                for (int k = off[cell]; k < off[cell + 1]; ++k) listed |= (bins[k].id & 0x7fffffff) == a;
                int64_t *r = rows + 9 * n++;
                r[0] = x; r[1] = y; r[2] = a; r[3] = b; r[4] = u1; r[5] = u2; r[6] = tie1; r[7] = tie2; r[8] = listed;
            }
        }
    return n;
}

/* Per 8x8 cell of the camera bins: [0] list length, [1] the wave's loop
 * iterations (the largest index a lane of the cell leaves walk_bins at, as
 * the device loop runs), [2] candidates the cell's lanes test in total,
 * [3] most candidates one lane tests, [4] longest proof / fallback (node +
 * triangle steps), [5] lanes with a tie, [6] lanes that fell back.  out: 8
 * per cell. */
extern "C" int bins_sim_cells(const crt_scene_desc *desc, int64_t *out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;   /* cells over the cap walk the BVH (crt_bins.h): no list to check */
    if ((rc = build_camera_bins(hs, bins, off, &over)) != CRT_OK) return rc;
    if (bins.empty()) return -1;
    DeviceScene ds{};
    const DCamera cam = host_camera(hs);
    const int tx = (hs.width + 7) / 8, ty = (hs.height + 7) / 8;
    for (int cy = 0; cy < ty; ++cy)
        for (int cx = 0; cx < tx; ++cx) {
            const int cell = cy * tx + cx;
            int64_t *r = out + 8 * (int64_t)cell;
            r[0] = off[cell + 1] - off[cell];
            r[1] = r[2] = r[3] = r[4] = r[5] = r[6] = r[7] = 0;
            for (int y = 8 * cy; y < std::min(hs.height, 8 * cy + 8); ++y)
                for (int x = 8 * cx; x < std::min(hs.width, 8 * cx + 8); ++x) {
                    Vec o, d;
                    camera_ray(cam, x, y, o, d);
                    const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
                    const int bit = 8 * (y - 8 * cy) + (x - 8 * cx);
                    int best = -1;
                    float bt = 0.f, lim = INFINITY;
                    bool tie = false;
                    int k = off[cell], tested = 0;
                    for (; k < off[cell + 1]; ++k) {
                        const CamCand &cc = bins[k];
                        if (((cc.rest >> bit) & 1ull) == 0ull) break;
                        if (best >= 0 && cc.dmin > bt) break;
                        if (((cc.mask >> bit) & 1ull) == 0ull) continue;
                        ++tested;
                        cand_test(cc, o, d, pr, best, bt, tie, lim);
                    }
                    r[1] = std::max<int64_t>(r[1], k - off[cell]);
                    r[2] += tested;
                    r[3] = std::max<int64_t>(r[3], tested);
                    WalkCounts pc = {0u, 0u};
                    bool fb = false;
                    float tt = 0.f;
                    (void)resolve_closest<true>(hs.nodes.data(), hs.pnodes.data(), (int)hs.nodes.size(), hs.slots.data(),
                                                hs.slot_cull.data(), hs.slot_tri.data(),
                                                hs.ktopo.empty() ? nullptr : hs.ktopo.data(), false, o, d, pr, best, bt,
                                                tie, tt, pc, &fb);
                    r[4] = std::max<int64_t>(r[4], pc.nodes + pc.tris);
                    r[5] += tie ? 1 : 0;
                    r[6] += fb ? 1 : 0;
                }
        }
    return CRT_OK;
}

/* Camera fuzz (tests/test_bins_fuzz.py).  Every camera ray of the scene's
 * camera: (a) the camera-bins walk against the BVH walk — the same t bits and
 * tie flag, and the same triangle without a tie — and (b) the whole product
 * answer (bins where the cell has a list, else the BVH walk; then the proof
 * or the exact kd fallback, resolve_closest) against the reference-order walk
 * (walk_reference: the reference's node order and first-found rule) — the
 * same triangle and t bits (the leaf copies of a triangle are one record).  Rows are spread over `nthreads` threads.
 * out: [0] rays, [1] bins != BVH, [2] product != reference, [3] 1 if bins
 * were built, [4] rays in cells over the cap (BVH walk), [5] rays with a tie,
 * [6] rays that took the kd fallback, [7] everywhere hulls, [8] hits,
 * [9] bin records, [10] 1 if the camera is beyond prune_origin_max.
 * sample: n_sample pixel indices whose product answer (slot's triangle or -1,
 * t bits) goes to sample_out (2 per pixel), for the oracle comparison. */
extern "C" int bins_fuzz(const crt_scene_desc *desc, int nthreads, uint64_t *out, const int64_t *sample,
                         int64_t n_sample, int64_t *sample_out) {
    HostScene hs;
    int rc = prepare_scene(desc, hs);
    if (rc != CRT_OK) return rc;
    if (hs.bnode_count == 0 && ((rc = build_bvh(hs)) != CRT_OK || (rc = build_proof_tables(hs)) != CRT_OK)) return rc;
    std::vector<CamCand> bins;
    std::vector<int32_t> off;
    std::vector<uint8_t> over;
    if ((rc = build_camera_bins(hs, bins, off, &over)) != CRT_OK) return rc;
    for (int k = 0; k < 11; ++k) out[k] = 0;
    const bool built = !off.empty();
    out[3] = built;
    out[9] = bins.size();
    {
        BinCamera cam;
        if (bin_camera(hs, cam)) {
            std::vector<CamCand> tpl;
            bin_templates(hs, tpl);
            for (const CamCand &c : tpl) {
                const float lo[3] = {c.lo_x, c.lo_y, c.lo_z}, hi[3] = {c.hi_x, c.hi_y, c.hi_z};
                out[7] += bin_project(lo, hi, cam).every;
            }
        }
        for (int k = 0; k < 3; ++k) out[10] |= !(std::fabs(hs.cam_loc[k]) <= hs.prune_origin_max);
    }
    auto ok = [](float x) {
        const float m = std::fabs(x);
        return x == 0.0f || (m >= 0x1p-40f && m <= 0x1p62f);
    };
    bool planes_ok = true;   /* as crt_api.hip scene_upload */
    for (const DNode &n : hs.nodes)
        planes_ok = planes_ok && ok(n.lo_x) && ok(n.lo_y) && ok(n.lo_z) && ok(n.hi_x) && ok(n.hi_y) && ok(n.hi_z) &&
                    n.lo_x <= n.hi_x && n.lo_y <= n.hi_y && n.lo_z <= n.hi_z;
    DeviceScene ds{};
    const DCamera cam = host_camera(hs);
    const int W = hs.width, H = hs.height, tx = (W + 7) / 8;
    std::vector<int32_t> res_slot((size_t)W * H);
    std::vector<float> res_t((size_t)W * H);
    const int nth = std::max(1, std::min(64, nthreads));
    std::vector<std::array<uint64_t, 7>> part((size_t)nth);
    auto work = [&](int th) {
        std::array<uint64_t, 7> c{};
        for (int y = th; y < H; y += nth)
            for (int x = 0; x < W; ++x) {
                Vec o, d;
                camera_ray(cam, x, y, o, d);
                const PruneRay pr = make_prune_ray(o, d, hs.prune_origin_max);
                WalkCounts w = {0u, 0u};
                float t1 = 0.f, t2 = 0.f;
                bool tie1 = false, tie2 = false;
                const int a = walk_bvh<false>(bnode_order(hs.bnodes.data(), hs.bnode_count, ray_octant(d)),
                                              hs.bnode_count, hs.btri.data(), hs.btri_id.data(), o, d, pr, t1, tie1, w);
                const int cell = (y / 8) * tx + x / 8;
                int tri = a;
                float tt = t1;
                bool tie = tie1;
                if (built && !over[(size_t)cell]) {
                    const int b = walk_bins<false>(bins.data(), off[cell], off[cell + 1], 8 * (y % 8) + x % 8, o, d, pr,
                                                   t2, tie2, w);
                    uint32_t u1, u2;
                    std::memcpy(&u1, &t1, 4);
                    std::memcpy(&u2, &t2, 4);
                    if ((a < 0) != (b < 0) || (a >= 0 && (u1 != u2 || tie1 != tie2 || (!tie1 && a != b)))) ++c[1];
                    tri = b;
                    tt = t2;
                    tie = tie2;
                } else if (built) {
                    ++c[4];
                }
                c[5] += tri >= 0 && tie;
                bool fb = false;
                float bt = 0.f;
                const int slot = resolve_closest<false>(hs.nodes.data(), hs.pnodes.data(), (int)hs.nodes.size(),
                                                        hs.slots.data(), hs.slot_cull.data(), hs.slot_tri.data(),
                                                        hs.ktopo.empty() ? nullptr : hs.ktopo.data(), planes_ok, o, d,
                                                        pr, tri, tt, tie, bt, w, &fb);
                c[6] += fb;
                float rt = 0.f;
                uint64_t rn = 0, rtr = 0;
                const int rs = walk_reference(hs, o, d, rt, rn, rtr);
                uint32_t v1, v2;
                std::memcpy(&v1, &bt, 4);
                std::memcpy(&v2, &rt, 4);
                /* copies of one triangle in several leaves are the same record (crt_acceleration_tree.cpp:44-58):
                 * the answer is the triangle and t */
                const int ta = slot >= 0 ? hs.slot_tri[(size_t)slot] : -1, tb = rs >= 0 ? hs.slot_tri[(size_t)rs] : -1;
                if (ta != tb || (slot >= 0 && v1 != v2)) ++c[2];
                c[3] += slot >= 0;
                ++c[0];
                res_slot[(size_t)y * W + x] = slot;
                res_t[(size_t)y * W + x] = bt;
            }
        part[(size_t)th] = c;
    };
    std::vector<std::thread> pool;
    for (int th = 0; th < nth; ++th) pool.emplace_back(work, th);
    for (auto &t : pool) t.join();
    for (const auto &c : part) {
        out[0] += c[0];
        out[1] += c[1];
        out[2] += c[2];
        out[4] += c[4];
        out[5] += c[5];
        out[6] += c[6];
        out[8] += c[3];
    }
    for (int64_t i = 0; i < n_sample; ++i) {
        const int64_t p = sample[i];
        if (p < 0 || p >= (int64_t)W * H) return -1;
        const int s = res_slot[(size_t)p];
        uint32_t u;
        std::memcpy(&u, &res_t[(size_t)p], 4);
        sample_out[2 * i] = s >= 0 ? hs.slot_tri[(size_t)s] : -1;
        sample_out[2 * i + 1] = s >= 0 ? (int64_t)u : 0;
    }
    return CRT_OK;
}
