/*
 * crt_gi_machine.h — GI frames (15-01/scene2, C4) as a per-lane state machine
 * (compiled in crt_render_gi.hip; declared in crt_kernels.h).
 *
 * What it computes: render_region + shade_ray (crt_renderer.cpp:46-155) for
 * every pixel of a tile list, each pixel's rays in the reference's
 * depth-first order with its own PCG stream (seed (x, y), crt_random.h), so
 * the image bits do not depend on which lane or when a pixel runs.
 *
 * How: persistent waves; every lane owns one pixel at a time and runs it as a
 * state machine — WALK (one step of the BVH walk of its current ray per loop
 * round, crt_bvh.h), then RESOLVE (the proof on the reference tree, the
 * hit's shading, the pending activations, the next ray or the pixel's end and
 * the next pixel).  A wave keeps stepping its walking lanes and resolves the
 * waiting ones only once half of its lanes wait (or none walks any more): a
 * lane whose ray is short no longer idles until the wave's longest walk ends,
 * and the long resolve code runs for many lanes at once.
 *
 * Pending activations (the recursion's frames): the frame of an activation
 * whose children are traced lives at index = its ray depth.  The two deepest
 * such depths (max_ray_depth - 2, - 1: the ones every bounce touches) are in
 * LDS, one 16-float frame per lane (8 KB per wave); the one above them
 * (max_ray_depth - 3, C4's depth 0) in registers; shallower ones (deep
 * recursion only) in a global buffer, 64 contiguous bytes per (lane, depth).
 * An activation at depth max_ray_depth has only untraced (black) children and
 * is resolved on the spot (its GI draws are still taken, crt_renderer.cpp:
 * 61-78).
 *
 * The walk postpones leaves (speculative while-while): a node step is
 * branch-free, a lane reaching a live leaf parks it and waits, and the leaf
 * triangles are tested when enough lanes hold one (or no lane can step), so
 * the triangle code runs for many lanes at once instead of for the few lanes
 * that happen to sit on a leaf in each round.
 */
#pragma once
#include "crt_shade.h"

namespace crt_amd {

constexpr int kGiLdsFrames = 2;

struct GiLds {
    float f[4][kGiLdsFrames][16][64];   /* [wave][slot][field][lane] */
};

/* One pending activation, 16 floats (kind: crt_render.hip FrameKind):
 *   diffuse GI: acc (GI sum), p, n (hit), r (right of from_axes), alb, meta
 *   reflect:    acc (albedo)
 *   refract:    acc (reflection colour, kind B), p / n = refraction ray o / d, alb.x = fresnel
 * meta = kind | has_refr << 2 | i << 3 (i: GI rays done). */
struct GiFrame {
    Vec acc, p, n, r, alb;
    uint32_t meta;
};

struct GiFrames {
    GiLds *L;
    float4 *g;                  /* this lane's frames of depths < base - 1: 4 float4 each */
    int w, lane, base;          /* LDS holds depths base, base + 1; registers base - 1 */
    float reg[16];

    __device__ __forceinline__ GiFrame load(int k) const {
        float v[16];
        const int sl = k - base;
        if (sl == -1) {
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = reg[q];
        } else if (sl >= 0 && sl < kGiLdsFrames) {
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = L->f[w][sl][q][lane];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 x = load_global(g, 4 * k + q);
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
        }
        GiFrame f;
        f.acc = vec(v[0], v[1], v[2]);
        f.p = vec(v[3], v[4], v[5]);
        f.n = vec(v[6], v[7], v[8]);
        f.r = vec(v[9], v[10], v[11]);
        f.alb = vec(v[12], v[13], v[14]);
        f.meta = __float_as_uint(v[15]);
        return f;
    }
    __device__ __forceinline__ void store(int k, const GiFrame &f) {
        const float v[16] = {f.acc.x, f.acc.y, f.acc.z, f.p.x, f.p.y, f.p.z, f.n.x, f.n.y, f.n.z,
                             f.r.x,   f.r.y,   f.r.z,   f.alb.x, f.alb.y, f.alb.z, __uint_as_float(f.meta)};
        const int sl = k - base;
        if (sl == -1) {
#pragma unroll
            for (int q = 0; q < 16; ++q) reg[q] = v[q];
        } else if (sl >= 0 && sl < kGiLdsFrames) {
#pragma unroll
            for (int q = 0; q < 16; ++q) L->f[w][sl][q][lane] = v[q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) g[4 * k + q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
    }
};

/* The GI direction of a diffuse activation (gi_ray, crt_renderer.cpp:61-77)
 * with forward = right x n recomputed (same operations as at the push). */
__device__ __forceinline__ void gi_dir(const DeviceScene &s, const DSettings &st, const GiFrame &f, Pcg32 &rng,
                                       Vec &o, Vec &d) {
    Frame fr;
    fr.p = f.p;
    fr.n = f.n;
    fr.a = f.r;
    fr.b = vcross(f.r, f.n);
    gi_ray(s, st, fr, rng, o, d);
}

/* Walk state of one lane's current ray (crt_bvh.h walk_bvh, one node per step) */
struct GiWalk {
    const BNode *nodes;   /* the ray's octant order */
    PruneRay pr;
    int i;
    float lim, t;
    int tri;
    bool tie;
    int leaf;             /* parked leaf (BNode::leaf), 0 = none */
};

__device__ __forceinline__ void gi_walk_begin(const DeviceScene &s, GiWalk &w, Vec o, Vec d) {
    w.nodes = bnode_order(s.bnodes, s.bnode_count, ray_octant(d));
    w.pr = make_prune_ray(o, d, s.prune_origin_max);
    w.i = 0;
    w.lim = INFINITY;
    w.t = 0.0f;
    w.tri = -1;
    w.tie = false;
    w.leaf = 0;
    /* rays with a NaN component miss every cell (crt_bvh.h trace_bvh_exact) */
    if (isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z)) w.i = s.bnode_count;
}

/* one node of the walk, branch-free: descend / move on, and park a live leaf */
template <bool COUNT>
__device__ __forceinline__ void gi_walk_node(GiWalk &w, LaneCounts &c) {
    const BNode nd = load_global(w.nodes, w.i);
    if (COUNT) ++c.nodes;
    const bool alive = bnode_alive(nd, w.pr, w.lim);
    w.i = alive ? w.i + 1 : nd.skip;      /* a leaf's skip is i + 1 */
    w.leaf = alive ? nd.leaf : 0;
}

/* the parked leaf's triangles (crt_bvh.h walk_bvh) */
template <bool COUNT>
__device__ __forceinline__ void gi_walk_leaf(const DeviceScene &s, GiWalk &w, Vec o, Vec d, LaneCounts &c) {
    const int cnt = w.leaf & 15;
    const int first = w.leaf >> 4;
    w.leaf = 0;
    for (int k = 0; k < cnt; ++k) {
        const DTriGeo g = load_global(s.btri, first + k);
        const int32_t id = load_global(s.btri_id, first + k);
        const uint8_t cull = (uint8_t)((uint32_t)id >> 31);
        float t;
        if (COUNT) ++c.tris;
        if (tri_hit(o, d, g, &cull, t)) {
            if (w.tri < 0 || t < w.t) {
                w.t = t;
                w.tri = id & 0x7fffffff;
                w.tie = false;
                w.lim = t;
            } else if (t == w.t) {
                w.tie = true;
            }
        }
    }
}

/* The walk's answer as the reference's (slot, t): proof on the reference
 * tree, else the exact pruned kd walk (crt_bvh.h steps 2-3). */
template <bool COUNT>
__device__ __forceinline__ int gi_walk_finish(const DeviceScene &s, const GiWalk &w, Vec o, Vec d, float &t,
                                              LaneCounts &c) {
    t = 0.0f;
    if (w.tri < 0) return -1;
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    WalkCounts wc = {0u, 0u};
    int slot = -1;
    if (!w.tie) {
        const Vec p = vadd(o, vscale(d, w.t));
        slot = CRT_PROOF_TOPO && s.ktopo ? verify_topo<COUNT>(s.ktopo, s.nodes, s.slot_tri, w.tri, o, d, rr, p, wc,
                                                                   CRT_PROOF_TOPO2 ? s.ktopo2 : nullptr)
                                         : verify_kd<COUNT>(s.nodes, s.slot_tri, w.tri, o, d, rr, p, wc);
        t = w.t;
    }
    if (slot < 0)
        slot = walk_pruned<COUNT>(pnode_order(s.pnodes, s.node_count, ray_octant(d)), s.node_count, s.slots,
                                  s.slot_cull, o, d, rr, w.pr, t, wc);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
    }
    return slot;
}

#ifndef CRT_GIM_WAVES
#define CRT_GIM_WAVES 4      /* min waves/SIMD of the GI machine */
#endif
#ifndef CRT_GIM_WAIT
#define CRT_GIM_WAIT 48      /* a wave resolves once this many of its lanes wait (C4 1080^2: 16 / 32 / 40 / 48 / 56 / 62 -> 41.5 / 30.1 / 28.4 / 28.0 / 28.6 / 30.8 ms, profiles/r03/ab_gim) */
#endif

#ifndef CRT_GIM_LEAVES
#define CRT_GIM_LEAVES 16    /* ... and tests parked leaves once this many lanes hold one (8 / 16 / 24 / 32 / 40: 32.3 / 27.6 / 28.0 / 28.2 / 31.6 ms) */
#endif

/* gframes: (grid lanes) x max(0, max_ray_depth - 3) frames of 64 B */
template <bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CRT_GIM_WAVES))) void k_render_gi(
    const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles, int ntiles,
    float *__restrict__ out, int32_t *__restrict__ next_px, unsigned long long *__restrict__ counters,
    float4 *__restrict__ gframes) {
    const int lane = (int)(threadIdx.x & 63);
    const DeviceScene &s = *scene;
    const int total = ntiles * 64;   /* pixel slots: tile k, lane j -> (j & 7, j >> 3) inside tile k */
    const unsigned long long lt = (1ull << lane) - 1ull;
    __shared__ GiLds lds;
    GiFrames fs;
    fs.L = &lds;
    fs.w = (int)(threadIdx.x >> 6);
    fs.lane = lane;
    fs.base = (int)st.max_ray_depth - kGiLdsFrames;
    fs.g = gframes + (int64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 4 * (fs.base > 1 ? fs.base - 1 : 0);
    LaneCounts cnt = {};
    const uint32_t maxd = st.max_ray_depth, nrays = st.diffuse_reflection_ray_count;
    const Vec bg = vec(s.background[0], s.background[1], s.background[2]);

    bool has = false, dry = false, walking = false;
    int opx = 0;
    uint32_t px = 0, py = 0, depth = 0;
    Vec o = vec(0.f, 0.f, 0.f), d = vec(0.f, 0.f, 1.f);
    Pcg32 rng;
    rng.state = 0;
    rng.inc = 1;
    GiWalk w;
    gi_walk_begin(s, w, o, d);
    for (;;) {
        /* ---- lanes without a pixel take the next slots of the list ---- */
        const unsigned long long need = __ballot(!has && !dry);
        if (need != 0ull) {
            const int leader = __ffsll((long long)need) - 1;
            int b = 0;
            if (lane == leader) b = atomicAdd(next_px, __popcll(need));
            b = __shfl(b, leader);
            if (!has && !dry) {
                const int k = b + __popcll(need & lt);
                if (k >= total) {
                    dry = true;
                } else {
                    const Tile tl = tiles[k >> 6];
                    const int lx = k & 7, ly = (k >> 3) & 7;
                    if (lx < tl.w && ly < tl.h) {   /* slots outside a partial tile: retry next round */
                        has = true;
                        opx = (int)(tl.out_base + (int64_t)ly * tl.out_stride + lx);
                        px = (uint32_t)(tl.x + lx);
                        py = (uint32_t)(tl.y + ly);
                        camera_ray(s.cam, (int)px, (int)py, o, d);
                        depth = 0;
                        rng = make_pcg(px, py);
                        if (COUNT) ++cnt.traversals;
                        gi_walk_begin(s, w, o, d);
                        walking = true;
                    }
                }
            }
        }
        const unsigned long long hm = __ballot(has);
        if (hm == 0ull) {
            if (__ballot(!dry) != 0ull) continue;
            break;
        }
        /* ---- WALK: step the walking lanes until enough lanes wait ---- */
        for (;;) {
            const unsigned long long wm = __ballot(walking);
            const int waiting = __popcll(hm) - __popcll(wm);
            if (wm == 0ull || waiting >= CRT_GIM_WAIT) break;
            const bool parked = w.leaf != 0;
            const unsigned long long pm = __ballot(parked);
            if (__popcll(pm) >= CRT_GIM_LEAVES || pm == wm) {   /* leaf round */
                if (parked) {
                    gi_walk_leaf<COUNT>(s, w, o, d, cnt);
                    walking = w.i < s.bnode_count;
                }
            } else if (walking && !parked) {                     /* node round */
                gi_walk_node<COUNT>(w, cnt);
                walking = w.i < s.bnode_count || w.leaf != 0;
            }
        }
        if (!has || walking) continue;
        /* ---- RESOLVE: the hit, its shading, the pending activations ---- */
        float t;
        const int slot = gi_walk_finish<COUNT>(s, w, o, d, t, cnt);
        Vec col = bg;
        bool called = false;
        if (slot >= 0) {
            if (COUNT) ++cnt.hits;
            HitRec h;
            make_hit(s, o, d, t, slot, h);
            const DMaterial m = s.materials[h.mat];
            if (m.type == CRT_MATERIAL_DIFFUSE) {
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (s.gi_on && nrays > 0) {
                    GiFrame f;
                    f.acc = vec(0.f, 0.f, 0.f);
                    f.p = h.p;
                    f.n = h.n;
                    f.r = vnormalize(vcross(d, h.n));          /* right */
                    f.alb = alb;
                    f.meta = (uint32_t)kDiffuseGI;
                    if (depth < maxd) {                        /* children traced: a pending activation */
                        fs.store((int)depth, f);
                        gi_dir(s, st, f, rng, o, d);
                        depth = depth + 1;
                        called = true;
                    } else {                                   /* children untraced: black, draws taken */
                        for (uint32_t i = 0; i < nrays; ++i) {
                            (void)rng.next();
                            (void)rng.next();
                        }
                        col = diffuse_finish(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb);
                    }
                } else {
                    col = diffuse_finish(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb);
                }
            } else if (m.type == CRT_MATERIAL_REFLECTIVE) {                  /* :103-107 */
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (s.reflections_on) {
                    if (depth < maxd) {
                        GiFrame f;
                        f.acc = alb;
                        f.meta = (uint32_t)kReflect;
                        fs.store((int)depth, f);
                        o = vadd(h.p, vscale(h.n, st.reflection_bias));
                        d = vsub(d, vscale(vscale(h.n, 2.0f), vdot(d, h.n)));
                        depth = depth + 1;
                        called = true;
                    } else {
                        col = vmul_quirk(alb, vec(0.f, 0.f, 0.f));
                    }
                } else {
                    col = alb;
                }
            } else if (m.type == CRT_MATERIAL_REFRACTIVE) {                  /* :109-135 */
                if (!s.refractions_on) {
                    col = vec(0.f, 0.f, 0.f);
                } else {
                    Vec n = h.n;
                    float n_out = 1.0f, n_in = m.ior;
                    if (vdot(d, n) > 0.0f) {
                        n = vneg(n);
                        const float tmp = n_in; n_in = n_out; n_out = tmp;
                    }
                    uint32_t has_refr = 0;
                    Vec rd = d;
                    {   /* Vector::refract (crt_vector.cpp:11-27) */
                        const float ca = -vdot(rd, n);
                        const float sa = sqrtf(1.0f - ca * ca);
                        if (!(sa > n_in / n_out)) {
                            const float sb = sa * n_out / n_in;
                            const float cb = sqrtf(1.0f - sb * sb);
                            rd = vadd(rd, vscale(n, ca));
                            rd = vnormalize(rd);
                            rd = vscale(rd, sb);
                            rd = vadd(rd, vscale(vneg(n), cb));
                            has_refr = 1;
                        }
                    }
                    const float fr = fresnel_of(s, vdot(d, n));
                    if (depth < maxd) {
                        GiFrame f;
                        f.acc = vec(0.f, 0.f, 0.f);
                        f.p = vadd(h.p, vscale(vneg(n), 1e-2f));   /* refract_at's default bias (crt_ray.h:30-50) */
                        f.n = rd;
                        f.alb = vec(fr, 0.f, 0.f);
                        f.meta = (uint32_t)kRefractA | (has_refr << 2);
                        fs.store((int)depth, f);
                        o = vadd(h.p, vscale(n, st.reflection_bias));
                        d = vsub(d, vscale(vscale(n, 2.0f), vdot(d, n)));
                        depth = depth + 1;
                        called = true;
                    } else {                                   /* both children black, untraced */
                        const Vec black = vec(0.f, 0.f, 0.f);
                        col = has_refr ? vadd(vscale(black, fr), vscale(black, 1.0f - fr)) : black;
                    }
                }
            } else {                                                          /* Constant :137-139 */
                col = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
            }
        }
        /* ---- return col to the pending activations until one needs a ray ---- */
        while (!called && depth > 0) {
            const int k = (int)depth - 1;
            GiFrame f = fs.load(k);
            const uint32_t kind = f.meta & 3u;
            if (kind == (uint32_t)kDiffuseGI) {
                f.acc = vadd(f.acc, col);
                const uint32_t i = (f.meta >> 3) + 1;
                if (i < nrays) {
                    f.meta = (uint32_t)kDiffuseGI | (i << 3);
                    fs.store(k, f);
                    gi_dir(s, st, f, rng, o, d);
                    called = true;           /* depth stays k + 1 */
                } else {
                    col = diffuse_finish(s, st, f.acc, f.p, f.n, f.alb);
                    depth = (uint32_t)k;
                }
            } else if (kind == (uint32_t)kReflect) {
                col = vmul_quirk(f.acc, col);
                depth = (uint32_t)k;
            } else if (kind == (uint32_t)kRefractA) {
                if ((f.meta >> 2) & 1u) {
                    f.acc = col;
                    f.meta = (uint32_t)kRefractB | (1u << 2);
                    fs.store(k, f);
                    o = f.p;
                    d = f.n;
                    called = true;           /* depth stays k + 1 */
                } else {
                    depth = (uint32_t)k;     /* total internal reflection: the reflection colour */
                }
            } else {
                const float fr = f.alb.x;
                col = vadd(vscale(f.acc, fr), vscale(col, 1.0f - fr));
                depth = (uint32_t)k;
            }
        }
        if (called) {
            if (COUNT) ++cnt.traversals;
            gi_walk_begin(s, w, o, d);
            walking = true;
        } else {
            float *po = out + 3 * (int64_t)opx;
            po[0] = col.x;
            po[1] = col.y;
            po[2] = col.z;
            has = false;
        }
    }
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
    }
}



}  // namespace crt_amd
