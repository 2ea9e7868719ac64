/*
 * crt_walks.h — the tree walks of the render kernels (crt_intersection.cpp:
 * 14-136 and the exact variants of DESIGN.md §4.1-4.2), all bit-identical in
 * result: reference order (7, 4), pruned packet (8, 12), window (13), pruned
 * cooperative (10), per-lane BVH + proof (14, crt_bvh.h).
 */
#pragma once
#include "crt_kernel_common.h"

namespace crt_amd {

/* ---------------------------------------------------------------------- */
/* ray_intersect_acceleration_tree (crt_intersection.cpp:109-136)           */
/* ---------------------------------------------------------------------- */
template <bool COUNT>
__device__ __forceinline__ int trace_closest(const DeviceScene &s, Vec o, Vec d, float &best_t, LaneCounts &c) {
    int best = -1;
    best_t = 0.0f;
    int i = 0;
    const int n = s.node_count;
    if (COUNT) ++c.traversals;
    while (i < n) {
        const DNode nd = s.nodes[i];
        const bool pass = box_hit(o, d, nd);
        if (COUNT) ++c.nodes;
        if (nd.b < 0) {               /* interior: descend on pass, else skip the subtree */
            i = pass ? i + 1 : nd.a;
            continue;
        }
        if (pass) {                    /* leaf: ray_intersect_triangle_span, strict '<' keeps the first */
            for (int k = 0; k < node_leaf_count(nd); ++k) {
                const int slot = nd.b + k;
                float t;
                if (COUNT) ++c.tris;
                if (tri_hit(o, d, s.slots[slot], s.slot_cull + slot, t) && (best < 0 || t < best_t)) {
                    best_t = t;
                    best = slot;
                }
            }
        }
        ++i;
    }
    if (COUNT && best >= 0) ++c.hits;
    return best;
}

/* ---------------------------------------------------------------------- */
/* Wave-cooperative walk (TRAV 4)                                           */
/* ---------------------------------------------------------------------- */
/* In the traversal-ordered layout every subtree is a contiguous node range
 * and a range made of whole subtrees can be walked stacklessly on its own.
 * So the reference's walk of one ray (the range [0, n)) can be cut into
 * pieces at any passing interior node i: [i+1, skip(i+1)) stays with the lane
 * (child1's subtree), [skip(i+1), end) is donated to the wave.  Idle lanes —
 * lanes whose own ray is done or cheap — pop donated pieces, so a ray that
 * crosses hundreds of nodes no longer serialises its whole wave.
 *
 * Exactness: the pieces partition exactly the node sequence the reference
 * visits (same box test per node, same leaves, same triangles), and the
 * winner is merged with a 64-bit key (t, slot): slots are numbered in the
 * reference's visit order, so the smallest key is the reference's first-found
 * closest hit (t >= 0; -0 and +0 are both mapped to 0, as '<' treats them). */
constexpr int kCoopStack = 448;   /* donated pieces per wave */

struct alignas(16) CoopLds {
    float ray[64][6];                       /* o, d of each lane's ray */
    unsigned long long key[64];             /* (t bits << 32) | slot, per ray */
    unsigned long long stack[kCoopStack];   /* ray(6) | start(29) | end(29) */
    int sp;                                 /* banked pieces (TRAV 5) */
    int pad[3];
};

__device__ __forceinline__ unsigned long long coop_key(float t, int slot) {
    const unsigned tb = t == 0.0f ? 0u : __float_as_uint(t);
    return ((unsigned long long)tb << 32) | (unsigned)slot;
}
__device__ __forceinline__ unsigned long long coop_piece(int ray, int start, int end) {
    return ((unsigned long long)ray << 58) | ((unsigned long long)start << 29) | (unsigned long long)end;
}

/* Node access of the sharing walks: the reference-order DNode array, or
 * (PRUNE) the octant-ordered PNode array of the piece's ray with its hull. */
template <bool PRUNE> struct WalkNode;
template <> struct WalkNode<false> {
    using T = DNode;
    static __device__ __forceinline__ const DNode *base(const DeviceScene &s, Vec) { return s.nodes; }
    static __device__ __forceinline__ DNode cell(const DNode &n) { return n; }
    static __device__ __forceinline__ bool alive(const DNode &, const PruneRay &, float) { return true; }
};
template <> struct WalkNode<true> {
    using T = PNode;
    static __device__ __forceinline__ const PNode *base(const DeviceScene &s, Vec d) {
        return pnode_order(s.pnodes, s.node_count, ray_octant(d));
    }
    static __device__ __forceinline__ DNode cell(const PNode &n) { return cell_of(n); }
    static __device__ __forceinline__ bool alive(const PNode &n, const PruneRay &p, float lim) {
        return hull_alive(n, p, lim);
    }
};

__device__ __forceinline__ float key_t(unsigned long long k) {
    return k == ~0ull ? INFINITY : __uint_as_float((unsigned)(k >> 32));
}

template <bool COUNT, bool PRUNE>
__device__ int trace_coop(const DeviceScene &s, CoopLds &L, bool active, Vec o, Vec d, float &best_t,
                          LaneCounts &c) {
    using WN = WalkNode<PRUNE>;
    using NT = typename WN::T;
    const int lane = (int)(threadIdx.x & 63);
    const int n = s.node_count;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    L.ray[lane][0] = o.x; L.ray[lane][1] = o.y; L.ray[lane][2] = o.z;
    L.ray[lane][3] = d.x; L.ray[lane][4] = d.y; L.ray[lane][5] = d.z;
    L.key[lane] = ~0ull;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (COUNT && active) ++c.traversals;
    if (COUNT) ++c.wave_tris;           /* coop walks: wave_tris = calls, wave_nodes = loop rounds */

    int r = lane;                       /* ray of the piece this lane walks */
    int i = active ? 0 : n, end = n;    /* the piece: [i, end) */
    int lf = 0, lc = 0, k = 0;          /* pending leaf triangles */
    Vec ro = o, rd = d;
    const NT *nb = WN::base(s, d);
    PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);   /* hoisted exact divisions (box_hit_r) */
    float lim = INFINITY;               /* best t known for the piece's ray (pruning bound) */
    unsigned long long mine = ~0ull;    /* best key found in the current piece */
    int sp = 0;                         /* wave-uniform stack depth */
    NT nd = load_global(nb, 0);
    for (;;) {
        if (COUNT) ++c.wave_nodes;
        bool busy = (i < end) || (lc > 0);
        /* ---- idle lanes pop donated pieces ---- */
        const unsigned long long idle = __ballot(!busy);
        if (idle != 0ull && sp > 0) {
            const int nidle = __popcll(idle);
            const int take = nidle < sp ? nidle : sp;
            if (!busy) {
                const int rank = __popcll(idle & lt_mask);
                if (rank < take) {
                    const unsigned long long pc = L.stack[sp - 1 - rank];
                    r = (int)(pc >> 58);
                    i = (int)((pc >> 29) & 0x1fffffff);
                    end = (int)(pc & 0x1fffffff);
                    ro = vec(L.ray[r][0], L.ray[r][1], L.ray[r][2]);
                    rd = vec(L.ray[r][3], L.ray[r][4], L.ray[r][5]);
                    nb = WN::base(s, rd);
                    rr = make_ray_rcp(ro, rd, s.planes_ok != 0);
                    if (PRUNE) {
                        pr = make_prune_ray(ro, rd, s.prune_origin_max);
                        lim = key_t(L.key[r]);
                    }
                    nd = load_global(nb, i);
                    busy = true;
                }
            }
            sp -= take;
        }
        if (!__any(busy)) break;
        /* ---- one step per busy lane: a triangle of its pending leaf, or a node ---- */
        bool donate = false;
        int rest = 0;
        if (busy) {
            if (lc > 0) {
                const int slot = lf + k;
                float t;
                if (COUNT) ++c.tris;
                /* the whole record and its cull flag in one round trip; branch-free
                 * test (a wave's scattered lanes take every branch of tri_hit anyway) */
                const DTriGeo g = load_global(s.slots, slot);
                const bool cl = load_global(s.slot_cull, slot) != 0;
                if (tri_hit_bf(ro, rd, g, cl, t)) {
                    const unsigned long long kk = coop_key(t, slot);
                    mine = kk < mine ? kk : mine;
                    if (PRUNE) lim = fminf(lim, t);
                }
                if (++k == lc) lc = 0;
            } else {
                const int i1 = i + 1 < n ? i + 1 : n - 1;
                const int alt = nd.b < 0 ? (nd.a < n ? nd.a : n - 1) : i1;
                const NT n1 = load_global(nb, i1);
                const NT n2 = load_global(nb, alt);
                bool pass = false;
                if (WN::alive(nd, pr, lim)) {
                    pass = box_hit_r(ro, rd, rr, WN::cell(nd));
                    if (COUNT) ++c.nodes;
                }
                if (nd.b < 0) {
                    if (pass) {
                        /* first child = i+1; its subtree ends at skip(i+1) */
                        rest = n1.b < 0 ? n1.a : i + 2;
                        donate = rest < end;
                        i = i + 1;
                        nd = n1;
                    } else {
                        i = nd.a;
                        nd = n2;
                    }
                } else {
                    if (pass) { lf = nd.b; lc = (nd.a & 0xffffff); k = 0; }
                    i = i + 1;
                    nd = n1;
                }
            }
            if (i >= end && lc == 0) {          /* piece finished: merge into its ray's key */
                atomicMin(&L.key[r], mine);
                mine = ~0ull;
            }
        }
        /* ---- donate the remainder of a split walk while lanes are (about to be) idle ---- */
        const unsigned long long want = __ballot(donate);
        if (want != 0ull) {
            const unsigned long long idle_next = __ballot(!((i < end) || (lc > 0)));
            const int room = __popcll(idle_next) + 8 - sp;   /* keep a few pieces banked */
            const int cap = kCoopStack - sp;
            const int give = __popcll(want) < room ? __popcll(want) : (room > 0 ? room : 0);
            const int g = give < cap ? give : cap;
            if (donate) {
                const int rank = __popcll(want & lt_mask);
                if (rank < g) {
                    L.stack[sp + rank] = coop_piece(r, rest, end);
                    end = rest;
                }
            }
            sp += g;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const unsigned long long kk = L.key[lane];
    if (!active || kk == ~0ull) return -1;
    const int slot = (int)(kk & 0xffffffffu);
    float t = 0.0f;
    (void)tri_hit(o, d, s.slots[slot], s.slot_cull + slot, t);   /* exact t (keeps the sign of a zero) */
    best_t = t;
    if (COUNT) ++c.hits;
    return slot;
}

/* ---------------------------------------------------------------------- */
/* Masked packet walk (TRAV 7) — coherent rays (primary rays of a tile)     */
/* ---------------------------------------------------------------------- */
/* The whole wave walks the traversal-ordered node array with ONE wave-uniform
 * index, so node and triangle records come through the scalar path (SGPRs)
 * and the control flow never diverges.  Each lane keeps 64 reach bits: bit D
 * is set iff every ancestor at depths < D of the current depth-D node passed
 * its box test for this lane's ray.  A node is tested for the lanes whose bit
 * is set; an interior node where no lane passes is skipped, otherwise the walk
 * descends with bit D+1 = this lane's pass.  Every lane therefore tests
 * exactly the nodes, leaves and triangles the reference visits for its ray, in
 * the reference's order (strict '<' keeps the first-found winner); the wave
 * pays once per node of the union of its lanes' visit sets.  Tree depth is at
 * most 40 (crt_acceleration_tree.h:12), within the 64 bits. */

template <bool COUNT>
__device__ int trace_packet(const DeviceScene &s, bool active, Vec o, Vec d, float &best_t, LaneCounts &c) {
    int best = -1;
    best_t = 0.0f;
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    unsigned long long reach = active ? 1ull : 0ull;
    if (COUNT && active) ++c.traversals;
    const int n = s.node_count;
    int i = 0;
    while (i < n) {
        i = uniform_i(i);
        const DNode nd = load_scalar(s.nodes, i);
        const int depth = node_depth(nd);
        const bool in = ((reach >> depth) & 1ull) != 0ull;
        const bool pass = in && box_hit_r(o, d, rr, nd);
        if (COUNT && in) ++c.nodes;
        if (COUNT) ++c.wave_nodes;
        const unsigned long long pm = __ballot(pass);
        if (nd.b < 0) {
            if (pm != 0ull) {
                const unsigned long long bit = 2ull << depth;
                reach = pass ? (reach | bit) : (reach & ~bit);
                i = i + 1;
            } else {
                i = nd.a;
            }
        } else {
            if (pm != 0ull) {
                const int first = nd.b, cnt = node_leaf_count(nd);
                for (int k = 0; k < cnt; ++k) {
                    const int slot = uniform_i(first + k);
                    const DTriGeo g = load_scalar(s.slots, slot);
                    const bool cull = ((load_scalar(s.slot_cull_bits, slot >> 5) >> (slot & 31)) & 1u) != 0u;
                    float t;
                    if (COUNT && pass) ++c.tris;
                    if (COUNT) ++c.wave_tris;
                    /* the edge tests only matter for a lane whose candidate
                     * distance would replace its best: skip them when no lane
                     * of the wave has one (same predicate, same arithmetic) */
                    const bool pre = pass && tri_plane(o, d, g, cull, t) && (best < 0 || t < best_t);
                    const bool any = __ballot(pre) != 0ull;
                    if (COUNT && any) ++c.wave_edges;
                    if (any && pre && tri_edges(o, d, g, t)) {
                        best_t = t;
                        best = slot;
                    }
                }
            }
            i = i + 1;
        }
    }
    if (COUNT && best >= 0) ++c.hits;
    return best;
}

/* ---------------------------------------------------------------------- */
/* Pruned walks (TRAV 8/12 packet, per-lane for the trace hook) over the    */
/* PNode arrays (crt_layout.h)                                               */
/* ---------------------------------------------------------------------- */
/* TRAV 8: the masked packet walk of TRAV 7 where a lane also drops a subtree
 * whose triangle hull it cannot hit at or before its best t (hull_alive), and
 * the wave walks the node order of the octant most of its lanes share, so
 * near children come first and best t shrinks early.  The wave skips the
 * six-face tests of a node no lane keeps alive.  Candidates are merged by
 * the key (t, slot), which equals the reference's first-found rule in any
 * visit order; every lane still tests its reference-eligible leaves only
 * (a lane enters a node iff its ancestors' cells passed for its ray). */
/* Exact box test for rays outside the hoisted-division window (crt_device.h
 * coord_ok) — out of line, so the packet walk's registers are sized for the
 * fast path; camera rays of every course scene take the fast path. */
__device__ __noinline__ bool box_hit_slow(Vec o, Vec d, const DNode n) {
    const RayRcp r = make_ray_rcp(o, d, false);
    return box_hit_r(o, d, r, n);
}

/* Face cache of the fast packet walk.  A node's six-face test reads, per
 * axis, the quotients and hit points of its two planes on that axis
 * (axis_points) and then only compares them with the other axes' ranges
 * (axis_pass).  Consecutive nodes of the walk share most planes — a child
 * differs from its parent in one plane — so each lane keeps the hit points of
 * the planes the wave last computed, and the wave recomputes an axis only
 * when the node's (lo, hi) pair on it differs from the cached one (a uniform
 * compare of the bit patterns).  Every lane of the wave updates the entries
 * (they do not depend on the lane's reach or best hit), so an entry always
 * holds exactly what box_hit_fast would compute for the cached planes. */
struct FaceCache {
    f2 pu[3], pw[3];
    unsigned long long key[3];   /* bits of the cached (lo, hi) pair per axis: equal in every lane, kept in
                                  * VGPRs (vgpr_u64) — the walk's SGPRs hold the prefetched node records */
};

/* the same value in every lane, in a VGPR pair (an asm result is divergent to the compiler) */
__device__ __forceinline__ unsigned long long vgpr_u64(unsigned long long x) {
    unsigned long long r;
    asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

__device__ __forceinline__ unsigned long long plane_key(float lo, float hi) {
    return ((unsigned long long)__float_as_uint(hi) << 32) | (unsigned long long)__float_as_uint(lo);
}

__device__ __forceinline__ void face_cache_init(FaceCache &fc) {
    for (int a = 0; a < 3; ++a) fc.key[a] = vgpr_u64(~0ull);   /* NaN planes: never a node of a planes_ok tree */
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"   /* branch-free ORs */
__device__ __forceinline__ bool face_cache_pass(FaceCache &fc, const PNode &n, Vec o, Vec d, const RayRcp &r) {
    const unsigned long long kx = plane_key(n.lo_x, n.hi_x), ky = plane_key(n.lo_y, n.hi_y),
                             kz = plane_key(n.lo_z, n.hi_z);
    if (kx != fc.key[0]) {
        axis_points((f2){n.lo_x, n.hi_x}, o.x, d.x, r.y1[0], o.y, d.y, o.z, d.z, fc.pu[0], fc.pw[0]);
        fc.key[0] = vgpr_u64(kx);
    }
    if (ky != fc.key[1]) {
        axis_points((f2){n.lo_y, n.hi_y}, o.y, d.y, r.y1[1], o.z, d.z, o.x, d.x, fc.pu[1], fc.pw[1]);
        fc.key[1] = vgpr_u64(ky);
    }
    if (kz != fc.key[2]) {
        axis_points((f2){n.lo_z, n.hi_z}, o.z, d.z, r.y1[2], o.x, d.x, o.y, d.y, fc.pu[2], fc.pw[2]);
        fc.key[2] = vgpr_u64(kz);
    }
    return axis_pass(fc.pu[0], fc.pw[0], n.lo_y, n.hi_y, n.lo_z, n.hi_z) |
           axis_pass(fc.pu[1], fc.pw[1], n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           axis_pass(fc.pu[2], fc.pw[2], n.lo_x, n.hi_x, n.lo_y, n.hi_y);
}
#pragma clang diagnostic pop

/* Closest-hit candidates of one ray spread over lanes congruent mod G (G a
 * power of two), merged branch-free as one 64-bit key: (t bits, slot) with
 * +-0 as 0 and a zero t's sign kept in slot bit 31 outside the order; no
 * hit = all ones.  Steps below 16 lanes rotate within the row by DPP
 * (row_ror, a multiple of G, so within the class), wider ones use LDS
 * permutes; every lane of a class ends with the class minimum — the
 * reference's first-found choice (key_better) whatever the lane order. */
struct HitKey { unsigned hi, lo; };
__device__ __forceinline__ HitKey hit_key(float t, int slot) {
    if (slot < 0) return HitKey{0xffffffffu, 0xffffffffu};
    return HitKey{t == 0.0f ? 0u : __float_as_uint(t),
                  (unsigned)slot | (__float_as_uint(t) == 0x80000000u ? 0x80000000u : 0u)};
}
__device__ __forceinline__ void hit_key_min(HitKey &k, unsigned ohi, unsigned olo) {
    const unsigned long long a = ((unsigned long long)k.hi << 32) | (k.lo & 0x7fffffffu);
    const unsigned long long b = ((unsigned long long)ohi << 32) | (olo & 0x7fffffffu);
    const bool take = b < a;
    k.hi = take ? ohi : k.hi;
    k.lo = take ? olo : k.lo;
}
template <int CTRL>
__device__ __forceinline__ void hit_key_dpp(HitKey &k) {
    hit_key_min(k, (unsigned)__builtin_amdgcn_update_dpp((int)k.hi, (int)k.hi, CTRL, 0xf, 0xf, false),
                (unsigned)__builtin_amdgcn_update_dpp((int)k.lo, (int)k.lo, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ void hit_key_allmin(HitKey &k, int G) {   /* G wave-uniform */
    if (G <= 1) hit_key_dpp<0x121>(k);   /* row_ror:1 */
    if (G <= 2) hit_key_dpp<0x122>(k);
    if (G <= 4) hit_key_dpp<0x124>(k);
    if (G <= 8) hit_key_dpp<0x128>(k);
    for (int off = G > 16 ? G : 16; off < 64; off <<= 1)
        hit_key_min(k, (unsigned)__shfl_xor((int)k.hi, off), (unsigned)__shfl_xor((int)k.lo, off));
}
/* decode into (t, slot) when the key holds a hit */
__device__ __forceinline__ void hit_key_get(const HitKey &k, float &t, int &slot) {
    if (k.hi != 0xffffffffu) {
        slot = (int)(k.lo & 0x7fffffffu);
        t = k.hi != 0u ? __uint_as_float(k.hi) : ((k.lo & 0x80000000u) ? -0.0f : 0.0f);
    }
}

/* Leaf phase of the fast packet walk when few rays entered the leaf (m of
 * 64 lanes, m <= 32): instead of 64 lanes per triangle with 64 - m of them
 * idle, the wave tests T = 64 / G triangles at once, G >= m lanes per
 * triangle, lane (g, q) testing triangle g (+ T, + 2T, ...) for the q-th
 * entering ray.  The rays' o, d and best keys pass through a per-wave LDS
 * table indexed by rank; each lane filters its candidates by the ray's best
 * key so far (key_better, as the packet loop does), the G-lane groups merge
 * by the key (t, slot) — the reference's first-found rule in any order — and
 * each entering lane takes its ray's result back.  Same tests, same result. */
struct LeafRayLds {
    float4 a[4][32];   /* (d.x, d.y, d.z, best_t) by rank, per wave of the 256-thread block */
    float4 b[4][32];   /* (o.x, o.y, o.z, best as bits) */
};

template <bool COUNT>
__device__ __forceinline__ void leaf_grouped(const DeviceScene &s, int first, int cnt, unsigned long long pm, bool pass,
                                             Vec o, Vec d, float &best_t, int &best, float &lim, LaneCounts &c) {
    __shared__ LeafRayLds L;
    const int w = (int)(threadIdx.x >> 6);
    const int lane = (int)__lane_id();
    const int m = __popcll(pm);
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
    if (pass) {
        L.a[w][rank] = make_float4(d.x, d.y, d.z, best_t);
        L.b[w][rank] = make_float4(o.x, o.y, o.z, __int_as_float(best));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int lg = m <= 1 ? 0 : 32 - __clz(m - 1);   /* G = 2^lg >= m */
    const int G = 1 << lg, T = 64 >> lg;
    const int q = lane & (G - 1), g = lane >> lg;
    const bool qok = q < m;
    const float4 ra = L.a[w][qok ? q : 0], rb = L.b[w][qok ? q : 0];
    const Vec ro = vec(rb.x, rb.y, rb.z), rd = vec(ra.x, ra.y, ra.z);
    float lt = ra.w;
    int ls = __float_as_int(rb.w);
    for (int k0 = 0; k0 < cnt; k0 += T) {
        if (COUNT) ++c.wave_tris;
        const int k = k0 + g;
        if (qok & (k < cnt)) {
            const int slot = first + k;
            const DTriGeo tg = load_global(s.slots, slot);
            const uint8_t cl = load_global(s.slot_cull, slot);
            float t;
            if (COUNT) ++c.tris;
            if (tri_plane(ro, rd, tg, cl != 0, t) && key_better(t, slot, lt, ls) && tri_edges(ro, rd, tg, t)) {
                lt = t;
                ls = slot;
            }
        }
    }
    HitKey key = hit_key(lt, ls);
    hit_key_allmin(key, G);
    key.hi = (unsigned)__shfl((int)key.hi, rank);
    key.lo = (unsigned)__shfl((int)key.lo, rank);
    float nt = 0.0f;
    int ns = -1;
    hit_key_get(key, nt, ns);
    if (pass) {
        best_t = nt;
        best = ns;
        lim = ns >= 0 ? nt : lim;
    }
    __builtin_amdgcn_wave_barrier();   /* the table is rewritten by the next leaf */
}

/* ANY (shadow rays): only whether a hit lies within the light matters — the
 * walk starts with lim0 (a bound past the light, so subtrees beyond it are
 * pruned) and a lane leaves as soon as it holds a hit with t * t <= r2. */
template <bool COUNT, bool FAST, bool ANY = false>
__device__ __forceinline__ int trace_packet_pruned_t(const DeviceScene &s, bool active, Vec o, Vec d,
                                                     const RayRcp &rr, float &best_t, LaneCounts &c,
                                                     float lim0 = INFINITY, float r2 = 0.0f) {
    int best = -1;
    best_t = 0.0f;
    float lim = ANY ? lim0 : INFINITY;
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    unsigned long long reach = active ? 1ull : 0ull;
    const int n = s.node_count;
    const int last = n - 1;
    const int na = __popcll(__ballot(active));
    int oct = 0;
    if (2 * __popcll(__ballot(active && d.x < 0.0f)) > na) oct |= 1;
    if (2 * __popcll(__ballot(active && d.y < 0.0f)) > na) oct |= 2;
    if (2 * __popcll(__ballot(active && d.z < 0.0f)) > na) oct |= 4;
    const PNode *nodes = pnode_order(s.pnodes, n, uniform_i(oct));
    /* The walk is a chain of dependent scalar loads (next index comes from the
     * current record), so each step issues the loads of both possible
     * successors — i+1 (descend / after a leaf) and the skip target — before
     * it tests the current node; the whole 64-B record is read up front.
     * Predicates are combined without short-circuit so the only branches are
     * wave-uniform (no exec-mask save/restore). */
    FaceCache fc;
    face_cache_init(fc);
    int i = 0;
    PNode cur = load_scalar(nodes, 0);
    while (i < n) {
        if (ANY && __ballot(reach != 0ull) == 0ull) break;   /* every lane settled */
        const bool interior = cur.b < 0;
        const int i1 = i + 1 < n ? i + 1 : last;
        const int i2 = interior ? (cur.a < n ? cur.a : last) : i1;
        const PNode n1 = load_scalar(nodes, i1);
        const PNode n2 = load_scalar(nodes, i2);
        const int depth = pnode_depth(cur);
        const bool in = ((reach >> depth) & 1ull) != 0ull;
        const bool alive = in & hull_alive(cur, pr, lim);
        if (COUNT) ++c.wave_nodes;
        bool pass = false;
        if (__ballot(alive) != 0ull) {
            if (COUNT) ++c.wave_box;
            if constexpr (FAST) {
                pass = alive & face_cache_pass(fc, cur, o, d, rr);
            } else {
                pass = alive & box_hit_fast(o, d, rr, cell_of(cur));
            }
            if (!FAST && __ballot(alive & !rr.fast) != 0ull) {
                if (alive & !rr.fast) pass = box_hit_slow(o, d, cell_of(cur));
            }
            if (COUNT && alive) ++c.nodes;
        }
        const unsigned long long pm = __ballot(pass);
        if (COUNT && pm != 0ull) ++c.wave_pass;
        if (interior) {
            if (pm != 0ull) {
                const unsigned long long bit = 2ull << depth;
                reach = pass ? (reach | bit) : (reach & ~bit);
                i = i + 1;
                cur = n1;
            } else {
                i = cur.a;
                cur = n2;
            }
            continue;
        }
        if (pm != 0ull) {
            const int first = cur.b, cnt = pnode_leaf_count(cur);
#ifndef CRT_GROUP_MAX
#define CRT_GROUP_MAX 32
#endif
            if (FAST && cnt >= 4 && __popcll(pm) <= CRT_GROUP_MAX) {
                leaf_grouped<COUNT>(s, first, cnt, pm, pass, o, d, best_t, best, lim, c);
                i = i + 1;
                cur = n1;
                continue;
            }
            DTriGeo g = load_scalar(s.slots, first);
            uint32_t cw = load_scalar(s.slot_cull_bits, first >> 5);
            for (int k = 0; k < cnt; ++k) {
                const int slot = first + k;
                const int sn = k + 1 < cnt ? slot + 1 : slot;
                const DTriGeo gn = load_scalar(s.slots, sn);           /* next triangle in flight */
                const uint32_t cwn = load_scalar(s.slot_cull_bits, sn >> 5);
                const bool cull = ((cw >> (slot & 31)) & 1u) != 0u;
                float t;
                if (COUNT && pass) ++c.tris;
                if (COUNT) ++c.wave_tris;
                const bool plane = tri_plane(o, d, g, cull, t);
                const bool better = (best < 0) | (t < best_t) | ((t == best_t) & (slot < best));
                const bool pre = pass & plane & better;
                if (__ballot(pre) != 0ull) {
                    if (COUNT) ++c.wave_edges;
                    const bool hit = pre & tri_edges(o, d, g, t);
                    best_t = hit ? t : best_t;
                    best = hit ? slot : best;
                    if constexpr (ANY) {
                        lim = hit ? fminf(t, lim) : lim;
                        if (hit && !(t * t > r2)) reach = 0ull;   /* occluded: this lane is done */
                    } else {
                        lim = hit ? t : lim;
                    }
                }
                g = gn;
                cw = cwn;
            }
        }
        i = i + 1;
        cur = n1;
    }
    return best;
}

/* A wave's shadow rays towards one light through the BVH (option "shadows";
 * crt_bvh.h occluded_bvh for one ray): the wave walks the union of its lanes'
 * alive boxes in one preorder — wave-uniform node index, scalar node and
 * triangle loads, branches on ballots — each lane testing the triangles of
 * the leaves its own ray reaches, and a lane leaves at its first hit within
 * the light; then every such hit is proved at once (the reference reaches
 * that triangle: the proof on the reference tree).  The walk order (the lanes' majority octant) changes nothing but
 * the time: every alive box is visited until a lane is settled.  Returns the
 * lane's verdict: 1 occluded, 0 lit, -1 undecided (its hit failed the proof:
 * the caller's exact walk decides). */
template <bool COUNT>
__device__ int occluded_bvh_wave(const DeviceScene &s, bool active, Vec o, Vec d, float r2, LaneCounts &c) {
    bool live = active && !(isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z));
    int res = 0;
    int ptri = -1;      /* the lane's first hit within the light: triangle, t */
    float pt = 0.0f;
    const int na = __popcll(__ballot(live));
    if (na == 0) {
        if (COUNT && active) ++c.traversals;
        return 0;
    }
    int oct = 0;
    if (2 * __popcll(__ballot(live && d.x < 0.0f)) > na) oct |= 1;
    if (2 * __popcll(__ballot(live && d.y < 0.0f)) > na) oct |= 2;
    if (2 * __popcll(__ballot(live && d.z < 0.0f)) > na) oct |= 4;
    const int bn = s.bnode_count;
    const BNode *ord = bnode_order(s.bnodes, bn, uniform_i(oct));
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    const float lim = sqrtf(r2) * (1.0f + 0x1p-20f);
    int i = 0;
    BNode cur = load_scalar(ord, 0);
    while (i < bn) {
        if (__ballot(live) == 0ull) break;   /* every lane settled */
        /* both successors in flight before the test (every order ends with a zero record: i + 1 <= bn) */
        const BNode n1 = load_scalar(ord, i + 1);
        const BNode n2 = load_scalar(ord, cur.skip);
        const bool alive = live && bnode_alive(cur, pr, lim);
        if (COUNT) {
            ++c.wave_nodes;
            if (alive) ++c.nodes;
        }
        if (__ballot(alive) == 0ull) {
            i = cur.skip;
            cur = n2;
            continue;
        }
        const int cnt = cur.leaf & 15, first = cur.leaf >> 4;
        for (int k = 0; k < cnt; ++k) {
            const DTriGeo g = load_scalar(s.btri, first + k);
            const int32_t id = load_scalar(s.btri_id, first + k);
            const uint8_t cull = (uint8_t)((uint32_t)id >> 31);
            float t = 0.0f;
            if (COUNT) {
                ++c.wave_tris;
                if (alive && live) ++c.tris;
            }
            if (alive && live && tri_hit(o, d, g, &cull, t) && !(t * t > r2)) {
                ptri = id & 0x7fffffff;   /* settled: its proof runs after the walk, with the wave's other ones */
                pt = t;
                live = false;
            }
        }
        i = i + 1;
        cur = n1;
    }
    /* the proofs of every settled lane at once (one descent each, side by
     * side, instead of one whenever a lane settles) */
    if (ptri >= 0) {
        const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
        const Vec p = vadd(o, vscale(d, pt));
        WalkCounts wc = {0u, 0u};
        const int slot = CRT_PROOF_TOPO && s.ktopo
                             ? verify_topo<COUNT>(s.ktopo, s.nodes, s.slot_tri, ptri, o, d, rr, p, wc,
                                                  CRT_PROOF_TOPO2 ? s.ktopo2 : nullptr)
                             : verify_kd<COUNT>(s.nodes, s.slot_tri, ptri, o, d, rr, p, wc);
        if (COUNT) {
            c.nodes += wc.nodes;
            c.tris += wc.tris;
        }
        res = slot >= 0 ? 1 : -1;
    }
    if (COUNT && active && res >= 0) ++c.traversals;
    return res;
}

/* The wave's shadow rays towards light `light` over its light bins
 * (crt_bvh.h lbin_setup / lbin_test, the lists as lbin_first_hit walks
 * them), wave-coherent: the near list, then one cell at a time — the cell of
 * the first lane still looking, walked with scalar loads by the lanes whose
 * ray is in it (a tile's rays share few cells) until each has a hit or is
 * past its cut-off; then the proofs of every lane that found a hit, side by
 * side.  1 occluded, 0 lit, -1 not decided here (the BVH decides). */
template <bool COUNT>
__device__ int occluded_lbins_wave(const DeviceScene &s, int light, bool active, Vec o, Vec d, float r2,
                                   LaneCounts &c) {
    const DLightBin P = load_scalar(s.lbin_par, light);
    const float lim = sqrtf(r2) * (1.0f + 0x1p-20f);
    LbinRay lr;
    lr.ok = false;
    lr.cell = -1;
    lr.cut_near = lr.cut_far = 0.0;
    if (active) lr = lbin_setup(P, s.lbin_n, s.prune_origin_max, o, d, lim);
    int tri = -1;
    float th = 0.0f;
    bool look = lr.ok;      /* near list */
    bool far = lr.ok && lr.cell >= 0;
    bool capped = false;
    const int base = P.base;
    for (int phase = 0; phase < 2; ++phase) {
        do {
            int beg, end;
            double cut;
            int cell = -1;
            if (phase == 0) {
                beg = load_scalar(s.lbin_off, base);
                end = load_scalar(s.lbin_off, base + 1);
                cut = lr.cut_near;
            } else {
                const uint64_t m = __ballot(far);
                if (m == 0ull) break;
                cell = uniform_i(__shfl(lr.cell, (int)__builtin_ctzll(m)));
                look = far && lr.cell == cell;
                beg = load_scalar(s.lbin_off, base + 1 + cell);
                end = load_scalar(s.lbin_off, base + 2 + cell);
                cut = lr.cut_far;
            }
            LightCand nx = load_scalar(s.lbins, beg);   /* (a zero record past the last list) */
            const int end0 = end;
            if (phase == 1 && end - beg > CRT_LBINS_CAP) end = beg + CRT_LBINS_CAP;
            for (int k = beg; k < end; ++k) {
                if (__ballot(look) == 0ull) break;
                const LightCand cc = nx;
                nx = load_scalar(s.lbins, k + 1);
                if (COUNT) ++c.wave_tris;
                if (look) {
                    float t;
                    if ((double)cc.dmin * (double)cc.dmin > cut) {
                        look = false;
                    } else {
                        if (COUNT) ++c.tris;
                        if (lbin_test(cc, o, d, r2, t)) {
                            tri = cc.id & 0x7fffffff;
                            th = t;
                            look = false;
                            far = false;
                        }
                    }
                }
            }
            if (phase == 1 && lr.cell == cell) {
                far = false;
                if (look && end < end0) capped = true;   /* still looking at the cap: undecided */
            }
        } while (phase == 1);
        look = false;
    }
    int res = active && (!lr.ok || capped) ? -1 : 0;
    if (tri >= 0) {
        WalkCounts wc = {0u, 0u};
        const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
        const Vec p = vadd(o, vscale(d, th));
        const int slot = CRT_PROOF_TOPO && s.ktopo
                             ? verify_topo<COUNT>(s.ktopo, s.nodes, s.slot_tri, tri, o, d, rr, p, wc,
                                                  CRT_PROOF_TOPO2 ? s.ktopo2 : nullptr)
                             : verify_kd<COUNT>(s.nodes, s.slot_tri, tri, o, d, rr, p, wc);
        res = slot >= 0 ? 1 : -1;
        if (COUNT) {
            c.nodes += wc.nodes;
            c.tris += wc.tris;
        }
    }
    if (COUNT && active && res >= 0) ++c.traversals;
    return res;
}

/* FAST (walk 12, picked by the host): every camera ray of the frame is in the
 * hoisted-division window (camera_rays_fast), so the out-of-line exact box
 * path is not compiled in — 77 instead of 82 VGPRs, 6 waves/SIMD. */
template <bool COUNT, bool FAST>
__device__ int trace_packet_pruned(const DeviceScene &s, bool active, Vec o, Vec d, float &best_t, LaneCounts &c) {
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    if (COUNT && active) ++c.traversals;
    const int best = trace_packet_pruned_t<COUNT, FAST>(s, active, o, d, rr, best_t, c);
    if (COUNT && best >= 0) ++c.hits;
    return best;
}

/* ---------------------------------------------------------------------- */
/* Window walk (TRAV 13, small tiles of ≤ 16 camera rays)                    */
/* ---------------------------------------------------------------------- */
/* The packet walk pays one dependent node load and ~90 instructions per node
 * step whatever the number of rays; for the few heavy tiles that set a C2
 * frame's length (2x2 / 4x4 splits of the dragon's silhouette, ~200 us waves
 * of one-node steps) that is a latency chain.  Here a wave holds R rays (4 or
 * 16) and K = 64 / R consecutive nodes of the walk's preorder at once: lane
 * (slot s, ray r) loads node i + s and evaluates its hull and box tests for
 * ray r, so a window of K nodes costs one round of loads.  The reach masks
 * then advance over the window exactly as the packet walk would visit those
 * nodes in order (bit depth+1 of an interior node := this ray entered it; a
 * node is entered iff its reach bit is set and its box passed), every lane
 * replaying its ray's sequence; evaluating a node no ray reaches is wasted
 * work, never a change of result.  Hull tests use the best t known at the
 * window's start (only ever larger than the packet walk's, so pruning stays
 * conservative).  Each entered leaf's triangles are tested by the lane that
 * entered it, and a ray's candidates are merged over its K lanes by the key
 * (t, slot) — the reference's first-found rule in any order (key_better).
 * The next window starts after the last one, or past the subtree of a window
 * node no ray entered. */
__device__ __forceinline__ int wave_max_i(int v) {
    for (int off = 32; off > 0; off >>= 1) {
        const int o2 = __shfl_xor(v, off);
        v = v > o2 ? v : o2;
    }
    return v;
}

template <bool COUNT, int R>
__device__ int trace_window(const DeviceScene &s, int r, int sl, bool active, Vec o, Vec d, float &best_t,
                            LaneCounts &c) {
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    const bool lead = sl == 0;                       /* one lane per ray for votes and counters */
    if (COUNT && active && lead) ++c.traversals;
    int best = -1;
    best_t = 0.0f;
    float lim = INFINITY;
    const int n = s.node_count;
    constexpr int K = 64 / R;
    /* reach state per depth as ray masks: lane dd of `vreach` holds the R-bit
     * mask of the rays that entered the window's last node at depth dd - 1
     * (bit r: ray r), i.e. the packet walk's reach bit dd of every ray */
    const uint32_t amask = (uint32_t)__ballot(active && lead);   /* lanes 0..R-1 are (slot 0, ray r) */
    uint32_t vreach = __lane_id() == 0 ? amask : 0u;
    const int na = __popcll(__ballot(active && lead));
    int oct = 0;
    if (2 * __popcll(__ballot(active && lead && d.x < 0.0f)) > na) oct |= 1;
    if (2 * __popcll(__ballot(active && lead && d.y < 0.0f)) > na) oct |= 2;
    if (2 * __popcll(__ballot(active && lead && d.z < 0.0f)) > na) oct |= 4;
    const PNode *nodes = pnode_order(s.pnodes, n, uniform_i(oct));
    constexpr unsigned long long rmask = (R >= 64) ? ~0ull : ((1ull << R) - 1ull);
    int i = 0;
    PNode nd = load_global(nodes, sl < n ? sl : n - 1);
    while (i < n) {
        const int j = i + sl;
        const bool valid = j < n;
        const bool interior = nd.count == 0;
        const bool alive = valid & active & hull_alive(nd, pr, lim);
        const bool pass = alive & box_hit_fast(o, d, rr, cell_of(nd));
        const unsigned long long P = __ballot(pass);
        /* replay the packet walk's reach update over the window, in order, on
         * wave-uniform ray masks: node a's rays in = reach mask of its depth;
         * an interior node sets the mask of depth + 1 to the rays that entered
         * it (in & pass) */
        /* the K window nodes in order, unrolled and branch-free: a node past
         * the array end (meta 0) reads depth 0 and writes nothing; its IN
         * bits are never used (the node is not valid) */
        const int meta = valid ? (nd.depth | (interior ? 256 : 0)) : 0;
        unsigned long long IN = 0ull;   /* bit a * R + r: ray r reaches window node a */
        int ms[K];
#pragma unroll
        for (int a = 0; a < K; ++a) ms[a] = __builtin_amdgcn_readlane(meta, a * R);
#pragma unroll
        for (int a = 0; a < K; ++a) {
            const int dd = ms[a] & 255;
            const uint32_t in_m = (uint32_t)__builtin_amdgcn_readlane((int)vreach, dd);
            const uint32_t e_m = in_m & (uint32_t)(P >> (a * R)) & (uint32_t)rmask;
            vreach = (((ms[a] & 256) != 0) & ((int)__lane_id() == dd + 1)) ? e_m : vreach;
            IN |= (unsigned long long)in_m << (a * R);
        }
        const bool my_in = ((IN >> __lane_id()) & 1ull) != 0ull;
        const int kk = n - i < K ? n - i : K;   /* valid nodes of the window */
        if (COUNT) {
            if (my_in & alive) ++c.nodes;
            c.wave_nodes += (uint32_t)kk;     /* node records of the window */
            ++c.win_steps;
            if (sl < kk && r < __popcll(__ballot(active && lead))) ++c.win_slots;
            if (my_in & alive) ++c.win_reached;
        }
        const bool enter = my_in & pass;
        const unsigned long long E = __ballot(enter);
        /* skip past the subtree of a window node no ray entered: the furthest
         * skip index of the dead nodes, read from one lane per dead node */
        const bool dead = valid & interior & (((E >> (sl * R)) & rmask) == 0ull);
        unsigned long long D = __ballot(dead & (r == 0));
        int skip_to = 0;
        while (D != 0ull) {
            const int l = __builtin_ctzll(D);
            D &= D - 1ull;
            const int v = __builtin_amdgcn_readlane(nd.a, l);
            skip_to = v > skip_to ? v : skip_to;
        }
        const int next = uniform_i(i + K > skip_to ? i + K : skip_to);
        /* triangles of the entered leaves, one leaf at a time over the whole
         * wave: lane (sl, r) tests triangles sl, sl + K, ... of the leaf for
         * its ray r if r entered it, so a leaf costs ceil(count / K) rounds
         * (its triangles load as K consecutive records); then a per-ray merge
         * of the candidates over the ray's K lanes by the key (t, slot). */
        const bool leaf = enter & !interior;
        if (__ballot(leaf) != 0ull) {
            float lt = best_t;
            int ls = best;
            unsigned long long Lm = __ballot(leaf);
            while (Lm != 0ull) {
                const int l0 = __builtin_ctzll(Lm);
                const int s0 = l0 / R;
                const unsigned long long sm = Lm & (rmask << (s0 * R));   /* the rays that entered leaf s0 */
                Lm &= ~sm;
                const int first = __builtin_amdgcn_readlane(nd.b, l0), cnt = __builtin_amdgcn_readlane(nd.count, l0);
                if (COUNT) {
                    c.wave_tris += (uint32_t)((cnt + K - 1) / K);
                    c.win_rounds += (uint32_t)((cnt + K - 1) / K);
                }
                if (((sm >> (s0 * R + r)) & 1ull) != 0ull) {
                    for (int k = sl; k < cnt; k += K) {
                        const int slot = first + k;
                        const DTriGeo g = load_global(s.slots, slot);
                        const uint8_t cl = load_global(s.slot_cull, slot);
                        float t;
                        if (COUNT) ++c.tris;
                        if (tri_plane(o, d, g, cl != 0, t) && key_better(t, slot, lt, ls) && tri_edges(o, d, g, t)) {
                            lt = t;
                            ls = slot;
                        }
                    }
                }
            }
            HitKey key = hit_key(lt, ls);   /* merge over the ray's K lanes */
            hit_key_allmin(key, R);
            hit_key_get(key, lt, ls);
            best_t = lt;
            best = ls;
            lim = best >= 0 ? best_t : INFINITY;
        }
        {
            nd = load_global(nodes, next + sl < n ? next + sl : n - 1);
        }
        i = next;
    }
    if (COUNT && best >= 0 && lead) ++c.hits;
    return best;
}

/* Per-lane pruned walk (crt_device.h walk_pruned) over the lane's own octant
 * order: crt_hip_trace_batch's pruned walk (arbitrary, unrelated rays). */
template <bool COUNT>
__device__ __forceinline__ int trace_lane_pruned(const DeviceScene &s, bool active, Vec o, Vec d, float &best_t,
                                                 LaneCounts &c) {
    best_t = 0.0f;
    if (!active) return -1;
    if (COUNT) ++c.traversals;
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    const int n = s.node_count;
    WalkCounts wc = {0u, 0u};
    const int best = walk_pruned<COUNT>(pnode_order(s.pnodes, n, ray_octant(d)), n, s.slots, s.slot_cull, o, d,
                                        rr, pr, best_t, wc);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (best >= 0) ++c.hits;
    }
    return best;
}

/* Per-lane BVH walk with its proof on the reference's tree (crt_bvh.h):
 * scattered rays (GI bounces, reflections, refractions) of the frame-stack,
 * refill and wavefront kernels when the scene has its BVH. */
template <bool COUNT, int PF = CRT_BVH_PREFETCH>
__device__ __forceinline__ int trace_lane_bvh(const DeviceScene &s, bool active, Vec o, Vec d, float &best_t,
                                              LaneCounts &c) {
    best_t = 0.0f;
    if (!active) return -1;
    if (COUNT) ++c.traversals;
    WalkCounts wc = {0u, 0u};
    const int best = trace_bvh_exact<COUNT, PF>(s.bnodes, s.bnode_count, s.btri, s.btri_id, s.nodes, s.pnodes,
                                            s.node_count, s.slots, s.slot_cull, s.slot_tri, s.ktopo, s.prune_origin_max,
                                            s.planes_ok != 0, o, d, best_t, wc, nullptr, s.ktopo2);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (best >= 0) ++c.hits;
    }
    return best;
}

/* All-reduce over groups of K consecutive lanes (K = 16: one DPP row, row
 * rotations 1/2/4/8; K = 4: one quad, quad permutations), every lane active. */
template <int K>
__device__ __forceinline__ int group_dpp(int v, int step) {
    static_assert(K == 4 || K == 16, "group of 4 or 16 lanes");
    if constexpr (K == 16) {
        switch (step) {
        case 0: return __builtin_amdgcn_update_dpp(v, v, 0x121, 0xf, 0xf, false);
        case 1: return __builtin_amdgcn_update_dpp(v, v, 0x122, 0xf, 0xf, false);
        case 2: return __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false);
        default: return __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false);
        }
    } else {
        return step == 0 ? __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xf, 0xf, false)    /* quad_perm [1,0,3,2] */
                         : __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xf, 0xf, false);   /* quad_perm [2,3,0,1] */
    }
}
template <int K> constexpr int kGroupSteps = K == 16 ? 4 : 2;
template <int K> __device__ __forceinline__ unsigned group_or(unsigned v) {
#pragma unroll
    for (int q = 0; q < kGroupSteps<K>; ++q) v |= (unsigned)group_dpp<K>((int)v, q);
    return v;
}
template <int K> __device__ __forceinline__ int group_max(int v) {
#pragma unroll
    for (int q = 0; q < kGroupSteps<K>; ++q) v = max(v, group_dpp<K>(v, q));
    return v;
}
template <int K> __device__ __forceinline__ int group_sum(int v) {
#pragma unroll
    for (int q = 0; q < kGroupSteps<K>; ++q) v += group_dpp<K>(v, q);
    return v;
}
template <int K> __device__ __forceinline__ float group_min(float v) {
#pragma unroll
    for (int q = 0; q < kGroupSteps<K>; ++q) v = fminf(v, __int_as_float(group_dpp<K>(__float_as_int(v), q)));
    return v;
}

/* BVH window walk for the split tiles (<= 16 rays) of camera frames: the
 * ray of lanes [K r, K r + K) is walked by all K of them (crt_bvh.h walk_bvh,
 * same order, same boxes, same triangle test).  Each step the K lanes load
 * the K nodes of the order from the ray's cursor on and test them at once; a
 * dead node kills the window lanes of its subtree (its preorder range up to
 * skip), a visited live leaf's lane tests its triangles, the group merges the
 * candidates (min t; two at the minimum = tie) and the cursor moves past the
 * window and every dead subtree that reaches beyond it.  The boxes are tested
 * with the bound from before the step, a looser bound than walk_bvh's, so the
 * triangles tested include every one walk_bvh tests at t <= its final bound:
 * the same closest triangle, t bits and tie flag.  One step is one dependent
 * node load for K nodes of the chain (the heavy rays' walks are ~100 nodes).
 * Returns the group's triangle id (-1: none), row-uniform. */
template <bool COUNT, int K>
__device__ int walk_bvh_window(const BNode *nodes, int n, const DTriGeo *geo, const int32_t *tid, int sl, bool act,
                               Vec o, Vec d, const PruneRay &pr, float &best_t, bool &tie, WalkCounts &c) {
    int best = -1, i = act ? 0 : n;
    float lim = INFINITY, bt = 0.0f;
    bool tb = false;
    while (__ballot(i < n) != 0ull) {
        const int j = i + sl;
        const bool in = i < n && j < n;
        BNode nd = {};
        if (in) nd = CRT_LDG(nodes, j);
        const bool alive = in && bnode_alive(nd, pr, lim);
        unsigned kill = 0u;
        int jump = 0;
        if (in && !alive) {   /* window lanes sl+1 .. e-1 lie in this dead subtree */
            const int e = min(nd.skip - i, K);
            kill = e > sl + 1 ? ((1u << e) - 1u) & ~((2u << sl) - 1u) : 0u;
            jump = nd.skip;
        }
        kill = group_or<K>(kill);
        jump = group_max<K>(jump);
        const bool visit = alive && !((kill >> sl) & 1u);
        float lt = INFINITY;
        int lid = -1;
        bool ltie = false;
        if (visit && nd.leaf != 0) {
            if (COUNT) ++c.nodes;
            const int cnt = nd.leaf & 15, first = nd.leaf >> 4;
            for (int k = 0; k < cnt; ++k) {
                const DTriGeo g = CRT_LDG(geo, first + k);
                const int32_t id = CRT_LDG(tid, first + k);
                const uint8_t cull = (uint8_t)((uint32_t)id >> 31);
                float t;
                if (COUNT) ++c.tris;
                if (tri_hit(o, d, g, &cull, t)) {
                    if (lid < 0 || t < lt) {
                        lt = t;
                        lid = id & 0x7fffffff;
                        ltie = false;
                    } else if (t == lt) {
                        ltie = true;
                    }
                }
            }
        } else if (COUNT && visit) {
            ++c.nodes;
        }
        const float m = group_min<K>(lt);
        const bool eq = lid >= 0 && lt == m;
        const int neq = group_sum<K>(eq ? (ltie ? 2 : 1) : 0);
        const int wid = group_max<K>(eq ? lid : -1);
        if (neq > 0) {
            if (best < 0 || m < bt) {
                best = wid;
                bt = m;
                tb = neq > 1;
                lim = m;
            } else if (m == bt) {
                tb = true;
            }
        }
        if (i < n) i = max(i + K, jump);
    }
    best_t = bt;
    tie = tb;
    return best;
}

/* trace_bvh_exact (crt_bvh.h) with the walk done by a group of K lanes per
 * ray (walk_bvh_window); the proof and the rare fallback run on every lane of
 * the group with the same inputs.  act: the group has a ray. */
template <bool COUNT, int K>
__device__ int trace_bvh_window(const DeviceScene &s, int sl, bool act, Vec o, Vec d, float &best_t, LaneCounts &c) {
    best_t = 0.0f;
    const bool nan_ray = isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z);
    const bool walk = act && !nan_ray;
    if (COUNT && act && sl == 0) ++c.traversals;
    const int oct = ray_octant(d);
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    WalkCounts wc = {0u, 0u};
    bool tie = false;
    float t = 0.0f;
    const int tri = walk_bvh_window<COUNT, K>(bnode_order(s.bnodes, s.bnode_count, oct), s.bnode_count, s.btri,
                                              s.btri_id, sl, walk, o, d, pr, t, tie, wc);
    int slot = -1;
    if (tri >= 0) {
        const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
        WalkCounts pc = {0u, 0u};
        if (!tie) {
            const Vec p = vadd(o, vscale(d, t));
            slot = CRT_PROOF_TOPO && s.ktopo ? verify_topo<COUNT>(s.ktopo, s.nodes, s.slot_tri, tri, o, d, rr, p, pc,
                                                                 CRT_PROOF_TOPO2 ? s.ktopo2 : nullptr)
                                             : verify_kd<COUNT>(s.nodes, s.slot_tri, tri, o, d, rr, p, pc);
            if (slot >= 0) best_t = t;
        }
        if (slot < 0)
            slot = walk_pruned<COUNT>(pnode_order(s.pnodes, s.node_count, oct), s.node_count, s.slots, s.slot_cull, o, d,
                                      rr, pr, best_t, pc);
        if (COUNT && sl == 0) {
            wc.nodes += pc.nodes;
            wc.tris += pc.tris;
        }
    }
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (slot >= 0 && sl == 0) ++c.hits;
    }
    return slot;
}

/* Camera rays of one camera-bins cell (crt_bvh.h walk_bins / trace_bins_exact)
 * with the whole wave on the cell's candidate list.  The list is staged
 * through LDS kBinChunk records at a time (one coalesced global load per
 * lane: one memory latency per chunk).  Each lane first gathers, from the
 * chunk's pixel masks (read by broadcast), the bits of the records that
 * cover its pixel, then walks only those, in list order, at its own pace —
 * so a chunk costs the wave as many rounds as its busiest lane has records,
 * not as many as the chunk holds.  Per lane this is walk_bins exactly: the
 * covered records in order, the same dmin exit (the list is sorted by dmin,
 * so an uncovered record past best t only means a covered one later is past
 * it too) and the same end when no later record covers the pixel.  Then the
 * proof / fallback per lane (resolve_closest).  stage: this wave's kBinChunk
 * LDS records; bit: the lane's pixel in the cell (8 y + x); act: the lane
 * has a pixel.  Returns the reference's slot (-1: miss). */
constexpr int kBinChunk = 32;
#ifndef CRT_BINS_LANE_ILP
#define CRT_BINS_LANE_ILP 1   /* records a lane tests side by side per round (A/B builds: 2) */
#endif

template <bool COUNT>
__device__ int trace_bins_wave(const DeviceScene &s, CamCand *stage, int beg, int end, int bit, bool act, Vec o,
                               Vec d, float &best_t, LaneCounts &c, unsigned long long *phase = nullptr) {
    best_t = 0.0f;
    const bool nan_ray = isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z);
    if (COUNT && act) ++c.traversals;
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    const int lane = (int)__lane_id();
    int best = -1;
    float bt = 0.0f, lim = INFINITY;
    bool tie = false, live = act && !nan_ray;
    WalkCounts wc = {0u, 0u};
    for (int k0 = beg; k0 < end; k0 += kBinChunk) {
        if (__ballot(live) == 0ull) break;
        const int n = min(kBinChunk, end - k0);
        if (lane < n) stage[lane] = load_global(s.bins, k0 + lane);
        __builtin_amdgcn_wave_barrier();
        live = live && ((stage[0].rest >> bit) & 1ull) != 0ull;   /* a later record covers the pixel */
        uint32_t w = 0u;
        if (__ballot(live) != 0ull) {
            for (int j = 0; j < n; ++j) w |= (uint32_t)((stage[j].mask >> bit) & 1ull) << j;
        }
        if (!live) w = 0u;
#if CRT_BINS_LANE_ILP > 1
        /* two of the lane's records per round, both tested against the
         * round's lim and merged in order (a record dead for the updated lim
         * can only hit past best t: no change) */
        while (__ballot(w != 0u) != 0ull) {
            if (w != 0u) {
                const int j1 = __builtin_ctz(w);
                w &= w - 1u;
                const bool two = w != 0u;
                const int j2 = two ? __builtin_ctz(w) : j1;
                if (two) w &= w - 1u;
                const CamCand c1 = stage[j1], c2 = stage[j2];
                if (best >= 0 && c1.dmin > bt) {
                    live = false;
                    w = 0u;
                } else {
                    float t1, t2;
                    const bool h1 = cand_hit_bf(c1, o, d, pr, lim, t1);
                    const bool h2 = two && cand_hit_bf(c2, o, d, pr, lim, t2);
                    if (COUNT) ++wc.nodes;
                    if (h1) {
                        if (best < 0 || t1 < bt) {
                            bt = t1;
                            best = c1.id & 0x7fffffff;
                            tie = false;
                            lim = t1;
                        } else if (t1 == bt) {
                            tie = true;
                        }
                    }
                    if (two) {
                        if (best >= 0 && c2.dmin > bt) {
                            live = false;
                            w = 0u;
                        } else {
                            if (COUNT) ++wc.nodes;
                            if (h2) {
                                if (best < 0 || t2 < bt) {
                                    bt = t2;
                                    best = c2.id & 0x7fffffff;
                                    tie = false;
                                    lim = t2;
                                } else if (t2 == bt) {
                                    tie = true;
                                }
                            }
                        }
                    }
                }
            }
        }
#else
        while (__ballot(w != 0u) != 0ull) {
            if (w != 0u) {
                const int j = __builtin_ctz(w);
                w &= w - 1u;
                const CamCand cc = stage[j];
                if (best >= 0 && cc.dmin > bt) {   /* sorted by dmin: nothing later can hit at t <= best t */
                    live = false;
                    w = 0u;
                } else {
                    if (COUNT) ++wc.nodes;
                    const bool tested = cand_test(cc, o, d, pr, best, bt, tie, lim);
                    if (COUNT && tested) ++wc.tris;
                }
            }
        }
#endif
        __builtin_amdgcn_wave_barrier();
    }
#ifdef CRT_BINS_PHASE
    if (phase && lane == 0) *phase = __builtin_amdgcn_s_memrealtime();   /* diagnostic builds: loop end */
#else
    (void)phase;
#endif
    int slot = -1;
    if (act && !nan_ray)
        slot = resolve_closest<COUNT>(s.nodes, s.pnodes, s.node_count, s.slots, s.slot_cull, s.slot_tri, s.ktopo,
                                      s.planes_ok != 0, o, d, pr, best, bt, tie, best_t, wc, nullptr, s.ktopo2);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (slot >= 0) ++c.hits;
    }
    return slot;
}

/* trace_bins_wave with K lanes per pixel (lane = K p + sl; K = 4: a tile of
 * at most 4x4 pixels, K = 2: at most 8x4): lane sl walks the pixel's covering
 * records at chunk positions j = sl (mod K), and the K share their lim (the
 * smallest best t among them) after every round.  Merged at the end: the
 * smallest t, the record of the lowest lane holding it, tie when two lanes
 * hold it or one of them saw two hits there.  That is walk_bins' (best, t,
 * tie): every record hitting at the final t is tested by its lane (its dmin
 * and hull pass any lim >= that t), and a lane's own best may lag the shared
 * lim but never lowers the minimum wrongly.  Lane sl = 0 resolves
 * (resolve_closest).  act: the lane's pixel exists (same on its K lanes). */
template <bool COUNT, int K>
__device__ int trace_bins_lanes(const DeviceScene &s, CamCand *stage, int beg, int end, int bit, int sl, bool act, Vec o,
                                Vec d, float &best_t, LaneCounts &c) {
    static_assert(K == 2 || K == 4, "two or four lanes per pixel");
    best_t = 0.0f;
    const bool nan_ray = isnan(o.x) || isnan(o.y) || isnan(o.z) || isnan(d.x) || isnan(d.y) || isnan(d.z);
    if (COUNT && act && sl == 0) ++c.traversals;
    const PruneRay pr = make_prune_ray(o, d, s.prune_origin_max);
    const int lane = (int)__lane_id();
    int best = -1;
    float bt = 0.0f, lim = INFINITY;
    bool tie = false, live = act && !nan_ray;
    WalkCounts wc = {0u, 0u};
    for (int k0 = beg; k0 < end; k0 += kBinChunk) {
        if (__ballot(live) == 0ull) break;
        const int n = min(kBinChunk, end - k0);
        if (lane < n) stage[lane] = load_global(s.bins, k0 + lane);
        __builtin_amdgcn_wave_barrier();
        live = live && ((stage[0].rest >> bit) & 1ull) != 0ull;   /* a later record covers the pixel */
        uint32_t w = 0u;
        if (live) {
            for (int j = sl; j < n; j += K) w |= (uint32_t)((stage[j].mask >> bit) & 1ull) << j;
        }
        while (__ballot(w != 0u) != 0ull) {
            if (w != 0u) {
                const int j = __builtin_ctz(w);
                w &= w - 1u;
                const CamCand cc = stage[j];
                if (cc.dmin > lim) {   /* sorted by dmin: nothing later hits at t <= the pixel's best t */
                    live = false;
                    w = 0u;
                } else {
                    if (COUNT) ++wc.nodes;
                    if (cand_alive(cc, pr, lim)) {
                        if (COUNT) ++wc.tris;
                        const uint8_t cull = (uint8_t)((uint32_t)cc.id >> 31);
                        float t;
                        if (tri_hit(o, d, cc.g, &cull, t)) {
                            if (best < 0 || t < bt) {
                                bt = t;
                                best = cc.id & 0x7fffffff;
                                tie = false;
                                lim = fminf(lim, t);
                            } else if (t == bt) {
                                tie = true;
                            }
                        }
                    }
                }
            }
            lim = fminf(lim, __shfl_xor(lim, 1));
            if (K == 4) lim = fminf(lim, __shfl_xor(lim, 2));
        }
        __builtin_amdgcn_wave_barrier();
    }
    /* merge the pixel's K lanes */
    const float mine = best >= 0 ? bt : INFINITY;
    float g = fminf(mine, __shfl_xor(mine, 1));
    if (K == 4) g = fminf(g, __shfl_xor(g, 2));
    const bool at = best >= 0 && bt == g;
    const int q = lane & ~(K - 1);
    const uint32_t holders = (uint32_t)(__ballot(at) >> q) & ((1u << K) - 1u);
    const uint32_t ties = (uint32_t)(__ballot(at && tie) >> q) & ((1u << K) - 1u);
    const int src = q + (holders ? __builtin_ctz(holders) : 0);
    const int gbest = __shfl(best, src);
    int slot = -1;
    if (act && !nan_ray && sl == 0 && holders != 0u)
        slot = resolve_closest<COUNT>(s.nodes, s.pnodes, s.node_count, s.slots, s.slot_cull, s.slot_tri, s.ktopo,
                                      s.planes_ok != 0, o, d, pr, gbest, g, __builtin_popcount(holders) > 1 || ties != 0u,
                                      best_t, wc, nullptr, s.ktopo2);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (slot >= 0) ++c.hits;
    }
    return slot;
}

/* Walks (TRAV), all bit-identical in result:
 *   7  packet walk in the reference's node order (work counters = the reference's)
 *   8  pruned packet walk (exact t-pruning), any camera ray
 *   12 8 for frames whose camera rays are all in the hoisted-division window
 *   13 12 + window walk for the plan's split tiles (k_render_tiles)
 *   4  cooperative walk in the reference's node order (scattered rays)
 *   10 pruned cooperative walk
 *   14 per-lane BVH walk + proof on the reference's tree (scattered rays, crt_bvh.h)
 *   15 camera bins (trace_bins_wave; k_render_tiles only, 14 elsewhere)
 * PF: the BVH walk loads both successors ahead (crt_bvh.h walk_bvh). */
template <int TRAV>
constexpr bool kIsCoop = TRAV == 4 || TRAV == 10;

template <int TRAV, bool COUNT, int PF = CRT_BVH_PREFETCH>
__device__ __forceinline__ int trace(const DeviceScene &s, CoopLds *L, bool active, Vec o, Vec d, float &best_t,
                                     LaneCounts &c) {
    static_assert(TRAV == 4 || TRAV == 7 || TRAV == 8 || TRAV == 10 || TRAV == 12 || TRAV == 13 || TRAV == 14,
                  "no such walk");
    if constexpr (TRAV == 8) return trace_packet_pruned<COUNT, false>(s, active, o, d, best_t, c);
    else if constexpr (TRAV == 12 || TRAV == 13) return trace_packet_pruned<COUNT, true>(s, active, o, d, best_t, c);
    else if constexpr (TRAV == 4) return trace_coop<COUNT, false>(s, *L, active, o, d, best_t, c);
    else if constexpr (TRAV == 10) return trace_coop<COUNT, true>(s, *L, active, o, d, best_t, c);
    else if constexpr (TRAV == 14) return trace_lane_bvh<COUNT, PF>(s, active, o, d, best_t, c);
    else return trace_packet<COUNT>(s, active, o, d, best_t, c);
}

}  // namespace crt_amd
