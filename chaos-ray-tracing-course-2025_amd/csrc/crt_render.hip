/*
 * crt_render.hip — gfx950 kernels + the C-ABI device layer (include/crt_hip.h).
 *
 * Replaces crt::render_image (src/core/crt_renderer.cpp:157-199) and the
 * per-ray hot path beneath it (crt_intersection.cpp:14-136).
 *
 * Kernel structure (one launch per frame):
 *   - one lane = one pixel; one wave = one 8x8 pixel tile (ray coherence inside
 *     the wave), 4 waves per 256-thread workgroup; the tile list covers the
 *     whole frame or one shard's buckets (multi-GPU);
 *   - primary ray generated in-kernel (Camera::generate_ray, crt_camera.cpp:7-35);
 *   - stackless tree walk over the traversal-ordered node array (crt_layout.h):
 *     exactly the reference's node visit sequence, no per-lane stack;
 *   - leaf triangles are contiguous 48-B records (no index indirection);
 *   - only the winning triangle's Intersection record is built (bary, smooth
 *     normal, uv), with the reference's arithmetic, after the walk;
 *   - shading (crt_renderer.cpp:46-145) runs in the same kernel: recursion
 *     becomes a per-lane LIFO of continuation frames, so the PCG draws happen in
 *     the reference's depth-first order and rays never leave the GPU.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crt_bvh.h"
#include "crt_device.h"
#include "crt_host.h"
#include "crt_tree_build.h"

namespace crt_amd {

constexpr float kPi = 3.14159265358979323846f;   /* std::numbers::pi_v<float> */

struct alignas(16) Tile {
    int32_t x, y, w, h;        /* pixel rectangle, w,h <= 8 */
    int64_t out_base;          /* output pixel index of (x, y) */
    int32_t out_stride;        /* output pixels per row */
    int32_t prio;              /* 1: one of the frame's heaviest waves — raised issue priority */
};

struct alignas(16) UnpackBucket {
    int32_t x, y, w, h;
    int64_t src;               /* float offset of the bucket inside the gathered buffer */
    int64_t pad;
};

enum FrameKind : int32_t { kDiffuseGI = 0, kReflect = 1, kRefractA = 2, kRefractB = 3 };

/* A pending shade_ray activation (crt_renderer.cpp:46-145) waiting for a child. */
struct Frame {
    int32_t kind, depth, i, has_refr;
    Vec acc;    /* diffuse: GI sum | reflect: albedo | refract: reflection colour */
    Vec p, n;   /* diffuse: hit point and shading normal                         */
    Vec a, b;   /* diffuse: right, forward basis | refract: refraction ray o, d   */
    Vec alb;    /* diffuse: albedo sample | refract: .x = fresnel                */
};

/* global (address space 1) load: a global_load instead of a flat one, whose
 * completion is tracked by vmcnt alone (flat loads also count in lgkmcnt, so
 * every wait on them drains the LDS queue too) */
template <class T>
__device__ __forceinline__ T load_global(const T *p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    using GT = const __attribute__((address_space(1))) T;
    return ((GT *)p)[i];
#else
    return p[i];
#endif
}


struct LaneCounts {
    uint32_t traversals, nodes, tris, hits;
    /* wave-uniform steps of the packet walks (kept by every lane, added once per wave) */
    uint32_t wave_nodes, wave_tris, wave_edges;
    uint32_t wave_box, wave_pass;   /* packet walks: node steps with a box test run / with a lane passing */
    uint32_t win_steps, win_slots, win_reached, win_rounds;   /* window walk (crt_wave_counts) */
};

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
__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

/* Scene records are read-only for the whole launch: reading them through the
 * constant address space lets a wave-uniform index become an s_load into SGPRs. */
template <class T>
__device__ __forceinline__ T load_scalar(const T *p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    using CT = const __attribute__((address_space(4))) T;
    return ((CT *)p)[i];
#else
    return p[i];
#endif
}

/* Same, at a 32-bit byte offset from a wave-uniform base (SMEM base + offset
 * addressing: no 64-bit address arithmetic per load). */
template <class T>
__device__ __forceinline__ T load_scalar_at(const char *base, uint32_t byte_off) {
#if defined(__HIP_DEVICE_COMPILE__)
    using CT = const __attribute__((address_space(4))) T;
    return *(CT *)((const __attribute__((address_space(4))) char *)base + byte_off);
#else
    return *(const T *)(base + byte_off);
#endif
}

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
            vreach = ((ms[a] & 256) != 0) & ((int)__lane_id() == dd + 1) ? e_m : vreach;
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
template <bool COUNT>
__device__ __forceinline__ int trace_lane_bvh(const DeviceScene &s, bool active, Vec o, Vec d, float &best_t,
                                              LaneCounts &c) {
    best_t = 0.0f;
    if (!active) return -1;
    if (COUNT) ++c.traversals;
    WalkCounts wc = {0u, 0u};
    const int best = trace_bvh_exact<COUNT>(s.bnodes, s.bnode_count, s.btri, s.btri_id, s.nodes, s.pnodes,
                                            s.node_count, s.slots, s.slot_cull, s.slot_tri, s.prune_origin_max,
                                            s.planes_ok != 0, o, d, best_t, wc);
    if (COUNT) {
        c.nodes += wc.nodes;
        c.tris += wc.tris;
        if (best >= 0) ++c.hits;
    }
    return best;
}

/* Walks (TRAV), all bit-identical in result:
 *   7  packet walk in the reference's node order (work counters = the reference's)
 *   8  pruned packet walk (exact t-pruning), any camera ray
 *   12 8 for frames whose camera rays are all in the hoisted-division window
 *   13 12 + window walk for the plan's split tiles (k_render_tiles)
 *   4  cooperative walk in the reference's node order (scattered rays)
 *   10 pruned cooperative walk
 *   14 per-lane BVH walk + proof on the reference's tree (scattered rays, crt_bvh.h) */
template <int TRAV>
constexpr bool kIsCoop = TRAV == 4 || TRAV == 10;

template <int TRAV, bool COUNT>
__device__ __forceinline__ int trace(const DeviceScene &s, CoopLds *L, bool active, Vec o, Vec d, float &best_t,
                                     LaneCounts &c) {
    static_assert(TRAV == 4 || TRAV == 7 || TRAV == 8 || TRAV == 10 || TRAV == 12 || TRAV == 13 || TRAV == 14,
                  "no such walk");
    if constexpr (TRAV == 8) return trace_packet_pruned<COUNT, false>(s, active, o, d, best_t, c);
    else if constexpr (TRAV == 12 || TRAV == 13) return trace_packet_pruned<COUNT, true>(s, active, o, d, best_t, c);
    else if constexpr (TRAV == 4) return trace_coop<COUNT, false>(s, *L, active, o, d, best_t, c);
    else if constexpr (TRAV == 10) return trace_coop<COUNT, true>(s, *L, active, o, d, best_t, c);
    else if constexpr (TRAV == 14) return trace_lane_bvh<COUNT>(s, active, o, d, best_t, c);
    else return trace_packet<COUNT>(s, active, o, d, best_t, c);
}

__device__ __forceinline__ void make_hit(const DeviceScene &s, Vec o, Vec d, float t, int slot, HitRec &h,
                                         int32_t *tri_out = nullptr) {
    const DTriGeo g = load_global(s.slots, slot);
    const int32_t tri = load_global(s.slot_tri, slot);
    const DTriAttr at = load_global(s.tri_attr, tri);
    const DVec4 zero = {0.f, 0.f, 0.f, 0.f};
    DVec4 n0 = zero, n1 = zero, n2 = zero;
    if (at.mat_flags < 0) {
        n0 = load_global(s.vnormal, at.i0);
        n1 = load_global(s.vnormal, at.i1);
        n2 = load_global(s.vnormal, at.i2);
    }
    hit_record(o, d, t, g, at, n0, n1, n2, load_global(s.vuv, at.i0), load_global(s.vuv, at.i1),
               load_global(s.vuv, at.i2), h);
    if (tri_out) *tri_out = tri;
}

/* Shadow ray (option "shadows", DeviceScene::shadows).  At HEAD
 * trace_ray_with_refractions never enters its loop (crt_renderer.cpp:29-44),
 * so every light is unoccluded.  The course's earlier renderer traced it: its
 * committed renders 09-02/scene3 and 09-03/scene5 equal, at every pixel, the
 * image in which a light counts only when the shadow ray's closest hit is
 * absent or farther than the light (:90-92: distance^2 > |light - p|^2) —
 * which is also what the loop computes when it runs, since it intersects the
 * unchanged shadow ray every time (tests/test_shadows.py).  Per-lane pruned
 * walk (called from divergent shading code), closest hit as the reference. */
template <bool COUNT>
__device__ __forceinline__ bool shadow_occluded(const DeviceScene &s, Vec o, Vec d, float r2, LaneCounts &c) {
    float t;
    const int best = trace_lane_pruned<COUNT>(s, true, o, d, t, c);
    return best >= 0 && !(t * t > r2);
}

/* Diffuse direct term + normalisation (crt_renderer.cpp:81-99).  SHADOW: the
 * shadow-ray kernels (option "shadows", k_render_tiles<..., true>); their
 * traversals count in the work counters (c) as the oracle's do. */
template <bool SHADOW = false, bool COUNT = false>
__device__ __forceinline__ Vec diffuse_finish(const DeviceScene &s, const DSettings &st, Vec acc, Vec p, Vec n, Vec alb,
                                              LaneCounts *c = nullptr) {
    for (int l = 0; l < s.light_count; ++l) {
        const DLight L = s.lights[l];
        Vec ld = vsub(vec(L.px, L.py, L.pz), p);
        const float r2 = vlen_sq(ld);
        ld = vnormalize(ld);
        const float dn = vdot(ld, n);
        const float cos_law = (0.0f < dn) ? dn : 0.0f;          /* std::max(0.0f, dn) */
        const float area = 4 * kPi * r2;
        if (SHADOW && shadow_occluded<COUNT>(s, vadd(p, vscale(n, st.shadow_bias)), ld, r2, *c)) continue;
        acc = vadd(acc, vscale(vdiv(vscale(alb, L.intensity), area), cos_law));
    }
    return vdiv(acc, (float)(st.diffuse_reflection_ray_count + 1));
}

struct alignas(8) F2 { float c, s; };

/* One GI sample direction (crt_renderer.cpp:61-77).  rng.uniform() is
 * m * 2^-23 with m = next() >> 9, so cosf/sinf of pi*u and 2pi*u are table
 * lookups computed by the host's libm — bit-identical to the reference. */
__device__ __forceinline__ void gi_ray(const DeviceScene &s, const DSettings &st, const Frame &f, Pcg32 &rng, Vec &o,
                                       Vec &d) {
    const uint32_t m1 = rng.next() >> 9;
    const F2 cs1 = load_global(reinterpret_cast<const F2 *>(s.gi_pi), (int)m1);
    Vec dir = vec(cs1.c, cs1.s, 0.0f);
    const uint32_t m2 = rng.next() >> 9;
    const F2 cs2 = load_global(reinterpret_cast<const F2 *>(s.gi_2pi), (int)m2);
    const float c = cs2.c, sn = cs2.s;
    const float roty[9] = {c, 0.0f, -sn, 0.0f, 1.0f, 0.0f, sn, 0.0f, c};      /* crt_matrix.cpp:14-20 */
    dir = vec_mat(dir, roty);
    const float basis[9] = {f.a.x, f.a.y, f.a.z, f.n.x, f.n.y, f.n.z, f.b.x, f.b.y, f.b.z};   /* from_axes */
    dir = vec_mat(dir, basis);
    o = vadd(f.p, vscale(f.n, st.diffuse_reflection_bias));
    d = dir;
}

/* fresnel = 0.5f * std::pow(1.0f + dot, 5.0f) (crt_renderer.cpp:130), the
 * host libm's powf bit for bit.  The normal is flipped so that dot <= 0
 * (:117-121; |dot| <= 2 for any normal of length <= 2), and then
 * x = fl(1 + dot) is a multiple of 2^-24 in [-1, 1]: for dot in (-0.5, 0]
 * x rounds into [0.5, 1] where floats are multiples of 2^-24; for dot in
 * [-2, -0.5] the exact sum 1 + dot is a multiple of ulp(dot) >= 2^-24 below 1
 * in magnitude, hence representable.  So x * 2^24 is an exact integer and
 * indexes a table of powf(x, 5) computed by the host's libm (crt_hip_scene:
 * ensure_pow5_table).  Any other dot (NaN, or a smooth normal longer than 2)
 * falls back to x^5 in double rounded once. */
__device__ __forceinline__ float fresnel_of(const DeviceScene &s, float dot) {
    const float x = 1.0f + dot;
    if (s.pow5 != nullptr && dot >= -2.0f && dot <= 0.0f) {
        const int k = (int)(x * 16777216.0f);
        return 0.5f * load_global(s.pow5, k + 16777216);
    }
    const double xd = x;
    double r = xd * xd;
    r = r * r;
    r = r * xd;
    return 0.5f * (float)r;
}

/* shade_ray of a camera ray whose closest hit is known, for frames without
 * recursion (FULL=false: diffuse / constant materials, GI off) — the same
 * operations as shade_pixel<false>. */
__device__ __forceinline__ Vec shade_primary(const DeviceScene &s, const DSettings &st, Vec o, Vec d, int slot, float t) {
    if (slot < 0) return vec(s.background[0], s.background[1], s.background[2]);
    HitRec h;
    make_hit(s, o, d, t, slot, h);
    const DMaterial m = s.materials[h.mat];
    const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
    if (m.type == CRT_MATERIAL_DIFFUSE) return diffuse_finish(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb);
    return alb;
}

/* shade_ray for one camera ray (crt_renderer.cpp:46-155).
 * FULL=false: scenes whose materials are only diffuse/constant with GI off —
 * no recursion, no frame stack.  FULL=true: GI + reflective + refractive with
 * a per-lane frame stack of MAXF entries (≥ max_ray_depth + 1, host-checked). */
/* One pass of shade_pixel's loop: trace the lane's current ray (a wave-wide
 * walk call), shade the hit, and return colours to the pending activations
 * until one of them needs another ray.  Returns true when (o, d) holds that
 * next ray, false when the pixel's colour is in col. */
template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW = false>
__device__ __forceinline__ bool shade_pass(const DeviceScene &s, const DSettings &st, LaneCounts &cnt, CoopLds *L,
                                           bool has_px, Vec &o, Vec &d, uint32_t &depth, Pcg32 &rng, Frame *stack,
                                           int &sp, Vec &col) {
    /* Every pass of this loop traces exactly one ray per live lane, so all of a
     * wave's lanes meet in the same walk call whatever their position in their
     * own recursion (a miss shifts one lane's DFS against the others).  A call
     * that shade_ray would answer without tracing (depth > max_ray_depth: black,
     * crt_renderer.cpp:47-49) is resolved in the return loop below instead of
     * costing a pass; its GI draws are still taken (gi_ray) in reference order. */
    /* ---- shade_ray(ray) with depth <= max_ray_depth ---- */
    bool called = false;
    {
        float t;
        /* the packet walk pays for the union of its lanes' visit sets: it
         * wins on camera rays (coherent by construction) and loses on the
         * scattered secondary rays, which take the range-sharing walk */
        const int slot = (SEC != TRAV && depth != 0) ? trace<SEC, COUNT>(s, L, has_px, o, d, t, cnt)
                                                     : trace<TRAV, COUNT>(s, L, has_px, o, d, t, cnt);
        if (slot < 0) {
            col = vec(s.background[0], s.background[1], s.background[2]);
        } else {
            HitRec h;
            make_hit(s, o, d, t, slot, h);
            const DMaterial m = s.materials[h.mat];
            if (m.type == CRT_MATERIAL_DIFFUSE) {
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (FULL && s.gi_on && st.diffuse_reflection_ray_count > 0) {
                    Frame &f = stack[sp++];
                    f.kind = kDiffuseGI;
                    f.depth = (int32_t)depth;
                    f.i = 0;
                    f.acc = vec(0.f, 0.f, 0.f);
                    f.p = h.p;
                    f.n = h.n;
                    f.a = vnormalize(vcross(d, h.n));       /* right   */
                    f.b = vcross(f.a, h.n);                  /* forward */
                    f.alb = alb;
                    gi_ray(s, st, f, rng, o, d);
                    depth = depth + 1;
                    called = true;
                } else {
                    col = diffuse_finish<SHADOW, COUNT>(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb, &cnt);
                }
            } else if (FULL && m.type == CRT_MATERIAL_REFLECTIVE) {          /* :103-107 */
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (s.reflections_on) {
                    Frame &f = stack[sp++];
                    f.kind = kReflect;
                    f.depth = (int32_t)depth;
                    f.acc = alb;
                    o = vadd(h.p, vscale(h.n, st.reflection_bias));
                    d = vsub(d, vscale(vscale(h.n, 2.0f), vdot(d, h.n)));
                    depth = depth + 1;
                    called = true;
                } else {
                    col = alb;
                }
            } else if (FULL && m.type == CRT_MATERIAL_REFRACTIVE) {          /* :109-135 */
                if (!s.refractions_on) {
                    col = vec(0.f, 0.f, 0.f);
                } else {
                    Vec n = h.n;
                    float n_out = 1.0f, n_in = m.ior;
                    if (vdot(d, n) > 0.0f) {
                        n = vneg(n);
                        const float tmp = n_in; n_in = n_out; n_out = tmp;
                    }
                    Frame &f = stack[sp++];
                    f.kind = kRefractA;
                    f.depth = (int32_t)depth;
                    f.has_refr = 0;
                    {   /* Vector::refract (crt_vector.cpp:11-27) */
                        Vec rd = d;
                        const float ca = -vdot(rd, n);
                        const float sa = sqrtf(1.0f - ca * ca);
                        if (!(sa > n_in / n_out)) {
                            const float sb = sa * n_out / n_in;
                            const float cb = sqrtf(1.0f - sb * sb);
                            rd = vadd(rd, vscale(n, ca));
                            rd = vnormalize(rd);
                            rd = vscale(rd, sb);
                            rd = vadd(rd, vscale(vneg(n), cb));
                            f.has_refr = 1;
                        }
                        /* refracted_at → refract_at with its default 1e-2f bias (crt_ray.h:30-50) */
                        f.a = vadd(h.p, vscale(vneg(n), 1e-2f));
                        f.b = rd;
                    }
                    f.alb.x = fresnel_of(s, vdot(d, n));
                    o = vadd(h.p, vscale(n, st.reflection_bias));
                    d = vsub(d, vscale(vscale(n, 2.0f), vdot(d, n)));
                    depth = depth + 1;
                    called = true;
                }
            } else {                                                          /* Constant :137-139 */
                col = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
            }
        }
    }
    if (!FULL) return false;
    if (called) {
        if (depth <= st.max_ray_depth) return true;
        col = vec(0.f, 0.f, 0.f);       /* the child call returns black untraced */
        called = false;
    }
    /* ---- return col to the pending activations ---- */
    while (sp > 0) {
        Frame &f = stack[sp - 1];
        if (f.kind == kDiffuseGI) {
            f.acc = vadd(f.acc, col);
            f.i += 1;
            if ((uint32_t)f.i < st.diffuse_reflection_ray_count) {
                gi_ray(s, st, f, rng, o, d);
                depth = (uint32_t)f.depth + 1;
                if (depth <= st.max_ray_depth) {
                    called = true;
                    break;
                }
                col = vec(0.f, 0.f, 0.f);
                continue;
            }
            --sp;
            col = diffuse_finish<SHADOW, COUNT>(s, st, f.acc, f.p, f.n, f.alb, &cnt);
        } else if (f.kind == kReflect) {
            --sp;
            col = vmul_quirk(f.acc, col);
        } else if (f.kind == kRefractA) {
            if (f.has_refr) {
                f.kind = kRefractB;
                f.acc = col;
                o = f.a;
                d = f.b;
                depth = (uint32_t)f.depth + 1;
                if (depth <= st.max_ray_depth) {
                    called = true;
                    break;
                }
                col = vec(0.f, 0.f, 0.f);
                continue;
            }
            --sp;   /* total internal reflection: the reflection colour is the result */
        } else {
            --sp;
            const float fr = f.alb.x;
            col = vadd(vscale(f.acc, fr), vscale(col, 1.0f - fr));
        }
    }
    return called;
}

/* Shadow ray of shade_shadowed: true iff its closest hit is within the light
 * (crt_renderer.cpp:92, distance^2 <= |light - p|^2).  Any hit with
 * fl(t * t) <= r2 has t <= sqrt(r2) (1 + 2^-24) < lim0, so pruning past lim0
 * and stopping at the first such hit give the same answer as the closest hit. */
template <bool COUNT>
__device__ __forceinline__ bool shadow_occluded_packet(const DeviceScene &s, bool active, Vec o, Vec d, float r2,
                                                       LaneCounts &c) {
    const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
    if (COUNT && active) ++c.traversals;
    const float lim0 = sqrtf(r2) * (1.0f + 0x1p-20f);
    float t;
    const int best = trace_packet_pruned_t<COUNT, false, true>(s, active, o, d, rr, t, c, lim0, r2);
    return best >= 0 && !(t * t > r2);
}

/* Camera ray + shading with shadow rays for frames without recursion
 * (FULL=false, option "shadows"): the same operations as diffuse_finish<true>,
 * but each light's shadow rays are traced by the whole wave at once with the
 * pruned packet walk — a tile's shadow rays towards one light are coherent —
 * instead of one per-lane walk per lane. */
template <bool COUNT>
__device__ Vec shade_hit_shadowed(const DeviceScene &s, const DSettings &st, bool has_px, Vec o, Vec d, int slot,
                                  float t, LaneCounts &cnt) {
    Vec col = vec(s.background[0], s.background[1], s.background[2]);
    bool diffuse = false;
    HitRec h;
    h.p = vec(0.f, 0.f, 0.f);
    h.n = vec(0.f, 0.f, 1.f);
    Vec alb = vec(0.f, 0.f, 0.f);
    if (has_px && slot >= 0) {
        make_hit(s, o, d, t, slot, h);
        const DMaterial m = s.materials[h.mat];
        alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
        if (m.type == CRT_MATERIAL_DIFFUSE) diffuse = true;
        else col = alb;                                               /* Constant :137-139 */
    }
    Vec acc = vec(0.f, 0.f, 0.f);
    const int nl = s.light_count;
    for (int l = 0; l < nl; ++l) {                                    /* :81-96 */
        const DLight Lt = s.lights[l];
        Vec ld = vsub(vec(Lt.px, Lt.py, Lt.pz), h.p);
        const float r2 = vlen_sq(ld);
        ld = vnormalize(ld);
        const float dn = vdot(ld, h.n);
        const float cos_law = (0.0f < dn) ? dn : 0.0f;
        const float area = 4 * kPi * r2;
        bool lit = true;
        if (__ballot(diffuse) != 0ull)
            lit = !shadow_occluded_packet<COUNT>(s, diffuse, vadd(h.p, vscale(h.n, st.shadow_bias)), ld, r2, cnt);
        if (diffuse && lit) acc = vadd(acc, vscale(vdiv(vscale(alb, Lt.intensity), area), cos_law));
    }
    if (diffuse) col = vdiv(acc, (float)(st.diffuse_reflection_ray_count + 1));
    return col;
}

template <int TRAV, bool COUNT>
__device__ Vec shade_shadowed(const DeviceScene &s, const DSettings &st, int x, int y, LaneCounts &cnt, CoopLds *L,
                              bool has_px) {
    Vec o, d;
    camera_ray(s, x, y, o, d);
    float t;
    const int slot = trace<TRAV, COUNT>(s, L, has_px, o, d, t, cnt);
    return shade_hit_shadowed<COUNT>(s, st, has_px, o, d, slot, t, cnt);
}

template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW = false>
__device__ Vec shade_pixel(const DeviceScene &s, const DSettings &st, int x, int y, LaneCounts &cnt, CoopLds *L,
                           bool has_px) {
    Vec o, d;
    camera_ray(s, x, y, o, d);
    uint32_t depth = 0;
    Pcg32 rng;
    if (FULL) rng = make_pcg((uint32_t)x, (uint32_t)y);
    Frame stack[MAXF > 0 ? MAXF : 1];
    int sp = 0;
    Vec col;
    while (shade_pass<FULL, MAXF, TRAV, SEC, COUNT, SHADOW>(s, st, cnt, L, has_px, o, d, depth, rng, stack, sp, col)) {
    }
    return col;
}

#ifndef CRT_GI_WAVES
#define CRT_GI_WAVES 5       /* min waves/SIMD asked of the depth<=3 frame-stack (GI) kernels: 96 VGPRs
                                * + 17 spilled beat 114 VGPRs at 4 waves (C4 1080^2: 102.8 vs 111.7 ms) and
                                * 80 VGPRs at 6 waves (116.6 ms) in same-box A/B */
#endif
#ifndef CRT_WINDOW_WAVES
#define CRT_WINDOW_WAVES 5   /* min waves/SIMD asked of the walk-13 kernel: 96 VGPRs (1 spilled); C2 0.1233 ms at
                              * its best plan vs 0.127-0.130 at 4 waves (profiles/r02/w5tune) */
#endif
#ifndef CRT_RENDER_BOUNDS
#define CRT_RENDER_BOUNDS __launch_bounds__(256)
#endif
template <bool FULL, int MAXF, int TRAV, int SEC, bool COUNT, bool SHADOW = false>
#ifndef CRT_PACKET_WAVES
#define CRT_PACKET_WAVES 5   /* min waves/SIMD asked of the walk-12 kernel (as walk 13) */
#endif
__global__ CRT_RENDER_BOUNDS __attribute__((amdgpu_waves_per_eu(TRAV == 13 ? CRT_WINDOW_WAVES : TRAV == 12 ? CRT_PACKET_WAVES : (FULL && MAXF == 4 ? CRT_GI_WAVES : 1)))) void k_render_tiles(const DeviceScene *__restrict__ scene, DSettings st,
                                                  const Tile *__restrict__ tiles,
                                                      int ntiles, float *__restrict__ out,
                                                      unsigned long long *__restrict__ counters,
                                                      unsigned long long *__restrict__ stamps) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = (int)(threadIdx.x & 63);
    if (wave >= ntiles) return;
    /* The scene record is read through a pointer (not a by-value kernel
     * argument): its fields are then loaded where they are used, so shading
     * constants are not held in SGPRs across the tree walk (6 -> more waves/SIMD). */
    const DeviceScene &s = *scene;
    /* diagnostic build only (stamps != nullptr): wave start / end in s_memrealtime ticks (100 MHz) */
    if (stamps && lane == 0) stamps[2 * wave] = __builtin_amdgcn_s_memrealtime();
    const Tile tl = tiles[wave];
    /* the heaviest tiles set the frame length (their walks are long chains of
     * dependent loads): they get issue priority over the light waves that
     * share their SIMD (s_setprio; scheduling only, results unchanged) */
    if (tl.prio) __builtin_amdgcn_s_setprio(3);
    if constexpr (TRAV == 13 && !FULL) {
        /* tiles of <= 16 rays (the measured plan's splits of heavy tiles): window walk */
        const int tw = uniform_i(tl.w), th = uniform_i(tl.h);
        const int npx = tw * th;
        if (npx <= 16) {
            const int R = npx <= 4 ? 4 : 16;
            const int r = lane & (R - 1), sl = lane / R;
            const bool act = r < npx;
            const int px = act ? r % tw : 0, py = act ? r / tw : 0;
            Vec o, d;
            camera_ray(s, tl.x + px, tl.y + py, o, d);
            LaneCounts cw = {};
            float t;
            const int slot = R == 4 ? trace_window<COUNT, 4>(s, r, sl, act, o, d, t, cw)
                                    : trace_window<COUNT, 16>(s, r, sl, act, o, d, t, cw);
            Vec c;
            if constexpr (SHADOW) c = shade_hit_shadowed<COUNT>(s, st, act && sl == 0, o, d, slot, t, cw);   /* wave-wide */
            if (act && sl == 0) {
                if constexpr (!SHADOW) c = shade_primary(s, st, o, d, slot, t);
                float *pxo = out + 3 * (tl.out_base + (int64_t)py * tl.out_stride + px);
                pxo[0] = c.x;
                pxo[1] = c.y;
                pxo[2] = c.z;
            }
            if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
            if (COUNT) {
                atomicAdd(&counters[0], (unsigned long long)cw.traversals);
                atomicAdd(&counters[1], (unsigned long long)cw.nodes);
                atomicAdd(&counters[2], (unsigned long long)cw.tris);
                atomicAdd(&counters[3], (unsigned long long)cw.hits);
                if (lane == 0) {
                    atomicAdd(&counters[4], (unsigned long long)cw.wave_nodes);
                    atomicAdd(&counters[5], (unsigned long long)cw.wave_tris);
                    atomicAdd(&counters[6], (unsigned long long)cw.wave_edges);
                    atomicAdd(&counters[7], 1ull);
                    atomicAdd(&counters[8], (unsigned long long)cw.wave_box);
                    atomicAdd(&counters[9], (unsigned long long)cw.wave_pass);
                    atomicAdd(&counters[10], 1ull);   /* window-walk waves */
                    atomicAdd(&counters[11], (unsigned long long)cw.win_steps);
                    atomicAdd(&counters[14], (unsigned long long)cw.win_rounds);
                }
                atomicAdd(&counters[12], (unsigned long long)cw.win_slots);
                atomicAdd(&counters[13], (unsigned long long)cw.win_reached);
            }
            return;
        }
    }
    const int lx = lane & 7, ly = lane >> 3;
    const bool has_px = lx < tl.w && ly < tl.h;
    /* the sharing walks keep pixel-less lanes as helpers (they take donated node
     * ranges of the wave's rays); the other walks drop them */
    constexpr bool kHelpers = !FULL;   /* sharing walks use them; packet walks ignore them */
    if (!kHelpers && !has_px) return;
    LaneCounts cnt = {};
    constexpr bool kCoop = kIsCoop<TRAV> || kIsCoop<SEC>;   /* LDS only for the sharing walks */
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    Vec c;
    if constexpr (SHADOW && !FULL)
        c = shade_shadowed<TRAV, COUNT>(s, st, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0), cnt,
                                        &coop[kCoop ? (threadIdx.x >> 6) : 0], has_px);
    else
        c = shade_pixel<FULL, MAXF, TRAV, SEC, COUNT, SHADOW>(s, st, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0),
                                                              cnt, &coop[kCoop ? (threadIdx.x >> 6) : 0], has_px);
    if (has_px) {
        float *px = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
        px[0] = c.x;
        px[1] = c.y;
        px[2] = c.z;
    }
    if (stamps && lane == 0) stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
        if (lane == 0) {
            atomicAdd(&counters[4], (unsigned long long)cnt.wave_nodes);
            atomicAdd(&counters[5], (unsigned long long)cnt.wave_tris);
            atomicAdd(&counters[6], (unsigned long long)cnt.wave_edges);
            atomicAdd(&counters[7], 1ull);
            atomicAdd(&counters[8], (unsigned long long)cnt.wave_box);
            atomicAdd(&counters[9], (unsigned long long)cnt.wave_pass);
        }
    }
}

/* Frame-stack kernel with pixel refill (GI frames, cooperative walk).  A
 * persistent grid of waves pulls pixels from the tile list in plan order
 * (one global counter, one atomic per wave and pass): a lane whose pixel is
 * finished takes the next one at the top of the following pass, so a wave no
 * longer waits for its tile's longest pixel with the other lanes idle.  Every
 * pixel runs exactly shade_pixel's sequence (camera ray, PCG seeded by (x, y),
 * the same passes), so the image bits do not depend on which lane or wave
 * renders it.  Lanes without a pixel stay in the walk calls as helpers (they
 * take donated pieces); the wave leaves when the list is exhausted and none
 * of its lanes holds a pixel. */
template <int MAXF, int TRAV, bool COUNT>
#ifndef CRT_GI10_WAVES
#define CRT_GI10_WAVES 4     /* min waves/SIMD of the refill kernel with the pruned walk (TRAV 10) */
#endif
#ifndef CRT_GI14_WAVES
#define CRT_GI14_WAVES 1     /* ... with the per-lane BVH walk (TRAV 14): no minimum */
#endif
__global__ CRT_RENDER_BOUNDS __attribute__((amdgpu_waves_per_eu(MAXF == 4 ? (TRAV == 10 ? CRT_GI10_WAVES : TRAV == 14 ? CRT_GI14_WAVES : CRT_GI_WAVES) : 1))) void k_render_refill(
    const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles, int ntiles,
    float *__restrict__ out, int32_t *__restrict__ next_px, unsigned long long *__restrict__ counters) {
    const int lane = (int)(threadIdx.x & 63);
    const DeviceScene &s = *scene;
    const int total = ntiles * 64;   /* pixel slots: tile k, lane j -> (j & 7, j >> 3) inside tile k */
    const unsigned long long lt = (1ull << lane) - 1ull;
    __shared__ CoopLds coop[kIsCoop<TRAV> ? 4 : 1];
    CoopLds *L = &coop[kIsCoop<TRAV> ? (threadIdx.x >> 6) : 0];
    LaneCounts cnt = {};
    bool has = false, dry = false;
    int64_t opx = 0;
    Vec o = vec(0.f, 0.f, 0.f), d = vec(0.f, 0.f, 1.f), col = vec(0.f, 0.f, 0.f);
    uint32_t depth = 0;
    Pcg32 rng = make_pcg(0u, 0u);
    Frame stack[MAXF];
    int sp = 0;
    for (;;) {
        /* ---- lanes without a pixel take the next slots of the list ---- */
        const unsigned long long need = __ballot(!has && !dry);
        if (need != 0ull) {
            const int leader = __ffsll((long long)need) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(next_px, __popcll(need));
            base = __shfl(base, leader);
            if (!has && !dry) {
                const int k = base + __popcll(need & lt);
                if (k >= total) {
                    dry = true;
                } else {
                    const Tile tl = tiles[k >> 6];
                    const int lx = k & 7, ly = (k >> 3) & 7;
                    if (lx < tl.w && ly < tl.h) {   /* slots outside a partial tile: retry next pass */
                        has = true;
                        opx = tl.out_base + (int64_t)ly * tl.out_stride + lx;
                        camera_ray(s, tl.x + lx, tl.y + ly, o, d);
                        depth = 0;
                        rng = make_pcg((uint32_t)(tl.x + lx), (uint32_t)(tl.y + ly));
                        sp = 0;
                    }
                }
            }
        }
        if (!__any(has)) {
            if (__any(!dry)) continue;
            break;
        }
        const bool more = shade_pass<true, MAXF, TRAV, TRAV, COUNT>(s, st, cnt, L, has, o, d, depth, rng, stack, sp,
                                                                     col);
        if (has && !more) {
            float *px = out + 3 * opx;
            px[0] = col.x;
            px[1] = col.y;
            px[2] = col.z;
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

/* The GI refill kernels are compiled in a translation unit of their own
 * (crt_render_gi.hip, which includes this file with CRT_GI_TU defined) so that
 * they can take their own LLVM scheduling strategy (max-memory-clause: C4
 * 1080^2 77.3 -> 75.3 ms, profiles/r01/ab_wf_waves_sched_strategy.log) while
 * the C2 camera kernel keeps the default one. */
#define CRT_REFILL_INSTANCES(X) X(4, 4, false) X(4, 4, true) X(4, 10, false) X(4, 10, true) \
    X(16, 4, false) X(16, 4, true) X(64, 4, false) X(64, 4, true) X(4, 14, false) X(4, 14, true) \
    X(16, 14, false) X(16, 14, true) X(64, 14, false) X(64, 14, true)
#define CRT_REFILL_SIG(MAXF, T, C) void k_render_refill<MAXF, T, C>(const DeviceScene *__restrict__, DSettings, \
    const Tile *__restrict__, int, float *__restrict__, int32_t *__restrict__, unsigned long long *__restrict__);
#ifdef CRT_GI_TU
#define CRT_REFILL_INST(MAXF, T, C) template __global__ CRT_REFILL_SIG(MAXF, T, C)
CRT_REFILL_INSTANCES(CRT_REFILL_INST)
#elif !defined(CRT_SIDE_TU)
#define CRT_REFILL_EXTERN(MAXF, T, C) extern template __global__ CRT_REFILL_SIG(MAXF, T, C)
CRT_REFILL_INSTANCES(CRT_REFILL_EXTERN)
#endif
}  // namespace crt_amd

#include "crt_gi_machine.h"   /* GI frames as a per-lane state machine (k_render_gi) */

namespace crt_amd {



/* Calibration probe (measured-cost tile plan): the camera rays of a tile
 * list traced with the frame's primary walk, no shading.  Each wave writes
 * its cost: for the packet walks the wave's node + triangle + edge steps
 * (what the wave pays: the union of its lanes' visit sets), for per-lane
 * walks the largest lane's node + triangle tests. */
template <int TRAV>
__global__ __launch_bounds__(256) void k_probe_tiles(const DeviceScene *__restrict__ scene,
                                                     const Tile *__restrict__ tiles, int ntiles,
                                                     uint32_t *__restrict__ wave_cost) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = (int)(threadIdx.x & 63);
    if (wave >= ntiles) return;
    const DeviceScene &s = *scene;
    const Tile tl = tiles[wave];
    const int lx = lane & 7, ly = lane >> 3;
    const bool has_px = lx < tl.w && ly < tl.h;
    Vec o, d;
    camera_ray(s, tl.x + (has_px ? lx : 0), tl.y + (has_px ? ly : 0), o, d);
    LaneCounts cnt = {};
    constexpr bool kCoop = kIsCoop<TRAV>;
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    float t;
    (void)trace<TRAV, true>(s, &coop[kCoop ? (threadIdx.x >> 6) : 0], has_px, o, d, t, cnt);
    constexpr bool kPacket = !kIsCoop<TRAV>;
    uint32_t c = kPacket ? cnt.wave_nodes + cnt.wave_tris + cnt.wave_edges : cnt.nodes + cnt.tris;
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o2 = (uint32_t)__shfl_xor((int)c, off);
        c = c > o2 ? c : o2;
    }
    if (lane == 0) wave_cost[wave] = c;
}

/* ====================================================================== */
/* Wavefront path: reflection / refraction recursion without GI (C3)       */
/* ====================================================================== */
/* With GI off, shade_ray (crt_renderer.cpp:46-145) draws no random numbers:
 * each activation's colour is a pure function of its ray and of its
 * children's colours.  So the recursion is run level by level: every ray of
 * depth L is traced by one lane (no per-lane frame stack, no lane waiting for
 * its pixel's other branches), its children are appended to the level-L+1
 * queue, and a backward pass composes each activation's colour from its
 * children with the reference's operations (reflective: albedo * L with the
 * Vector quirk; refractive: fresnel blend, or the reflection colour on total
 * internal reflection).  A child deeper than max_ray_depth is black without
 * a trace, as in the reference (:47-48).  Level 0 is the camera rays of the
 * tile plan (packet walk); deeper levels are scattered rays (range-sharing
 * walk). */
enum WKind : int32_t { wFinal = 0, wReflect = 1, wRefract2 = 2, wRefract1 = 3 };

struct alignas(16) WRay {
    float ox, oy, oz, dx, dy, dz;
    int32_t id, depth;
};

struct alignas(16) WNode {
    int32_t kind, c0, c1, pad;   /* children ids, -1 = black (deeper than max_ray_depth) */
    float a0, a1, a2, a3;        /* reflective: albedo | refractive: a0 = fresnel */
};

struct WLevel {
    const WRay *in;
    int32_t n;               /* rays of this level (levels >= 1) */
    int32_t depth;
    WRay *out;               /* children of this level */
    int32_t *out_count;
    int32_t out_base;        /* id of out[0] */
    WNode *nodes;            /* by ray id */
    DVec4 *cols;             /* by ray id */
    int32_t rpw;             /* levels >= 1: rays per wave (lanes rpw..63 start idle and take donated pieces) */
    int32_t out_cap;         /* children this level may queue (recorded level sizes: exactly the next level) */
    int32_t *overflow;       /* set when a level queued more children than out_cap (none written) */
};

template <int TRAV, bool LEVEL0, bool COUNT>
#ifndef CRT_WF_WAVES
#define CRT_WF_WAVES 1       /* min waves/SIMD asked of the wavefront levels >= 1 */
#endif
#ifndef CRT_WF0_WAVES
#define CRT_WF0_WAVES 1      /* ... and of level 0 (camera rays) */
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LEVEL0 ? CRT_WF0_WAVES : CRT_WF_WAVES))) void k_wf_level(const DeviceScene *__restrict__ scene, DSettings st,
                                                  const Tile *__restrict__ tiles, int ntiles, WLevel lv,
                                                  unsigned long long *__restrict__ counters) {
    const DeviceScene &s = *scene;
    const int gid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int lane = (int)(threadIdx.x & 63);
    bool has;
    Vec o = vec(0.f, 0.f, 0.f), d = vec(0.f, 0.f, 1.f);
    int id = gid, depth = 0;
    if (LEVEL0) {
        const int wave = gid >> 6;
        if (wave >= ntiles) return;
        const Tile tl = tiles[wave];
        if (tl.prio) __builtin_amdgcn_s_setprio(3);
        const int lx = lane & 7, ly = lane >> 3;
        has = lx < tl.w && ly < tl.h;
        if (has) camera_ray(s, tl.x + lx, tl.y + ly, o, d);
    } else {
        const int ray0 = (gid >> 6) * lv.rpw;
        if (ray0 >= lv.n) return;          /* whole wave past the queue */
        const int ray = ray0 + lane;
        has = lane < lv.rpw && ray < lv.n;
        if (has) {
            const WRay r = lv.in[ray];
            o = vec(r.ox, r.oy, r.oz);
            d = vec(r.dx, r.dy, r.dz);
            id = r.id;
            depth = r.depth;
        }
    }
    LaneCounts cnt = {};
    constexpr bool kCoop = kIsCoop<TRAV>;
    __shared__ CoopLds coop[kCoop ? 4 : 1];
    float t;
    const int slot = trace<TRAV, COUNT>(s, &coop[kCoop ? (threadIdx.x >> 6) : 0], has, o, d, t, cnt);

    WNode node = {wFinal, -1, -1, 0, 0.f, 0.f, 0.f, 0.f};
    Vec col = vec(0.f, 0.f, 0.f);
    int nch = 0;
    Vec co[2], cd[2];
    if (has) {
        if (slot < 0) {
            col = vec(s.background[0], s.background[1], s.background[2]);
        } else {
            HitRec h;
            make_hit(s, o, d, t, slot, h);
            const DMaterial m = s.materials[h.mat];
            if (m.type == CRT_MATERIAL_DIFFUSE) {
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                col = diffuse_finish(s, st, vec(0.f, 0.f, 0.f), h.p, h.n, alb);
            } else if (m.type == CRT_MATERIAL_REFLECTIVE) {                 /* :103-107 */
                const Vec alb = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
                if (s.reflections_on) {
                    node.kind = wReflect;
                    node.a0 = alb.x; node.a1 = alb.y; node.a2 = alb.z;
                    co[0] = vadd(h.p, vscale(h.n, st.reflection_bias));
                    cd[0] = vsub(d, vscale(vscale(h.n, 2.0f), vdot(d, h.n)));
                    nch = 1;
                } else {
                    col = alb;
                }
            } else if (m.type == CRT_MATERIAL_REFRACTIVE) {                 /* :109-135 */
                if (s.refractions_on) {
                    Vec n = h.n;
                    float n_out = 1.0f, n_in = m.ior;
                    if (vdot(d, n) > 0.0f) {
                        n = vneg(n);
                        const float tmp = n_in; n_in = n_out; n_out = tmp;
                    }
                    bool has_refr = false;
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
                            has_refr = true;
                        }
                    }
                    node.kind = has_refr ? wRefract2 : wRefract1;
                    node.a0 = fresnel_of(s, vdot(d, n));
                    co[0] = vadd(h.p, vscale(n, st.reflection_bias));
                    cd[0] = vsub(d, vscale(vscale(n, 2.0f), vdot(d, n)));
                    co[1] = vadd(h.p, vscale(vneg(n), 1e-2f));   /* refract_at's default bias (crt_ray.h:30-50) */
                    cd[1] = rd;
                    nch = has_refr ? 2 : 1;
                }
            } else {                                                         /* Constant :137-139 */
                col = sample_texture(s.textures[m.tex], s.texels, h.uv, h.bu, h.bv);
            }
        }
    }
    /* children deeper than max_ray_depth are black without a trace: not queued */
    if ((uint32_t)depth + 1u > st.max_ray_depth) nch = 0;
    const unsigned long long b1 = __ballot(nch >= 1), b2 = __ballot(nch >= 2);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int total = __popcll(b1) + __popcll(b2);
    if (total > 0) {
        int base = 0;
        if (lane == __ffsll((long long)(b1 | b2)) - 1) {
            base = atomicAdd(lv.out_count, total);
            if (base + total > lv.out_cap) atomicOr(lv.overflow, 1);
        }
        base = __shfl(base, __ffsll((long long)(b1 | b2)) - 1);
        if (base + total > lv.out_cap) nch = 0;   /* never past the queue (the frame is then reported, not used) */
        /* a lane's children side by side */
        const int k0 = base + __popcll(b1 & lt) + __popcll(b2 & lt);
        const int k1 = k0 + 1;
        for (int c = 0; c < nch; ++c) {
            const int k = c == 0 ? k0 : k1;
            WRay r;
            r.ox = co[c].x; r.oy = co[c].y; r.oz = co[c].z;
            r.dx = cd[c].x; r.dy = cd[c].y; r.dz = cd[c].z;
            r.id = lv.out_base + k;
            r.depth = depth + 1;
            lv.out[k] = r;
            if (c == 0) node.c0 = r.id; else node.c1 = r.id;
        }
    }
    if (has) {
        lv.nodes[id] = node;
        if (node.kind == wFinal) lv.cols[id] = DVec4{col.x, col.y, col.z, 0.f};
    }
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
        /* levels >= 1 (coop walks): loop rounds per wave — sum, longest wave, waves */
        if (!LEVEL0 && kCoop && lane == 0) {
            atomicAdd(&counters[4], (unsigned long long)cnt.wave_nodes);
            atomicMax(&counters[6], (unsigned long long)cnt.wave_nodes);
            atomicAdd(&counters[7], 1ull);
        }
    }
}

__device__ __forceinline__ Vec wf_compose(const WNode &nd, const DVec4 *__restrict__ cols, Vec own) {
    if (nd.kind == wFinal) return own;
    const Vec black = vec(0.f, 0.f, 0.f);
    const Vec c0 = nd.c0 >= 0 ? vec(cols[nd.c0].x, cols[nd.c0].y, cols[nd.c0].z) : black;
    if (nd.kind == wReflect) return vmul_quirk(vec(nd.a0, nd.a1, nd.a2), c0);
    if (nd.kind == wRefract1) return c0;   /* total internal reflection */
    const Vec c1 = nd.c1 >= 0 ? vec(cols[nd.c1].x, cols[nd.c1].y, cols[nd.c1].z) : black;
    const float fr = nd.a0;
    return vadd(vscale(c0, fr), vscale(c1, 1.0f - fr));
}

/* Wavefront levels >= 1 (C3): own translation unit (crt_render_wf.hip) and
 * LLVM scheduling strategy, as for the GI refill kernels above. */
#define CRT_WF_INSTANCES(X) X(4, false) X(4, true) X(10, false) X(10, true) X(14, false) X(14, true)
#define CRT_WF_SIG(SEC, C) void k_wf_level<SEC, false, C>(const DeviceScene *__restrict__, DSettings, \
    const Tile *__restrict__, int, WLevel, unsigned long long *__restrict__);
#ifdef CRT_WF_TU
#define CRT_WF_INST(SEC, C) template __global__ CRT_WF_SIG(SEC, C)
CRT_WF_INSTANCES(CRT_WF_INST)
#elif !defined(CRT_SIDE_TU)
#define CRT_WF_EXTERN(SEC, C) extern template __global__ CRT_WF_SIG(SEC, C)
CRT_WF_INSTANCES(CRT_WF_EXTERN)
#endif

#ifndef CRT_SIDE_TU
/* levels >= 1, deepest first: colour of every activation of the level */
__global__ __launch_bounds__(256) void k_wf_compose(const WNode *__restrict__ nodes, DVec4 *__restrict__ cols,
                                                    int32_t begin, int32_t n) {
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= n) return;
    const int id = begin + k;
    const WNode nd = nodes[id];
    if (nd.kind == wFinal) return;
    const Vec c = wf_compose(nd, cols, vec(0.f, 0.f, 0.f));
    cols[id] = DVec4{c.x, c.y, c.z, 0.f};
}

/* level 0: compose the camera rays and write the pixels */
__global__ __launch_bounds__(256) void k_wf_pixels(const WNode *__restrict__ nodes, const DVec4 *__restrict__ cols,
                                                   const Tile *__restrict__ tiles, int ntiles,
                                                   float *__restrict__ out) {
    const int gid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int wave = gid >> 6, lane = gid & 63;
    if (wave >= ntiles) return;
    const Tile tl = tiles[wave];
    const int lx = lane & 7, ly = lane >> 3;
    if (!(lx < tl.w && ly < tl.h)) return;
    const WNode nd = nodes[gid];
    const Vec own = vec(cols[gid].x, cols[gid].y, cols[gid].z);
    const Vec c = wf_compose(nd, cols, own);
    float *px = out + 3 * (tl.out_base + (int64_t)ly * tl.out_stride + lx);
    px[0] = c.x;
    px[1] = c.y;
    px[2] = c.z;
}

/* crt_hip_trace_batch: closest hit of arbitrary rays (a1–a4 KATs). */
__global__ __launch_bounds__(256) void k_trace_rays(DeviceScene s, const float *__restrict__ rays, int64_t n,
                                                    crt_hit *__restrict__ hits, int walk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
    const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    LaneCounts cnt;
    float t;
    const int slot = walk == 2 && s.bnodes ? trace_lane_bvh<false>(s, true, o, d, t, cnt)
                     : walk >= 1 ? trace_lane_pruned<false>(s, true, o, d, t, cnt) : trace_closest<false>(s, o, d, t, cnt);
    crt_hit r;
    r.distance = 0.f;
    r.point[0] = r.point[1] = r.point[2] = 0.f;
    r.normal[0] = r.normal[1] = r.normal[2] = 0.f;
    r.uv[0] = r.uv[1] = r.uv[2] = 0.f;
    r.bary_u = r.bary_v = 0.f;
    r.material_index = 0;
    r.hit = 0;
    r.triangle_index = -1;
    if (slot >= 0) {
        HitRec h;
        int32_t tri;
        make_hit(s, o, d, t, slot, h, &tri);
        r.distance = h.t;
        r.point[0] = h.p.x; r.point[1] = h.p.y; r.point[2] = h.p.z;
        r.normal[0] = h.n.x; r.normal[1] = h.n.y; r.normal[2] = h.n.z;
        r.uv[0] = h.uv.x; r.uv[1] = h.uv.y; r.uv[2] = h.uv.z;
        r.bary_u = h.bu; r.bary_v = h.bv;
        r.material_index = h.mat;
        r.hit = 1;
        r.triangle_index = tri;
    }
    hits[i] = r;
}

/* Scatter gathered shard buffers back into the row-major frame (fp32 RGB or
 * the quantised 8-bit RGB of k_quantize). */
template <class T>
struct Rgb { T c[3]; };

template <class T>
__global__ __launch_bounds__(256) void k_unpack(const UnpackBucket *__restrict__ buckets, const T *__restrict__ src,
                                                T *__restrict__ dst, int width, Rgb<T> bg) {
    const UnpackBucket b = buckets[blockIdx.x];
    const int npx = b.w * b.h;
    for (int p = (int)threadIdx.x; p < npx; p += (int)blockDim.x) {
        const int lx = p % b.w, ly = p / b.w;
        T *d = dst + 3 * ((int64_t)(b.y + ly) * width + (b.x + lx));
        if (b.src < 0) {   /* dead tile of a compact shard: the background (shade_ray's miss colour) */
            d[0] = bg.c[0];
            d[1] = bg.c[1];
            d[2] = bg.c[2];
        } else {
            const T *s = src + b.src + 3 * (int64_t)p;
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
        }
    }
}

/* Live pixels for the compact shards: the camera ray passes the reference's
 * six-face test on the root cell (crt_intersection.cpp:14-45, node 0 popped
 * first, :114-121).  A ray that fails it is a miss, i.e. shade_ray returns the
 * background colour (crt_renderer.cpp:142-144) — so dead pixels need neither
 * rendering nor transport. */
__global__ __launch_bounds__(256) void k_live_pixels(const DeviceScene *__restrict__ scene, uint8_t *__restrict__ live) {
    const DeviceScene &s = *scene;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)s.width * s.height) return;
    const int x = (int)(i % s.width), y = (int)(i / s.width);
    Vec o, d;
    camera_ray(s, x, y, o, d);
    bool hit = false;
    if (s.node_count > 0) {
        const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
        hit = box_hit_r(o, d, rr, load_global(s.nodes, 0));
    }
    live[i] = hit ? 1 : 0;
}

/* write_ppm's per-component conversion (crt_image_ppm.cpp:15-18):
 * clamp(static_cast<int>(c * max), 0, max), with x86 cvttss2si semantics for
 * the cast (NaN / out of range -> INT_MIN -> 0).  Four components per thread:
 * 16-B loads, one 4-B store (HBM-bound: 5 B moved per component). */
__global__ __launch_bounds__(256) void k_quantize(const float *__restrict__ src, uint8_t *__restrict__ dst, int64_t n,
                                                  float maxf, int maxi) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = 4 * q;
    if (i >= n) return;
    auto cv = [&](float c) -> uint32_t {
        int v = trunc_x86(c * maxf);
        v = v < 0 ? 0 : (v > maxi ? maxi : v);
        return (uint32_t)v;
    };
    if (i + 4 <= n && ((reinterpret_cast<uintptr_t>(src + i) & 15u) == 0) &&
        ((reinterpret_cast<uintptr_t>(dst + i) & 3u) == 0)) {
        const float4 c = *reinterpret_cast<const float4 *>(src + i);
        const uint32_t w = cv(c.x) | (cv(c.y) << 8) | (cv(c.z) << 16) | (cv(c.w) << 24);
        *reinterpret_cast<uint32_t *>(dst + i) = w;
    } else {
        for (int64_t k = i; k < n && k < i + 4; ++k) dst[k] = (uint8_t)cv(src[k]);
    }
}

#endif  // CRT_SIDE_TU
}  // namespace crt_amd
#ifndef CRT_SIDE_TU

/* ====================================================================== */
/*  C-ABI                                                                  */
/* ====================================================================== */
using namespace crt_amd;

namespace {

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        const hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                                    \
            return set_error(CRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

struct ShardPlan {
    Tile *d_tiles = nullptr;
    int ntiles = 0;
    int64_t packed_pixels = 0;
    std::vector<Tile> tiles;     /* host copy, dispatch order */
    std::vector<float> cost;     /* measured cost per tile (calibrated plans), else empty */
    bool has_small = false;      /* some tile has <= 16 pixels (walk 13 runs them with the window walk) */
};

struct GiTables { float *d = nullptr; };   /* 4 * 2^23 floats on one device */

std::mutex g_gi_mu;
std::map<int, GiTables> g_gi;              /* per device, process lifetime */
std::vector<float> g_gi_host;

constexpr int64_t kGiN = int64_t(1) << 23;

void build_gi_host_tables() {
    if (!g_gi_host.empty()) return;
    g_gi_host.resize((size_t)(4 * kGiN));
    /* (cos, sin) pairs: one 8-B read per angle (the tables are 64 MB each and
     * read at random: one cache line per angle instead of two) */
    float *pi2 = g_gi_host.data(), *tau2 = pi2 + 2 * kGiN;
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < nt; ++w) {
        pool.emplace_back([=]() {
            for (int64_t m = w; m < kGiN; m += nt) {
                const float u = (float)m * (1.0f / 8388608.0f);          /* = uniform() exactly */
                const float a = kPi * u;                                  /* crt_renderer.cpp:68 */
                const float b = 2.0f * kPi * u;                           /* crt_renderer.cpp:71 */
                pi2[2 * m] = std::cos(a);
                pi2[2 * m + 1] = std::sin(a);
                tau2[2 * m] = std::cos(b);
                tau2[2 * m + 1] = std::sin(b);
            }
        });
    }
    for (auto &t : pool) t.join();
}

}  // namespace

/* Device buffers of the wavefront path, grown on demand (kept across frames). */
struct WfBuffers {
    crt_amd::WNode *nodes = nullptr;
    crt_amd::DVec4 *cols = nullptr;
    int64_t cap = 0;             /* ray ids */
    crt_amd::WRay *q[2] = {nullptr, nullptr};
    int64_t qcap[2] = {0, 0};
    int32_t *counts = nullptr;   /* children queued per level; counts[count_cap - 1]: overflow flag */
    int count_cap = 0;
    /* Level sizes of the last frame traced with host read-backs, and what they
     * depend on (settings, tile list): a frame's level sizes are a function of
     * its rays alone, so later frames with the same key launch every level
     * with these sizes and no host sync (render_wavefront). */
    struct Rec {
        std::vector<int32_t> sizes;   /* rays of levels 1, 2, ... */
        crt_renderer_settings st{};
        int ntiles = 0;
    };
    std::map<const void *, Rec> recs;   /* by tile list (device pointer; cleared when plans are freed) */
    /* overflow flag of recorded-size frames: device word, copied into pinned
     * host memory behind each such frame and read once that copy is done */
    int32_t *d_flag = nullptr;
    int32_t *h_flag = nullptr;
    hipEvent_t flag_ev = nullptr;
    bool flag_pending = false;
    /* recorded-size frames captured as HIP graphs, by everything their
     * launches bake in (cleared whenever a buffer, tile list or record changes) */
    struct Graph {
        const void *tiles;
        crt_renderer_settings st;
        const float *out;
        hipStream_t stream;
        const void *scene;
        hipGraphExec_t exec;
    };
    std::vector<Graph> graphs;
};

void wf_graphs_clear(WfBuffers &w) {
    for (auto &g : w.graphs) (void)hipGraphExecDestroy(g.exec);
    w.graphs.clear();
}

/* Deepest recursion the wavefront path accepts (levels are launched one by one). */
constexpr int kWfMaxDepth = 4096;

struct crt_hip_scene {
    int device = 0;
    crt_scene_info info{};
    bool has_secondary = false;    /* any reflective / refractive material */
    bool has_diffuse = false;
    bool has_refractive = false;   /* Fresnel term: needs the powf table (fresnel_of) */
    DeviceScene ds{};
    DeviceScene ds_uploaded{};   /* what d_ds holds */
    DeviceScene *d_ds = nullptr;
    crt_wave_counts wave_counts{};   /* from the last crt_hip_count_work */
    std::vector<void *> allocs;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    ShardPlan full;
    std::map<std::pair<int, int>, ShardPlan> shard_plans;
    std::map<int, std::pair<UnpackBucket *, int>> unpack_plans;
    /* compact shards (crt_hip_*_compact): live-pixel mask of the frame (host),
     * per-(shard, count) render plans, per-count unpack lists */
    std::vector<uint8_t> live_mask;
    std::map<std::pair<int, int>, ShardPlan> compact_plans;
    std::map<int, std::pair<UnpackBucket *, int>> compact_unpack;
    float *d_out = nullptr;
    unsigned long long *d_counters = nullptr;
    int32_t *d_next_px = nullptr;      /* pixel-refill list head (k_render_refill) */
    int gi_refill = 1;                 /* GI frames: persistent waves with pixel refill (env CRT_GI_REFILL, option "gi_refill") */
    int gi_machine = 1;                /* ... as per-lane state machines (k_render_gi; option "gi_machine") */
    int gi_blocks = 1024;              /* blocks of the k_render_gi grid (resident blocks per CU x CUs) */
    void *gi_frames = nullptr;         /* k_render_gi: frames below the LDS ones (grown on demand) */
    int64_t gi_frames_bytes = 0;
    int refill_waves = 5120;           /* waves of the refill grid: CUs x 4 SIMDs x CRT_GI_WAVES */
    bool grid_empty = false;
    int traversal = 8;             /* 7 reference order | 8 pruned (default), see trace<> (env CRT_TRAVERSAL) */
    int shadows = 0;               /* option "shadows": trace the shadow rays (k_render_tiles<..., SHADOW>) */
    int trace_walk = 1;            /* crt_hip_trace_batch: 0 reference-order walk, 1 pruned per-lane walk */
    bool camera_fast = false;      /* every camera ray takes the fast box path (camera_rays_fast) */
    /* estimate plan (no calibration): a tile is split into 4x4 (2x2) pixel
     * waves when its work estimate exceeds split4 (split16) times the mean work
     * per resident wave slot, i.e. when it would run for several times the
     * ideal makespan */
    float split4 = 4.5f, split16 = 9.0f;
    int wave_slots = 6144;   /* CUs x 4 SIMDs x 6 resident render waves */
    int secondary = 0;       /* walk for secondary rays: 0 = by frame, 4, 10 (env CRT_SECONDARY) */
    std::vector<float> tile_work;  /* per 8x8 tile of the full frame */
    /* measured-cost tile plan (calibrate_plan): per 8x8 tile of the full frame,
     * the sub-tiles it is split into and their probed costs */
    struct SubTile { int32_t dx, dy, w, h; float cost; };
    std::vector<std::vector<SubTile>> calib;
    int calib_walk = -1;           /* primary walk the calibration was measured with (-1: none) */
    int calibrate = 1;             /* 0 estimate plan, 1 measured costs with a tuned k, 2 with calib_k (env CRT_CALIBRATE) */
    int window_walk = 1;           /* camera walk 12 -> 13 (window walk for split tiles), env CRT_WINDOW */
    int record_events = 1;         /* start/stop events around every render (crt_hip_last_kernel_ms), option "events" */
    bool events_valid = false;
    float calib_k = 4.0f;          /* split a wave whose cost exceeds k x (total cost / wave slots) (env CRT_CALIB_K) */
    int calib_min = 2;             /* smallest sub-tile side */
    int prio_tiles = 1024;         /* heaviest tiles run at raised issue priority */
    float prio_min = 2.0f;         /* ... if they cost more than this x the mean per wave slot */
    std::vector<void *> plan_allocs;   /* tile lists of the current plans */
    /* the tree in the reference's numbering (crt_hip_scene_tree): host copies
     * for a host-built tree, device arrays for a device-built one */
    std::vector<float> ref_bounds;
    std::vector<int32_t> ref_children, ref_leaf_tris;
    std::vector<int64_t> ref_leaf_off;
    const float *dt_ref_bounds = nullptr;
    const int32_t *dt_ref_children = nullptr, *dt_ref_leaf_tris = nullptr;
    const int64_t *dt_ref_leaf_off = nullptr;
    int wavefront = 1;             /* level-by-level recursion when GI is off (env CRT_WAVEFRONT) */
    int wf_graph = 1;              /* recorded-size wavefront frames replayed from captured HIP graphs (option "wf_graph") */
    int wf_replay = 1;             /* wavefront frames after the first: 1 recorded level sizes, 0 read back every level,
                                    * 2 recorded sizes minus one (tests: forces the overflow path) (option "wf_replay") */
    int wf_rays_per_wave = 48;     /* cap on the rays per wave of wavefront levels >= 1 (each level takes
                                    * min(cap, max(8, n / 4096)), render_wavefront), coop walks (env CRT_WF_RPW,
                                    * option "wf_rpw"); fixed 48 / 32 / 16 / 64: 3.55 / 3.64 / 3.62 / 3.68 ms */
    WfBuffers wf;
};

namespace {

template <class T>
int upload(crt_hip_scene *sc, const std::vector<T> &v, const T **dst, size_t pad = 0) {
    /* pad: zeroed records after the data, so grouped reads past a run's end stay in bounds */
    *dst = nullptr;
    if (v.empty() && pad == 0) return CRT_OK;
    void *p = nullptr;
    const size_t bytes = (v.size() + pad) * sizeof(T);
    HIP_TRY(hipMalloc(&p, bytes));
    sc->allocs.push_back(p);
    if (pad) HIP_TRY(hipMemset(static_cast<char *>(p) + v.size() * sizeof(T), 0, pad * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    sc->info.device_bytes += (int64_t)bytes;
    *dst = static_cast<const T *>(p);
    return CRT_OK;
}

/* Every camera ray of the frame takes the fast box path of make_ray_rcp:
 * node planes and the camera origin inside the exact-division window, and
 * d = normalize(v R) with |d_i| <= 2^20 for every pixel.  v = (dx, dy, -1),
 * |dx| <= aspect tan(fov/2), |dy| <= tan(fov/2) (crt_camera.cpp:7-35): with R
 * finite and bounded, w = v R is finite; with sigma_min(R) >= |det R| /
 * |R|_F^2 far above the rounding of v R (and above 2^-50, so |w|^2 stays
 * normal), w cannot round to 0 — then each |d_i| = |w_i| / |w| <= 1. */
bool camera_rays_fast(const HostScene &hs, bool planes_ok) {
    if (!planes_ok) return false;
    for (int k = 0; k < 3; ++k)
        if (!coord_ok(hs.cam_loc[k])) return false;
    const double ta = std::fabs((double)hs.tan_half_fov), aa = std::fabs((double)hs.aspect) * ta;
    if (!std::isfinite(ta) || !std::isfinite(aa) || ta > 0x1p40 || aa > 0x1p40) return false;
    double R[9], fro = 0.0, mx = 0.0;
    for (int k = 0; k < 9; ++k) {
        R[k] = hs.cam_rot[k];
        if (!std::isfinite(R[k]) || std::fabs(R[k]) > 0x1p40) return false;
        fro += R[k] * R[k];
        mx = std::max(mx, std::fabs(R[k]));
    }
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (!(fro > 0.0)) return false;
    const double smin = std::fabs(det) / fro;
    return smin > 0x1p-50 && smin > 1e-4 * (2.0 + aa + ta) * mx;
}

int make_tile_plan(crt_hip_scene *sc, const std::vector<DBucket> &buckets, bool full_frame, ShardPlan &plan) {
    std::vector<Tile> tiles;
    const int W = sc->info.width;
    if (full_frame) {
        for (int y = 0; y < sc->info.height; y += 8)
            for (int x = 0; x < W; x += 8)
                tiles.push_back(Tile{x, y, std::min(8, W - x), std::min(8, sc->info.height - y),
                                     (int64_t)y * W + x, W, 0});
        plan.packed_pixels = (int64_t)W * sc->info.height;
    } else {
        int64_t total = 0;
        for (const DBucket &b : buckets) {
            for (int ty = 0; ty < b.h; ty += 8)
                for (int tx = 0; tx < b.w; tx += 8)
                    tiles.push_back(Tile{b.x + tx, b.y + ty, std::min(8, b.w - tx), std::min(8, b.h - ty),
                                         b.packed_offset + (int64_t)ty * b.w + tx, b.w, 0});
            total += (int64_t)b.w * b.h;
        }
        plan.packed_pixels = total;
    }
    if (!sc->calib.empty() && !tiles.empty()) {
        /* measured costs: split as calibrated, heaviest first */
        const int tx = (W + 7) / 8;
        std::vector<std::pair<float, Tile>> out;
        out.reserve(tiles.size() * 2);
        for (const Tile &t : tiles) {
            const size_t k = (size_t)(t.y / 8) * tx + t.x / 8;
            const auto &cal = sc->calib[k];
            const bool aligned = t.x % 8 == 0 && t.y % 8 == 0 && t.w == std::min(8, W - t.x) &&
                                 t.h == std::min(8, sc->info.height - t.y);
            if (aligned) {
                for (const auto &st : cal)
                    out.push_back({st.cost, Tile{t.x + st.dx, t.y + st.dy, st.w, st.h,
                                                 t.out_base + (int64_t)st.dy * t.out_stride + st.dx, t.out_stride, 0}});
            } else {   /* bucket grid not on the 8x8 grid: keep the tile, cost of its 8x8 cell */
                float c = 0.f;
                for (const auto &st : cal) c += st.cost;
                out.push_back({c, t});
            }
        }
        std::stable_sort(out.begin(), out.end(),
                         [](const std::pair<float, Tile> &a, const std::pair<float, Tile> &b) { return a.first > b.first; });
        tiles.clear();
        plan.cost.clear();
        for (const auto &e : out) {
            tiles.push_back(e.second);
            plan.cost.push_back(e.first);
        }
        /* issue priority for the heaviest waves, at most prio_tiles of them and
         * only those costing more than prio_min x the mean per wave slot */
        double csum = 0.0;
        for (float c : plan.cost) csum += c;
        const double slot_cost = csum / std::max(1, sc->wave_slots);
        for (size_t k = 0; k < tiles.size() && (int)k < sc->prio_tiles; ++k)
            tiles[k].prio = plan.cost[k] > sc->prio_min * slot_cost ? 1 : 0;
    } else if (!tiles.empty() && !sc->tile_work.empty()) {
        /* dispatch the expensive tiles first so the longest waves start at t=0;
         * with a sharing walk, split the heaviest tiles so each of their waves
         * carries fewer rays and the rest of its lanes help (4x4 or 2x2 pixels) */
        const int tx = (W + 7) / 8;
        auto work = [&](const Tile &t) { return sc->tile_work[(size_t)(t.y / 8) * tx + t.x / 8]; };
        double wsum = 0.0;
        for (const Tile &t : tiles) wsum += work(t);
        const float slot_work = (float)(wsum / sc->wave_slots);
        std::vector<Tile> split;
        if (slot_work > 0.f && (sc->split4 > 0.f || sc->split16 > 0.f)) {
            for (const Tile &t : tiles) {
                const float w = work(t) / slot_work;
                const int sub = (sc->split16 > 0.f && w >= sc->split16) ? 2 : (sc->split4 > 0.f && w >= sc->split4) ? 4 : 8;
                for (int yy = 0; yy < t.h; yy += sub)
                    for (int xx = 0; xx < t.w; xx += sub)
                        split.push_back(Tile{t.x + xx, t.y + yy, std::min(sub, t.w - xx), std::min(sub, t.h - yy),
                                             t.out_base + (int64_t)yy * t.out_stride + xx, t.out_stride, 0});
            }
            tiles.swap(split);
        }
        std::vector<std::pair<float, int>> key(tiles.size());
        for (size_t k = 0; k < tiles.size(); ++k) key[k] = {-work(tiles[k]), (int)k};
        std::stable_sort(key.begin(), key.end());
        std::vector<Tile> sorted(tiles.size());
        for (size_t k = 0; k < tiles.size(); ++k) sorted[k] = tiles[key[k].second];
        tiles.swap(sorted);
    }
    plan.ntiles = (int)tiles.size();
    plan.has_small = false;
    for (const Tile &t : tiles) plan.has_small = plan.has_small || t.w * t.h <= 16;
    plan.tiles = tiles;
    if (!tiles.empty()) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, tiles.size() * sizeof(Tile)));
        HIP_TRY(hipMemcpy(p, tiles.data(), tiles.size() * sizeof(Tile), hipMemcpyHostToDevice));
        sc->plan_allocs.push_back(p);
        plan.d_tiles = static_cast<Tile *>(p);
    }
    return CRT_OK;
}

/* Probe costs of a tile list (k_probe_tiles) with walk `walk`, synchronously. */
int probe_tiles(crt_hip_scene *sc, const DeviceScene *d_scene, int walk, const std::vector<Tile> &tiles,
                std::vector<uint32_t> &cost, hipStream_t stream) {
    cost.assign(tiles.size(), 0u);
    if (tiles.empty()) return CRT_OK;
    void *dt = nullptr, *dc = nullptr;
    HIP_TRY(hipMalloc(&dt, tiles.size() * sizeof(Tile)));
    hipError_t e = hipMalloc(&dc, tiles.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpyAsync(dt, tiles.data(), tiles.size() * sizeof(Tile), hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) {
        const int n = (int)tiles.size();
        const dim3 grid((unsigned)((n + 3) / 4));
        const Tile *t = static_cast<const Tile *>(dt);
        uint32_t *c = static_cast<uint32_t *>(dc);
        switch (walk) {
        case 7: hipLaunchKernelGGL(k_probe_tiles<7>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        case 12: hipLaunchKernelGGL(k_probe_tiles<12>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        case 13: hipLaunchKernelGGL(k_probe_tiles<13>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        default: hipLaunchKernelGGL(k_probe_tiles<8>, grid, dim3(256), 0, stream, d_scene, t, n, c); break;
        }
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(cost.data(), dc, tiles.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(dt);
    if (dc) (void)hipFree(dc);
    if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("tile probe: ") + hipGetErrorString(e));
    return CRT_OK;
}

/* Measured-cost tile plan.  The frame's 8x8 tiles are probed with the primary
 * walk; a tile whose wave cost exceeds k x (total cost / resident wave slots)
 * would run past the ideal makespan, so it is split into quadrants, which are
 * probed in turn, down to calib_min pixels.  The leaves and their costs give
 * every later plan (full frame and shards): split as measured, dispatched
 * heaviest first.  Results do not depend on the plan. */
int calibrate_plan(crt_hip_scene *sc, const DeviceScene *d_scene, int walk, hipStream_t stream) {
    const int W = sc->info.width, H = sc->info.height;
    const int tx = (W + 7) / 8, ty = (H + 7) / 8;
    struct Item { int k; int32_t dx, dy, w, h; };
    std::vector<Item> cur;
    cur.reserve((size_t)tx * ty);
    for (int y = 0; y < ty; ++y)
        for (int x = 0; x < tx; ++x)
            cur.push_back(Item{y * tx + x, 0, 0, std::min(8, W - 8 * x), std::min(8, H - 8 * y)});
    std::vector<std::vector<crt_hip_scene::SubTile>> cal((size_t)tx * ty);
    double thresh = -1.0;
    int side = 8;
    while (!cur.empty()) {
        std::vector<Tile> tl(cur.size());
        for (size_t i = 0; i < cur.size(); ++i) {
            const int x0 = 8 * (cur[i].k % tx) + cur[i].dx, y0 = 8 * (cur[i].k / tx) + cur[i].dy;
            tl[i] = Tile{x0, y0, cur[i].w, cur[i].h, (int64_t)y0 * W + x0, W, 0};
        }
        std::vector<uint32_t> cost;
        const int rc = probe_tiles(sc, d_scene, walk, tl, cost, stream);
        if (rc != CRT_OK) return rc;
        if (thresh < 0.0) {
            double sum = 0.0;
            for (uint32_t c : cost) sum += c;
            thresh = sc->calib_k * sum / std::max(1, sc->wave_slots);
        }
        std::vector<Item> next;
        const int half = side / 2;
        for (size_t i = 0; i < cur.size(); ++i) {
            const Item &it = cur[i];
            if ((double)cost[i] > thresh && half >= sc->calib_min && (it.w > half || it.h > half)) {
                for (int yy = 0; yy < it.h; yy += half)
                    for (int xx = 0; xx < it.w; xx += half)
                        next.push_back(Item{it.k, it.dx + xx, it.dy + yy, std::min(half, it.w - xx), std::min(half, it.h - yy)});
            } else {
                cal[it.k].push_back(crt_hip_scene::SubTile{it.dx, it.dy, it.w, it.h, (float)cost[i]});
            }
        }
        cur.swap(next);
        side = half;
    }
    sc->calib.swap(cal);
    sc->calib_walk = walk;
    return CRT_OK;
}

void free_plans(crt_hip_scene *sc) {
    for (void *p : sc->plan_allocs) (void)hipFree(p);
    sc->plan_allocs.clear();
    sc->wf.recs.clear();   /* keyed by the tile lists' device pointers */
    wf_graphs_clear(sc->wf);
    sc->full = ShardPlan{};
    sc->shard_plans.clear();
    sc->compact_plans.clear();
}

/* powf(x, 5.0f) for x = k * 2^-24, k = -2^24 .. 2^24 (fresnel_of), computed
 * by this process's libm — the one the reference's std::pow resolves to on
 * this host.  Called through a volatile pointer so the compiler cannot
 * replace the libm call by its own expansion. */
constexpr int64_t kPow5N = (int64_t(1) << 25) + 1;
std::mutex g_pow5_mu;
std::map<int, float *> g_pow5;             /* per device, process lifetime */
std::vector<float> g_pow5_host;

void build_pow5_host_table() {
    if (!g_pow5_host.empty()) return;
    g_pow5_host.resize((size_t)kPow5N);
    float *t = g_pow5_host.data();
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < nt; ++w) {
        pool.emplace_back([=]() {
            float (*volatile pw)(float, float) = ::powf;
            for (int64_t k = w; k < kPow5N; k += nt) {
                const float x = (float)(k - (int64_t(1) << 24)) * (1.0f / 16777216.0f);   /* exact */
                t[k] = pw(x, 5.0f);
            }
        });
    }
    for (auto &th : pool) th.join();
}

int ensure_pow5_table(crt_hip_scene *sc) {
    if (sc->ds.pow5) return CRT_OK;
    std::lock_guard<std::mutex> g(g_pow5_mu);
    float *&d = g_pow5[sc->device];
    if (!d) {
        build_pow5_host_table();
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)kPow5N * sizeof(float)));
        HIP_TRY(hipMemcpy(p, g_pow5_host.data(), (size_t)kPow5N * sizeof(float), hipMemcpyHostToDevice));
        d = static_cast<float *>(p);
    }
    sc->ds.pow5 = d;
    return CRT_OK;
}

int ensure_gi_tables(crt_hip_scene *sc) {
    if (sc->ds.gi_pi) return CRT_OK;
    std::lock_guard<std::mutex> g(g_gi_mu);
    GiTables &t = g_gi[sc->device];
    if (!t.d) {
        build_gi_host_tables();
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)(4 * kGiN) * sizeof(float)));
        HIP_TRY(hipMemcpy(p, g_gi_host.data(), (size_t)(4 * kGiN) * sizeof(float), hipMemcpyHostToDevice));
        t.d = static_cast<float *>(p);
    }
    sc->ds.gi_pi = t.d;
    sc->ds.gi_2pi = t.d + 2 * kGiN;
    return CRT_OK;
}

/* Device copy of sc->ds for the render kernels.  Re-uploaded only when the
 * host record changed (first GI frame, new resolution); kernels of earlier
 * frames may still read the old copy, so the device is drained first. */
int sync_device_record(crt_hip_scene *sc, const DeviceScene **out) {
    if (!sc->d_ds || std::memcmp(&sc->ds_uploaded, &sc->ds, sizeof(DeviceScene)) != 0) {
        if (!sc->d_ds) {
            void *p = nullptr;
            HIP_TRY(hipMalloc(&p, sizeof(DeviceScene)));
            sc->allocs.push_back(p);
            sc->d_ds = static_cast<DeviceScene *>(p);
        } else {
            HIP_TRY(hipDeviceSynchronize());
        }
        HIP_TRY(hipMemcpy(sc->d_ds, &sc->ds, sizeof(DeviceScene), hipMemcpyHostToDevice));
        std::memcpy(&sc->ds_uploaded, &sc->ds, sizeof(DeviceScene));
    }
    *out = sc->d_ds;
    return CRT_OK;
}

int check_settings(const crt_renderer_settings *st) {
    if (!st) return set_error(CRT_E_INVALID, "null settings");
    return CRT_OK;
}

/* The packet walk camera rays take: walk 8 becomes its fast-only build 12
 * when the host has proven every camera ray fast. */
int camera_walk(const crt_hip_scene *sc, int trav) {
    return (trav == 8 && sc->camera_fast) ? (sc->window_walk ? 13 : 12) : trav;
}

/* The primary walk a tile plan is measured with (-1: keep the estimate plan):
 * camera rays of diffuse frames and level 0 of the wavefront recursion. */
int plan_walk(const crt_hip_scene *sc, const crt_renderer_settings *st) {
    const bool gi = sc->info.gi_on && sc->has_diffuse && st->diffuse_reflection_ray_count > 0;
    const bool full = gi || sc->has_secondary;
    if (gi) return -1;
    if (full) return sc->wavefront ? camera_walk(sc, sc->traversal == 8 ? 8 : 7) : -1;
    return camera_walk(sc, sc->traversal);
}

/* Calibrate the tile plan for this frame's primary walk once (see
 * calibrate_plan), then rebuild the full-frame plan; shard plans are rebuilt
 * on their next use. */
/* Split threshold of the calibrated plan (calibrate_plan: a tile whose
 * measured cost exceeds k x mean cost per wave slot is split).  The best k
 * depends on the scene and on how the walks' step counts relate to time (a
 * split tile's window waves cost more per step than a packet wave), so by
 * default it is tuned: each candidate's plan renders the frame (one untimed,
 * five timed launches, median taken) and the fastest plan is kept.  Only the
 * tiling changes with k; every plan produces the same image bits.
 * calibrate = 2 (or env CRT_CALIB_K) keeps the given k instead.  The grid
 * is fine around 2-3: C2's frame moves by 5-10 % between neighbouring k. */
static const float kCalibK[] = {1.5f, 1.75f, 2.0f, 2.25f, 2.5f, 2.75f, 3.0f, 3.5f, 4.0f, 6.0f};

int launch_render(crt_hip_scene *sc, const crt_renderer_settings *st, const ShardPlan &plan, float *d_out,
                  hipStream_t stream, bool count, unsigned long long *stamps = nullptr);
bool wf_overflowed(WfBuffers &w, bool wait);

int ensure_plans(crt_hip_scene *sc, const crt_renderer_settings *st, hipStream_t stream) {
    if (!sc->calibrate || sc->grid_empty) return CRT_OK;
    const int walk = plan_walk(sc, st);
    if (walk < 0 || walk == sc->calib_walk) return CRT_OK;
    const DeviceScene *d_scene = nullptr;
    int rc = sync_device_record(sc, &d_scene);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());   /* earlier frames may still read the old tile lists */
    int64_t px = 0;
    const std::vector<DBucket> all = shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, 0, 1, &px);
    if (sc->calibrate == 2) {
        if ((rc = calibrate_plan(sc, d_scene, walk, stream)) != CRT_OK) return rc;
        free_plans(sc);
        return make_tile_plan(sc, all, true, sc->full);
    }
    float *scratch = nullptr;
    HIP_TRY(hipMalloc(&scratch, (size_t)sc->info.width * sc->info.height * 3 * sizeof(float)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float best_ms = INFINITY, best_k = kCalibK[0];
    std::vector<std::vector<crt_hip_scene::SubTile>> best_cal;
    auto tune = [&]() -> int {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        for (const float k : kCalibK) {
            sc->calib_k = k;
            int r = calibrate_plan(sc, d_scene, walk, stream);
            if (r != CRT_OK) return r;
            free_plans(sc);
            if ((r = make_tile_plan(sc, all, true, sc->full)) != CRT_OK) return r;
            std::vector<float> reps;
            for (int rep = 0; rep < 6; ++rep) {
                HIP_TRY(hipEventRecord(e0, stream));
                if ((r = launch_render(sc, st, sc->full, scratch, stream, false)) != CRT_OK) return r;
                HIP_TRY(hipEventRecord(e1, stream));
                HIP_TRY(hipEventSynchronize(e1));
                (void)wf_overflowed(sc->wf, true);   /* a wrong trial frame only drops the recorded level sizes */
                float t = 0.f;
                HIP_TRY(hipEventElapsedTime(&t, e0, e1));
                if (rep > 0) reps.push_back(t);
            }
            std::sort(reps.begin(), reps.end());
            const float ms = reps[reps.size() / 2];   /* median of 5 timed frames */
            if (ms < best_ms) {
                best_ms = ms;
                best_k = k;
                best_cal = sc->calib;
            }
        }
        return CRT_OK;
    };
    rc = tune();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(scratch);
    if (rc != CRT_OK) return rc;
    sc->calib_k = best_k;
    sc->calib.swap(best_cal);
    sc->calib_walk = walk;
    free_plans(sc);
    return make_tile_plan(sc, all, true, sc->full);
}

DSettings to_dsettings(const crt_renderer_settings *st) {
    DSettings d;
    d.max_ray_depth = st->max_ray_depth;
    d.diffuse_reflection_ray_count = st->diffuse_reflection_ray_count;
    d.shadow_bias = st->shadow_bias;
    d.reflection_bias = st->reflection_bias;
    d.diffuse_reflection_bias = st->diffuse_reflection_bias;
    d.refraction_bias = st->refraction_bias;
    return d;
}

int wf_grow_ids(WfBuffers &w, int64_t need, int64_t used, hipStream_t stream) {
    if (need <= w.cap) return CRT_OK;
    wf_graphs_clear(w);
    const int64_t cap = std::max<int64_t>(need, 2 * w.cap);
    void *pn = nullptr, *pc = nullptr;
    HIP_TRY(hipMalloc(&pn, (size_t)cap * sizeof(WNode)));
    HIP_TRY(hipMalloc(&pc, (size_t)cap * sizeof(DVec4)));
    if (used > 0) {
        HIP_TRY(hipMemcpyAsync(pn, w.nodes, (size_t)used * sizeof(WNode), hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipMemcpyAsync(pc, w.cols, (size_t)used * sizeof(DVec4), hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));
    }
    if (w.nodes) (void)hipFree(w.nodes);
    if (w.cols) (void)hipFree(w.cols);
    w.nodes = static_cast<WNode *>(pn);
    w.cols = static_cast<DVec4 *>(pc);
    w.cap = cap;
    return CRT_OK;
}

int wf_grow_queue(WfBuffers &w, int k, int64_t need) {
    if (need <= w.qcap[k]) return CRT_OK;
    wf_graphs_clear(w);
    const int64_t cap = std::max<int64_t>(need, 2 * w.qcap[k]);
    if (w.q[k]) (void)hipFree(w.q[k]);
    w.q[k] = nullptr;
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)cap * sizeof(WRay)));
    w.q[k] = static_cast<WRay *>(p);
    w.qcap[k] = cap;
    return CRT_OK;
}

void wf_free(WfBuffers &w) {
    wf_graphs_clear(w);
    for (void *p : {(void *)w.nodes, (void *)w.cols, (void *)w.q[0], (void *)w.q[1], (void *)w.counts, (void *)w.d_flag})
        if (p) (void)hipFree(p);
    if (w.h_flag) (void)hipHostFree(w.h_flag);
    if (w.flag_ev) (void)hipEventDestroy(w.flag_ev);
    w = WfBuffers{};
}

/* The last recorded-size frame's overflow flag, if its copy has landed
 * (wait: block until it has).  Returns true when that frame overflowed; the
 * recorded sizes are then dropped, so the next frame reads its sizes back. */
bool wf_overflowed(WfBuffers &w, bool wait) {
    if (!w.flag_pending) return false;
    if (wait) {
        if (hipEventSynchronize(w.flag_ev) != hipSuccess) return false;
    } else if (hipEventQuery(w.flag_ev) != hipSuccess) {
        return false;
    }
    w.flag_pending = false;
    if (*w.h_flag == 0) return false;
    /* consumed: frames still in flight were queued with the same stale sizes
     * and are covered by this report; re-arm the device flag behind them */
    (void)hipDeviceSynchronize();
    (void)hipMemset(w.d_flag, 0, sizeof(int32_t));
    *w.h_flag = 0;
    w.recs.clear();
    wf_graphs_clear(w);
    return true;
}

/* One frame of the wavefront path (see k_wf_level).  A level's size is
 * known only once the level before it has run, so the first frame of a
 * (settings, tile list) reads each level's queue length back before launching
 * the next level (one host sync per level) and records the sizes.  The sizes
 * are a function of the frame's rays alone, so every later frame with the same
 * key launches all levels back to back with the recorded sizes, no host sync:
 * each level may queue exactly the recorded size of the next, and a level
 * that would queue more sets an overflow flag instead (checked behind the
 * frame: crt_hip_render re-renders that frame with read-backs, the device-side
 * entry points report it on the next call). */
int render_wavefront(crt_hip_scene *sc, const DSettings &ds, const crt_renderer_settings *st, const ShardPlan &plan,
                     float *d_out, hipStream_t stream, bool count, const DeviceScene *d_scene, int sec, int primary) {
    WfBuffers &w = sc->wf;
    /* levels 0..max_ray_depth are traced (a child deeper than max_ray_depth is
     * never queued, crt_renderer.cpp:47-48), so the loop below always drains
     * the queue: counts[max_ray_depth] is written by nobody and stays 0 */
    if (ds.max_ray_depth > (uint32_t)kWfMaxDepth)
        return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > " + std::to_string(kWfMaxDepth) +
                                                " with reflective/refractive materials is not supported");
    if (wf_overflowed(w, false))
        return set_error(CRT_E_STATE, "a wavefront level outgrew its recorded size in the previous frame; "
                                         "that frame is wrong (sizes are now read back again)");
    const int kMaxLevels = (int)ds.max_ray_depth + 2;
    if (!w.counts || w.count_cap < kMaxLevels) {
        if (w.counts) (void)hipFree(w.counts);
        w.counts = nullptr;
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, (size_t)kMaxLevels * sizeof(int32_t)));
        w.counts = static_cast<int32_t *>(p);
        w.count_cap = kMaxLevels;
        wf_graphs_clear(w);
    }
    if (!w.d_flag) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, sizeof(int32_t)));
        w.d_flag = static_cast<int32_t *>(p);
        HIP_TRY(hipMemsetAsync(w.d_flag, 0, sizeof(int32_t), stream));
        HIP_TRY(hipHostMalloc(&p, sizeof(int32_t), hipHostMallocDefault));
        w.h_flag = static_cast<int32_t *>(p);
        *w.h_flag = 0;
        HIP_TRY(hipEventCreateWithFlags(&w.flag_ev, hipEventDisableTiming));
    }
    const int64_t n0 = (int64_t)plan.ntiles * 64;
    const auto rit = w.recs.find((const void *)plan.d_tiles);
    const bool replay = !count && sc->wf_replay && rit != w.recs.end() && rit->second.ntiles == plan.ntiles &&
                        std::memcmp(&rit->second.st, st, sizeof *st) == 0;
    static const std::vector<int32_t> kNone;
    const std::vector<int32_t> &rec = replay ? rit->second.sizes : kNone;
    int rc;
    int64_t qneed = 2 * n0, ids = 3 * n0;
    if (replay) {
        int64_t tot = n0, mx = 0;
        for (int32_t n : rec) {
            tot += n;
            mx = std::max<int64_t>(mx, n);
        }
        qneed = std::max<int64_t>(mx, 1);
        ids = tot;
    }
    if ((rc = wf_grow_ids(w, ids, 0, stream)) != CRT_OK) return rc;
    if ((rc = wf_grow_queue(w, 0, qneed)) != CRT_OK) return rc;
    if (replay && (rc = wf_grow_queue(w, 1, qneed)) != CRT_OK) return rc;
    /* a recorded-size frame is a fixed launch sequence: replayed from a HIP
     * graph captured the first time (one launch instead of ~2 per level) */
    if (replay && sc->wf_graph) {
        for (const auto &g : w.graphs)
            if (g.tiles == (const void *)plan.d_tiles && g.out == d_out && g.stream == stream &&
                g.scene == (const void *)d_scene && std::memcmp(&g.st, st, sizeof *st) == 0) {
                HIP_TRY(hipGraphLaunch(g.exec, stream));
                HIP_TRY(hipEventRecord(w.flag_ev, stream));
                w.flag_pending = true;
                return CRT_OK;
            }
    }
    const bool capture = replay && sc->wf_graph;
    if (capture) HIP_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    auto cap_of = [](int64_t c) { return (int32_t)std::min<int64_t>(c, INT32_MAX); };
    std::vector<int32_t> sizes;
    auto enqueue = [&]() -> int {
    HIP_TRY(hipMemsetAsync(w.counts, 0, kMaxLevels * sizeof(int32_t), stream));
    unsigned long long *cnt = sc->d_counters;
    WLevel lv{nullptr, 0, 0, w.q[0], w.counts, (int32_t)n0, w.nodes, w.cols, 64,
              replay ? (rec.empty() ? 0 : rec[0]) : cap_of(w.qcap[0]), w.d_flag};
    const int blocks0 = (plan.ntiles + 3) / 4;
#define CRT_WF0(T, COUNT)                                                                                   \
    hipLaunchKernelGGL((k_wf_level<T, true, COUNT>), dim3(blocks0), dim3(256), 0, stream, d_scene, ds,      \
                       plan.d_tiles, plan.ntiles, lv, cnt)
    if (primary == 12 || primary == 13) {   /* level 0 keeps 8x8 tiles' packet walk (no window build) */
        if (count) CRT_WF0(12, true); else CRT_WF0(12, false);
    } else if (primary == 8) {
        if (count) CRT_WF0(8, true); else CRT_WF0(8, false);
    } else {
        if (count) CRT_WF0(7, true); else CRT_WF0(7, false);
    }
#undef CRT_WF0
    HIP_TRY(hipGetLastError());
    std::vector<std::pair<int64_t, int64_t>> levels;   /* (first id, count) of levels >= 1 */
    int64_t base = n0;
    int cur = 0;
    const int rpw = std::min(64, std::max(1, sc->wf_rays_per_wave));   /* coop walks: idle lanes take donated pieces */
    for (int L = 1; L < kMaxLevels; ++L) {
        int32_t n = 0;
        int32_t out_cap = 0;
        if (replay) {
            if (L - 1 >= (int)rec.size()) break;
            n = rec[L - 1];
            out_cap = L < (int)rec.size() ? rec[L] : 0;
        } else {
            HIP_TRY(hipMemcpyAsync(&n, w.counts + (L - 1), sizeof n, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            if (n == 0) break;
            if (base + 3 * (int64_t)n > INT32_MAX) return set_error(CRT_E_UNSUPPORTED, "wavefront ray ids exceed 2^31");
            if ((rc = wf_grow_ids(w, base + 3 * (int64_t)n, base, stream)) != CRT_OK) return rc;
            if ((rc = wf_grow_queue(w, cur ^ 1, 2 * (int64_t)n)) != CRT_OK) return rc;
            out_cap = cap_of(w.qcap[cur ^ 1]);
            sizes.push_back(n);
        }
        /* rays per wave of this level: fewer (more helper lanes per ray) when
         * the level has fewer rays than ~4096 waves' worth, at least 8, at most
         * the wf_rpw cap — a level's time is its slowest waves'
         * (C3 3.60 -> 3.33 ms, profiles/r02/ab_c3_rpw) */
        const int rpw_l = sec == 14 ? 64 : std::min(rpw, std::max(8, (int)((n + 4095) / 4096)));
        WLevel l{w.q[cur], n, L, w.q[cur ^ 1], w.counts + L, (int32_t)(base + n), w.nodes, w.cols, rpw_l, out_cap,
                 w.d_flag};
        const int64_t waves = ((int64_t)n + rpw_l - 1) / rpw_l;
        const int blocks = (int)((waves + 3) / 4);
#define CRT_WF(SEC, COUNT)                                                                                  \
    hipLaunchKernelGGL((k_wf_level<SEC, false, COUNT>), dim3(blocks), dim3(256), 0, stream, d_scene, ds,     \
                       plan.d_tiles, plan.ntiles, l, cnt)
        if (sec == 14) {
            if (count) CRT_WF(14, true); else CRT_WF(14, false);
        } else if (sec == 10) {
            if (count) CRT_WF(10, true); else CRT_WF(10, false);
        } else {
            if (count) CRT_WF(4, true); else CRT_WF(4, false);
        }
#undef CRT_WF
        HIP_TRY(hipGetLastError());
        levels.emplace_back(base, n);
        base += n;
        cur ^= 1;
    }
    for (auto it = levels.rbegin(); it != levels.rend(); ++it)
        hipLaunchKernelGGL(k_wf_compose, dim3((unsigned)((it->second + 255) / 256)), dim3(256), 0, stream, w.nodes,
                           w.cols, (int32_t)it->first, (int32_t)it->second);
    hipLaunchKernelGGL(k_wf_pixels, dim3(blocks0), dim3(256), 0, stream, w.nodes, w.cols, plan.d_tiles,
                       plan.ntiles, d_out);
    HIP_TRY(hipGetLastError());
    if (replay)   /* the device flag is sticky: a later frame's copy cannot hide an earlier overflow */
        HIP_TRY(hipMemcpyAsync(w.h_flag, w.d_flag, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    return CRT_OK;
    };
    rc = enqueue();
    if (capture) {
        hipGraph_t graph = nullptr;
        const hipError_t e = hipStreamEndCapture(stream, &graph);
        if (rc != CRT_OK) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        hipGraphExec_t exec = nullptr;
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_error(CRT_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
        w.graphs.push_back(WfBuffers::Graph{(const void *)plan.d_tiles, *st, d_out, stream, (const void *)d_scene, exec});
        HIP_TRY(hipGraphLaunch(exec, stream));
    } else if (rc != CRT_OK) {
        return rc;
    }
    if (replay) {
        HIP_TRY(hipEventRecord(w.flag_ev, stream));
        w.flag_pending = true;
    } else if (!count && sc->wf_replay) {
        WfBuffers::Rec &r = w.recs[(const void *)plan.d_tiles];
        if (sc->wf_replay == 2)
            for (int32_t &n : sizes) n = n > 1 ? n - 1 : n;
        r.sizes.swap(sizes);
        r.st = *st;
        r.ntiles = plan.ntiles;
    }
    return CRT_OK;
}

/* Pick and launch the kernel variant for this scene + settings. */
int launch_render(crt_hip_scene *sc, const crt_renderer_settings *st, const ShardPlan &plan, float *d_out,
                  hipStream_t stream, bool count, unsigned long long *stamps) {
    const bool gi = sc->info.gi_on && sc->has_diffuse && st->diffuse_reflection_ray_count > 0;
    const bool full = gi || sc->has_secondary;
    if (gi) {
        const int rc = ensure_gi_tables(sc);
        if (rc != CRT_OK) return rc;
    }
    if (sc->has_refractive && sc->info.refractions_on) {
        const int rc = ensure_pow5_table(sc);
        if (rc != CRT_OK) return rc;
    }
    if (plan.ntiles == 0) return CRT_OK;
    const DeviceScene *d_scene = nullptr;
    {
        const int rc = sync_device_record(sc, &d_scene);
        if (rc != CRT_OK) return rc;
    }
    const DSettings ds = to_dsettings(st);
    /* Walks: camera rays take the packet walk (traversal 7, or 8 pruned).
     * Secondary rays scatter and take the cooperative walk: pruned (10) for
     * reflect/refract levels (C3), reference order (4) for GI fan-out — the
     * pruned form needs 134 VGPRs (3 waves/SIMD) and loses on C4 (378 vs 320
     * ms); with GI every ray of the per-lane frame-stack kernel takes that walk
     * (the packet walk's registers would cost a wave per SIMD).
     * CRT_SECONDARY / "secondary" overrides the secondary walk. */
    const bool pruned = sc->traversal == 8;
    int sec = sc->secondary;
    if (sec == 14 && !sc->ds.bnodes) sec = 10;   /* no BVH (device-built tree) */
    if (sec == 0) sec = !pruned ? 4 : sc->ds.bnodes ? 14 : gi ? 4 : 10;
    if (sc->shadows) {
        /* shadow-ray frames (option "shadows"): frame-stack kernel, pruned
         * cooperative walk for every traced ray, per-lane shadow walks */
        if (stamps) return set_error(CRT_E_UNSUPPORTED, "wave profiles of shadow-ray frames are not supported");
        const uint64_t nf = (uint64_t)st->max_ray_depth + 1;
        const int nb = (plan.ntiles + 3) / 4;
        unsigned long long *cn = sc->d_counters;
        if (!full) {   /* no recursion: the frame's camera walk, packet walks for shadow rays (shade_hit_shadowed) */
            int tr = camera_walk(sc, sc->traversal);
            if (tr == 13 && !plan.has_small) tr = 12;
#define CRT_LAUNCH_SH(TR, COUNT)                                                                            \
    hipLaunchKernelGGL((k_render_tiles<false, 0, TR, TR, COUNT, true>), dim3(nb), dim3(256), 0, stream, d_scene, ds, \
                       plan.d_tiles, plan.ntiles, d_out, cn, nullptr)
            if (tr == 13) {
                if (count) CRT_LAUNCH_SH(13, true); else CRT_LAUNCH_SH(13, false);
            } else if (tr == 12) {
                if (count) CRT_LAUNCH_SH(12, true); else CRT_LAUNCH_SH(12, false);
            } else {
                if (count) CRT_LAUNCH_SH(8, true); else CRT_LAUNCH_SH(8, false);
            }
#undef CRT_LAUNCH_SH
            HIP_TRY(hipGetLastError());
            return CRT_OK;
        }
#define CRT_LAUNCH_S(MAXF, COUNT)                                                                           \
    hipLaunchKernelGGL((k_render_tiles<true, MAXF, 10, 10, COUNT, true>), dim3(nb), dim3(256), 0, stream,      \
                       d_scene, ds, plan.d_tiles, plan.ntiles, d_out, cn, nullptr)
        if (nf <= 4) {
            if (count) CRT_LAUNCH_S(4, true); else CRT_LAUNCH_S(4, false);
        } else if (nf <= 16) {
            if (count) CRT_LAUNCH_S(16, true); else CRT_LAUNCH_S(16, false);
        } else if (nf <= 64) {
            if (count) CRT_LAUNCH_S(64, true); else CRT_LAUNCH_S(64, false);
        } else {
            return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > 63 with shadow rays is not supported");
        }
#undef CRT_LAUNCH_S
        HIP_TRY(hipGetLastError());
        return CRT_OK;
    }
    if (full && !gi && sc->wavefront && !stamps)
        return render_wavefront(sc, ds, st, plan, d_out, stream, count, d_scene, sec, camera_walk(sc, sc->traversal));
    /* frame-stack kernel: one walk for every ray */
    int trav = full ? sec : camera_walk(sc, sc->traversal);
    if (trav == 13 && !plan.has_small) trav = 12;   /* no split tiles: the leaner packet-only kernel */
    const int blocks = (plan.ntiles + 3) / 4;
    const uint64_t frames = (uint64_t)st->max_ray_depth + 1;
    unsigned long long *cnt = sc->d_counters;
#define CRT_LAUNCH_T(FULL, MAXF, TRAV, COUNT)                                                               \
    hipLaunchKernelGGL((k_render_tiles<FULL, MAXF, TRAV, TRAV, COUNT>), dim3(blocks), dim3(256), 0, stream,      \
                       d_scene, ds, plan.d_tiles, plan.ntiles, d_out, cnt, stamps)
#define CRT_LAUNCH(MAXF, COUNT)                                                                             \
    do {                                                                                                   \
        if (trav == 10 || trav == 14) CRT_LAUNCH_T(true, MAXF, 10, COUNT);                                  \
        else CRT_LAUNCH_T(true, MAXF, 4, COUNT);                                                           \
    } while (0)
    if (!full) {
        switch (trav) {
        case 7: if (count) CRT_LAUNCH_T(false, 0, 7, true); else CRT_LAUNCH_T(false, 0, 7, false); break;
        case 8: if (count) CRT_LAUNCH_T(false, 0, 8, true); else CRT_LAUNCH_T(false, 0, 8, false); break;
        case 12: if (count) CRT_LAUNCH_T(false, 0, 12, true); else CRT_LAUNCH_T(false, 0, 12, false); break;
        case 13: if (count) CRT_LAUNCH_T(false, 0, 13, true); else CRT_LAUNCH_T(false, 0, 13, false); break;
        default: return set_error(CRT_E_INVALID, "no such camera walk");
        }
    } else if (gi && (trav == 4 || trav == 10 || trav == 14) && sc->gi_refill && sc->d_next_px && !stamps && frames <= 64) {
        /* GI: persistent waves with pixel refill (k_render_refill) */
        HIP_TRY(hipMemsetAsync(sc->d_next_px, 0, sizeof(int32_t), stream));
        const int nw = std::max(1, std::min(plan.ntiles, sc->refill_waves));
        const unsigned rb = (unsigned)((nw + 3) / 4);
#define CRT_REFILL_T(MAXF, T, COUNT)                                                                        \
    hipLaunchKernelGGL((k_render_refill<MAXF, T, COUNT>), dim3(rb), dim3(256), 0, stream, d_scene, ds,       \
                       plan.d_tiles, plan.ntiles, d_out, sc->d_next_px, cnt)
#define CRT_REFILL(MAXF, COUNT) CRT_REFILL_T(MAXF, 4, COUNT)
        if (trav == 14 && sc->gi_machine && (uint64_t)st->diffuse_reflection_ray_count < (1ull << 29) &&
            (int64_t)sc->info.width * sc->info.height < INT32_MAX) {
            /* per-lane state machine over the BVH walk (crt_gi_machine.h) */
            const unsigned gb = (unsigned)std::max(1, std::min((plan.ntiles + 3) / 4, sc->gi_blocks));
            /* frames below the two LDS ones and the register one: 64 B per lane and depth */
            const int64_t gneed = (int64_t)gb * 256 * std::max<int64_t>(0, (int64_t)st->max_ray_depth - 3) * 64;
            if (gneed > sc->gi_frames_bytes) {
                HIP_TRY(hipStreamSynchronize(stream));
                if (sc->gi_frames) (void)hipFree(sc->gi_frames);
                sc->gi_frames = nullptr;
                sc->gi_frames_bytes = 0;
                HIP_TRY(hipMalloc(&sc->gi_frames, (size_t)gneed));
                sc->gi_frames_bytes = gneed;
            }
            float4 *gf = static_cast<float4 *>(sc->gi_frames);
            if (count)
                hipLaunchKernelGGL((k_render_gi<true>), dim3(gb), dim3(256), 0, stream, d_scene, ds, plan.d_tiles,
                                   plan.ntiles, d_out, sc->d_next_px, cnt, gf);
            else
                hipLaunchKernelGGL((k_render_gi<false>), dim3(gb), dim3(256), 0, stream, d_scene, ds, plan.d_tiles,
                                   plan.ntiles, d_out, sc->d_next_px, cnt, gf);
        } else if (trav == 14) {                   /* per-lane BVH walk (crt_bvh.h) */
            if (frames <= 4) {
                if (count) CRT_REFILL_T(4, 14, true); else CRT_REFILL_T(4, 14, false);
            } else if (frames <= 16) {
                if (count) CRT_REFILL_T(16, 14, true); else CRT_REFILL_T(16, 14, false);
            } else {
                if (count) CRT_REFILL_T(64, 14, true); else CRT_REFILL_T(64, 14, false);
            }
        } else if (frames <= 4 && trav == 10) {   /* pruned cooperative walk for GI (secondary = 10) */
            if (count) CRT_REFILL_T(4, 10, true); else CRT_REFILL_T(4, 10, false);
        } else if (frames <= 4) {
            if (count) CRT_REFILL(4, true); else CRT_REFILL(4, false);
        } else if (frames <= 16) {
            if (count) CRT_REFILL(16, true); else CRT_REFILL(16, false);
        } else {
            if (count) CRT_REFILL(64, true); else CRT_REFILL(64, false);
        }
#undef CRT_REFILL
#undef CRT_REFILL_T
    } else if (frames <= 4) {
        if (count) CRT_LAUNCH(4, true); else CRT_LAUNCH(4, false);
    } else if (frames <= 16) {
        if (count) CRT_LAUNCH(16, true); else CRT_LAUNCH(16, false);
    } else if (frames <= 64) {
        if (count) CRT_LAUNCH(64, true); else CRT_LAUNCH(64, false);
    } else {
        return set_error(CRT_E_UNSUPPORTED, "max_ray_depth > 63 with recursive materials is not supported");
    }
#undef CRT_LAUNCH
#undef CRT_LAUNCH_T
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

int render_into(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, hipStream_t stream, bool count) {
    if (sc->grid_empty) {
        /* bucket grid rounds to zero buckets: the reference renders nothing and
         * returns the zero-initialised image (crt_renderer.cpp:158-174) */
        HIP_TRY(hipMemsetAsync(d_rgb, 0, (size_t)sc->info.width * sc->info.height * 3 * sizeof(float), stream));
        return CRT_OK;
    }
    int rc = ensure_plans(sc, st, stream);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_start, stream));
    rc = launch_render(sc, st, sc->full, d_rgb, stream, count);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_stop, stream));
    sc->events_valid = sc->record_events != 0;
    return CRT_OK;
}

}  // namespace

extern "C" {

int crt_hip_scene_upload(const crt_host_scene *h, int device, crt_hip_scene **out) {
    if (!h || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = nullptr;
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_error(CRT_E_INVALID, "no such HIP device");
    HIP_TRY(hipSetDevice(device));
    std::unique_ptr<crt_hip_scene> sc(new crt_hip_scene());
    sc->device = device;
    /* environment overrides of the options (crt_hip_scene_set_option names) */
    static const char *const kEnv[][2] = {{"CRT_TRAVERSAL", "traversal"}, {"CRT_SECONDARY", "secondary"},
                                           {"CRT_WAVEFRONT", "wavefront"}, {"CRT_GI_REFILL", "gi_refill"},
                                           {"CRT_WF_RPW", "wf_rpw"},       {"CRT_TRACE_WALK", "trace_walk"},
                                           {"CRT_CALIBRATE", "calibrate"}, {"CRT_WINDOW", "window"},
                                           {"CRT_EVENTS", "events"}};
    for (const auto &kv : kEnv)
        if (const char *e = std::getenv(kv[0]))
            if (crt_hip_scene_set_option(sc.get(), kv[1], std::atoi(e)) != CRT_OK) return CRT_E_INVALID;
    if (const char *e = std::getenv("CRT_CALIB_K")) {   /* a fixed split threshold instead of the tuned one */
        sc->calib_k = (float)std::atof(e);
        if (sc->calibrate) sc->calibrate = 2;
    }
    if (hs.tree_on_host) sc->tile_work = tile_work_estimate(hs, (hs.width + 7) / 8, (hs.height + 7) / 8);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) {
            sc->wave_slots = prop.multiProcessorCount * 4 * 6;
            sc->refill_waves = prop.multiProcessorCount * 4 * CRT_GI_WAVES;
            int per_cu = 0;   /* resident blocks of the GI machine (registers, LDS) */
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_render_gi<false>, 256, 0) == hipSuccess &&
                per_cu > 0)
                sc->gi_blocks = prop.multiProcessorCount * per_cu;
        }
    }
    crt_host_scene_info(h, &sc->info);
    sc->info.device_bytes = 0;
    for (const DMaterial &m : hs.materials) {
        if (m.type == CRT_MATERIAL_REFLECTIVE || m.type == CRT_MATERIAL_REFRACTIVE) sc->has_secondary = true;
        if (m.type == CRT_MATERIAL_REFRACTIVE) sc->has_refractive = true;
        if (m.type == CRT_MATERIAL_DIFFUSE) sc->has_diffuse = true;
    }
    DeviceScene &ds = sc->ds;
    int rc;
    ds.prune_origin_max = hs.prune_origin_max;
    if (hs.tree_on_host) {
        if ((rc = upload(sc.get(), hs.nodes, &ds.nodes)) != CRT_OK) return rc;
        ds.node_count = (int32_t)hs.nodes.size();
        if ((rc = upload(sc.get(), hs.pnodes, &ds.pnodes)) != CRT_OK) return rc;
        auto ok = [](float x) {
            const float m = std::fabs(x);
            return x == 0.0f || (m >= 0x1p-40f && m <= 0x1p62f);
        };
        ds.planes_ok = 1;
        for (const DNode &n : hs.nodes)
            if (!(ok(n.lo_x) && ok(n.lo_y) && ok(n.lo_z) && ok(n.hi_x) && ok(n.hi_y) && ok(n.hi_z) &&
                  n.lo_x <= n.hi_x && n.lo_y <= n.hi_y && n.lo_z <= n.hi_z))   /* ordered: crt_device.h in_slab */
                ds.planes_ok = 0;
        if ((rc = upload(sc.get(), hs.slots, &ds.slots)) != CRT_OK) return rc;
        if ((rc = upload(sc.get(), hs.slot_tri, &ds.slot_tri)) != CRT_OK) return rc;
        if ((rc = upload(sc.get(), hs.slot_cull, &ds.slot_cull)) != CRT_OK) return rc;
        std::vector<uint32_t> bits((hs.slot_cull.size() + 31) / 32 + 1, 0u);
        for (size_t k = 0; k < hs.slot_cull.size(); ++k)
            if (hs.slot_cull[k]) bits[k >> 5] |= 1u << (k & 31);
        if ((rc = upload(sc.get(), bits, &ds.slot_cull_bits)) != CRT_OK) return rc;
        sc->ref_bounds = hs.ref_bounds;
        sc->ref_children = hs.ref_children;
        sc->ref_leaf_off = hs.ref_leaf_off;
        sc->ref_leaf_tris = hs.ref_leaf_tris;
    } else {
        /* exact tree build on the device (crt_tree_build.hip) */
        DeviceTree dt;
        rc = build_tree_device(hs, nullptr, dt);
        for (void *p : dt.allocs) sc->allocs.push_back(p);
        if (rc != CRT_OK) return rc;
        ds.nodes = dt.nodes;
        ds.node_count = dt.node_count;
        ds.pnodes = dt.pnodes;
        ds.planes_ok = dt.planes_ok;
        ds.slots = dt.slots;
        ds.slot_tri = dt.slot_tri;
        ds.slot_cull = dt.slot_cull;
        ds.slot_cull_bits = dt.slot_cull_bits;
        sc->dt_ref_bounds = dt.ref_bounds;
        sc->dt_ref_children = dt.ref_children;
        sc->dt_ref_leaf_off = dt.ref_leaf_off;
        sc->dt_ref_leaf_tris = dt.ref_leaf_tris;
        sc->info.node_count = dt.node_count;
        sc->info.leaf_count = dt.leaf_count;
        sc->info.leaf_ref_count = dt.slot_count;
        sc->info.max_depth = dt.max_depth;
        sc->info.max_leaf_size = dt.max_leaf_size;
        sc->info.tree_build_ms = dt.build_ms;
        sc->info.tree_on_device = 1;
        const int64_t n = dt.node_count, m = dt.slot_count;
        sc->info.device_bytes += n * (int64_t)sizeof(DNode) + 8 * (n + 1) * (int64_t)sizeof(PNode) +
                                 m * (int64_t)(sizeof(DTriGeo) + 4 + 1) + (m / 32 + 1) * 4;
    }
    if (hs.bnode_count > 0) {   /* secondary-ray BVH (crt_bvh.h) */
        if ((rc = upload(sc.get(), hs.bnodes, &ds.bnodes)) != CRT_OK) return rc;
        if ((rc = upload(sc.get(), hs.btri, &ds.btri)) != CRT_OK) return rc;
        if ((rc = upload(sc.get(), hs.btri_id, &ds.btri_id)) != CRT_OK) return rc;
        ds.bnode_count = hs.bnode_count;
    }
    sc->camera_fast = camera_rays_fast(hs, ds.planes_ok != 0);
    if ((rc = upload(sc.get(), hs.tri_attr, &ds.tri_attr)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.vnormal, &ds.vnormal)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.vuv, &ds.vuv)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.materials, &ds.materials)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.textures, &ds.textures)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.texels, &ds.texels)) != CRT_OK) return rc;
    if ((rc = upload(sc.get(), hs.lights, &ds.lights)) != CRT_OK) return rc;
    ds.light_count = (int32_t)hs.lights.size();
    std::memcpy(ds.cam_loc, hs.cam_loc, sizeof ds.cam_loc);
    std::memcpy(ds.cam_rot, hs.cam_rot, sizeof ds.cam_rot);
    ds.width = hs.width;
    ds.height = hs.height;
    ds.aspect = hs.aspect;
    ds.tan_half_fov = hs.tan_half_fov;
    std::memcpy(ds.background, hs.background, sizeof ds.background);
    ds.gi_on = hs.gi_on;
    ds.reflections_on = hs.reflections_on;
    ds.refractions_on = hs.refractions_on;

    HIP_TRY(hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&sc->ev_start));
    HIP_TRY(hipEventCreate(&sc->ev_stop));
    void *p = nullptr;
    HIP_TRY(hipMalloc(&p, 16 * sizeof(unsigned long long)));
    sc->allocs.push_back(p);
    sc->d_counters = static_cast<unsigned long long *>(p);
    p = nullptr;
    HIP_TRY(hipMalloc(&p, 64));
    sc->allocs.push_back(p);
    sc->d_next_px = static_cast<int32_t *>(p);

    int64_t px = 0;
    const std::vector<DBucket> all = shard_buckets(hs.width, hs.height, hs.bucket_size, 0, 1, &px);
    sc->grid_empty = all.empty();
    if ((rc = make_tile_plan(sc.get(), all, true, sc->full)) != CRT_OK) return rc;
    *out = sc.release();
    return CRT_OK;
}

int crt_hip_scene_create_ex(const crt_scene_desc *desc, int device, int flags, crt_hip_scene **out) {
    if (!desc || !out) return set_error(CRT_E_INVALID, "null argument");
    int mode = flags & 3;
    if (mode == CRT_SCENE_TREE_AUTO) {
        if (const char *e = std::getenv("CRT_TREE_BUILD")) {
            if (std::strcmp(e, "host") == 0) mode = CRT_SCENE_TREE_HOST;
            if (std::strcmp(e, "device") == 0) mode = CRT_SCENE_TREE_DEVICE;
        }
    }
    if (mode == CRT_SCENE_TREE_AUTO) {
        int64_t nt = 0;
        for (int i = 0; i < desc->mesh_count && desc->meshes; ++i) nt += desc->meshes[i].index_count / 3;
        mode = nt >= CRT_SCENE_DEVICE_BUILD_MIN ? CRT_SCENE_TREE_DEVICE : CRT_SCENE_TREE_HOST;
    }
    if (mode != CRT_SCENE_TREE_HOST && mode != CRT_SCENE_TREE_DEVICE) return set_error(CRT_E_INVALID, "bad tree build flag");
    std::unique_ptr<HostScene> hs(new HostScene());
    int rc = prepare_scene(desc, *hs, mode == CRT_SCENE_TREE_HOST);
    if (rc != CRT_OK) return rc;
    return crt_hip_scene_upload(reinterpret_cast<crt_host_scene *>(hs.get()), device, out);
}

int crt_hip_scene_from_tree(const crt_tree_scene_desc *desc, int device, crt_hip_scene **out) {
    if (!desc || !out) return set_error(CRT_E_INVALID, "null argument");
    std::unique_ptr<HostScene> hs(new HostScene());
    const int rc = prepare_scene_from_tree(desc, *hs);
    if (rc != CRT_OK) return rc;
    return crt_hip_scene_upload(reinterpret_cast<crt_host_scene *>(hs.get()), device, out);
}

int crt_hip_scene_create(const crt_scene_desc *desc, int device, crt_hip_scene **out) {
    return crt_hip_scene_create_ex(desc, device, CRT_SCENE_TREE_AUTO, out);
}

int crt_hip_scene_tree(const crt_hip_scene *sc, float *bounds, int32_t *children, int64_t *leaf_offsets,
                       int32_t *leaf_tris) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    const int64_t n = sc->info.node_count, m = sc->info.leaf_ref_count;
    if (sc->info.tree_on_device) {
        HIP_TRY(hipSetDevice(sc->device));
        if (bounds) HIP_TRY(hipMemcpy(bounds, sc->dt_ref_bounds, (size_t)n * 6 * sizeof(float), hipMemcpyDeviceToHost));
        if (children) HIP_TRY(hipMemcpy(children, sc->dt_ref_children, (size_t)n * 2 * sizeof(int32_t), hipMemcpyDeviceToHost));
        if (leaf_offsets)
            HIP_TRY(hipMemcpy(leaf_offsets, sc->dt_ref_leaf_off, (size_t)(n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
        if (leaf_tris && m > 0)
            HIP_TRY(hipMemcpy(leaf_tris, sc->dt_ref_leaf_tris, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost));
        return CRT_OK;
    }
    if (bounds) std::memcpy(bounds, sc->ref_bounds.data(), sc->ref_bounds.size() * sizeof(float));
    if (children) std::memcpy(children, sc->ref_children.data(), sc->ref_children.size() * sizeof(int32_t));
    if (leaf_offsets) std::memcpy(leaf_offsets, sc->ref_leaf_off.data(), sc->ref_leaf_off.size() * sizeof(int64_t));
    if (leaf_tris) std::memcpy(leaf_tris, sc->ref_leaf_tris.data(), sc->ref_leaf_tris.size() * sizeof(int32_t));
    return CRT_OK;
}

int crt_hip_scene_info(const crt_hip_scene *sc, crt_scene_info *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = sc->info;
    return CRT_OK;
}

void crt_hip_scene_destroy(crt_hip_scene *sc) {
    if (!sc) return;
    (void)hipSetDevice(sc->device);
    if (sc->stream) (void)hipStreamSynchronize(sc->stream);
    for (void *p : sc->allocs) (void)hipFree(p);
    for (void *p : sc->plan_allocs) (void)hipFree(p);
    if (sc->d_out) (void)hipFree(sc->d_out);
    if (sc->gi_frames) (void)hipFree(sc->gi_frames);
    wf_free(sc->wf);
    for (auto &kv : sc->unpack_plans) (void)hipFree(kv.second.first);
    for (auto &kv : sc->compact_unpack) (void)hipFree(kv.second.first);
    if (sc->ev_start) (void)hipEventDestroy(sc->ev_start);
    if (sc->ev_stop) (void)hipEventDestroy(sc->ev_stop);
    if (sc->stream) (void)hipStreamDestroy(sc->stream);
    delete sc;
}

int crt_hip_render_device(crt_hip_scene *sc, const crt_renderer_settings *st, float *d_rgb, void *stream) {
    if (!sc || !d_rgb) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    return render_into(sc, st, d_rgb, s, false);
}

int crt_hip_render(crt_hip_scene *sc, const crt_renderer_settings *st, float *rgb_out, crt_render_stats *stats) {
    if (!sc || !rgb_out) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(sc->device));
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    rc = render_into(sc, st, sc->d_out, sc->stream, false);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(rgb_out, sc->d_out, nfl * sizeof(float), hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    if (wf_overflowed(sc->wf, true)) {   /* recorded level sizes did not hold: render again with read-backs */
        if ((rc = render_into(sc, st, sc->d_out, sc->stream, false)) != CRT_OK) return rc;
        HIP_TRY(hipMemcpyAsync(rgb_out, sc->d_out, nfl * sizeof(float), hipMemcpyDeviceToHost, sc->stream));
        HIP_TRY(hipStreamSynchronize(sc->stream));
    }
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        float ms = 0.f;
        if (!sc->grid_empty && sc->full.ntiles > 0 && sc->events_valid)
            HIP_TRY(hipEventElapsedTime(&ms, sc->ev_start, sc->ev_stop));
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->width = sc->info.width;
        stats->height = sc->info.height;
    }
    return CRT_OK;
}

int crt_hip_plan_info(const crt_hip_scene *sc, crt_plan_info *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    std::memset(out, 0, sizeof *out);
    out->calib_k = (sc->calib_walk >= 0 && !sc->calib.empty()) ? (double)sc->calib_k : 0.0;
    out->tiles = sc->full.ntiles;
    for (const Tile &t : sc->full.tiles) out->small_tiles += t.w * t.h <= 16 ? 1 : 0;
    return CRT_OK;
}

int crt_hip_last_kernel_ms(crt_hip_scene *sc, double *ms) {
    if (!sc || !ms) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    if (!sc->events_valid) return set_error(CRT_E_INVALID, "no timed render (option \"events\" is off)");
    HIP_TRY(hipEventSynchronize(sc->ev_stop));
    float f = 0.f;
    HIP_TRY(hipEventElapsedTime(&f, sc->ev_start, sc->ev_stop));
    *ms = f;
    return CRT_OK;
}

int64_t crt_hip_shard_floats(const crt_hip_scene *sc, int shard, int shard_count) {
    if (!sc || shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    int64_t px = 0;
    shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, shard, shard_count, &px);
    return 3 * px;
}

int64_t crt_hip_shard_stride(const crt_hip_scene *sc, int shard_count) {
    if (!sc || shard_count <= 0) return set_error(CRT_E_INVALID, "bad shard count");
    int64_t m = 0;
    for (int s = 0; s < shard_count; ++s) m = std::max(m, crt_hip_shard_floats(sc, s, shard_count));
    return (m + 63) / 64 * 64;
}

}  // extern "C"

namespace {

/* The frame's live-pixel mask (k_live_pixels), computed once per scene. */
int ensure_live_mask(crt_hip_scene *sc) {
    if (!sc->live_mask.empty() || sc->grid_empty) return CRT_OK;
    const DeviceScene *d_scene = nullptr;
    int rc = sync_device_record(sc, &d_scene);
    if (rc != CRT_OK) return rc;
    const int64_t npx = (int64_t)sc->info.width * sc->info.height;
    uint8_t *d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)npx));
    hipLaunchKernelGGL(k_live_pixels, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, sc->stream, d_scene, d);
    hipError_t e = hipGetLastError();
    std::vector<uint8_t> m((size_t)npx);
    if (e == hipSuccess) e = hipMemcpyAsync(m.data(), d, (size_t)npx, hipMemcpyDeviceToHost, sc->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return set_error(CRT_E_HIP, std::string("live mask: ") + hipGetErrorString(e));
    sc->live_mask.swap(m);
    return CRT_OK;
}

std::vector<DBucket> compact_tiles(crt_hip_scene *sc, int shard, int shard_count, int64_t *px,
                                   std::vector<DBucket> *dead = nullptr) {
    return shard_live_tiles(sc->info.width, sc->info.height, sc->info.bucket_size, shard, shard_count,
                            sc->live_mask.empty() ? nullptr : sc->live_mask.data(), px, dead);
}

int render_shard_t(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count, float *d_packed,
                   void *stream, bool compact) {
    if (!sc || !d_packed) return set_error(CRT_E_INVALID, "null argument");
    if (shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    if ((rc = ensure_plans(sc, st, s)) != CRT_OK) return rc;
    if (compact && (rc = ensure_live_mask(sc)) != CRT_OK) return rc;
    auto &plans = compact ? sc->compact_plans : sc->shard_plans;
    auto key = std::make_pair(shard, shard_count);
    auto it = plans.find(key);
    if (it == plans.end()) {
        int64_t px = 0;
        const std::vector<DBucket> b = compact ? compact_tiles(sc, shard, shard_count, &px)
                                               : shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size,
                                                               shard, shard_count, &px);
        ShardPlan plan;
        if ((rc = make_tile_plan(sc, b, false, plan)) != CRT_OK) return rc;
        it = plans.emplace(key, plan).first;
    }
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_start, s));
    rc = launch_render(sc, st, it->second, d_packed, s, false);
    if (rc != CRT_OK) return rc;
    if (sc->record_events) HIP_TRY(hipEventRecord(sc->ev_stop, s));
    sc->events_valid = sc->record_events != 0;
    return CRT_OK;
}

/* write_ppm's conversion of one component on the host (k_quantize). */
uint8_t quantize_host(float c) {
    const float x = c * 255.0f;
    int v = (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : (int)0x80000000;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

template <class T>
int unpack_shards_t(crt_hip_scene *sc, int shard_count, const T *d_gathered, T *d_rgb, void *stream, bool compact) {
    if (!sc || !d_gathered || !d_rgb || shard_count <= 0) return set_error(CRT_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(sc->device));
    if (compact) {
        const int rc = ensure_live_mask(sc);
        if (rc != CRT_OK) return rc;
    }
    auto &plans = compact ? sc->compact_unpack : sc->unpack_plans;
    auto it = plans.find(shard_count);
    if (it == plans.end()) {
        const int64_t stride = compact ? crt_hip_compact_stride(sc, shard_count) : crt_hip_shard_stride(sc, shard_count);
        if (stride < 0) return (int)stride;
        std::vector<UnpackBucket> ub;
        std::vector<DBucket> dead;
        for (int s = 0; s < shard_count; ++s) {
            int64_t px = 0;
            const std::vector<DBucket> b = compact ? compact_tiles(sc, s, shard_count, &px, &dead)
                                                   : shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size,
                                                                   s, shard_count, &px);
            for (const DBucket &x : b) ub.push_back(UnpackBucket{x.x, x.y, x.w, x.h, s * stride + 3 * x.packed_offset, 0});
        }
        for (const DBucket &x : dead) ub.push_back(UnpackBucket{x.x, x.y, x.w, x.h, -1, 0});
        UnpackBucket *d = nullptr;
        if (!ub.empty()) {
            HIP_TRY(hipMalloc(&d, ub.size() * sizeof(UnpackBucket)));
            HIP_TRY(hipMemcpy(d, ub.data(), ub.size() * sizeof(UnpackBucket), hipMemcpyHostToDevice));
        }
        it = plans.emplace(shard_count, std::make_pair(d, (int)ub.size())).first;
    }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : sc->stream;
    if (sc->grid_empty)
        HIP_TRY(hipMemsetAsync(d_rgb, 0, (size_t)sc->info.width * sc->info.height * 3 * sizeof(T), s));
    if (it->second.second > 0) {
        Rgb<T> bg;
        for (int k = 0; k < 3; ++k) {
            if constexpr (sizeof(T) == 1) bg.c[k] = quantize_host(sc->ds.background[k]);
            else bg.c[k] = sc->ds.background[k];
        }
        hipLaunchKernelGGL(k_unpack<T>, dim3(it->second.second), dim3(256), 0, s, it->second.first, d_gathered, d_rgb,
                           sc->info.width, bg);
        HIP_TRY(hipGetLastError());
    }
    return CRT_OK;
}
}  // namespace

extern "C" {

int crt_hip_render_shard(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count,
                         float *d_packed, void *stream) {
    return render_shard_t(sc, st, shard, shard_count, d_packed, stream, false);
}

int crt_hip_unpack_shards(crt_hip_scene *sc, int shard_count, const float *d_gathered, float *d_rgb, void *stream) {
    return unpack_shards_t<float>(sc, shard_count, d_gathered, d_rgb, stream, false);
}

int crt_hip_unpack_shards_rgb8(crt_hip_scene *sc, int shard_count, const uint8_t *d_gathered, uint8_t *d_rgb8,
                               void *stream) {
    return unpack_shards_t<uint8_t>(sc, shard_count, d_gathered, d_rgb8, stream, false);
}

int crt_hip_live_mask(crt_hip_scene *sc, uint8_t *out) {
    if (!sc) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_live_mask(sc);
    if (rc != CRT_OK) return rc;
    if (out && !sc->live_mask.empty()) std::memcpy(out, sc->live_mask.data(), sc->live_mask.size());
    else if (out) std::memset(out, 0, (size_t)sc->info.width * sc->info.height);
    return CRT_OK;
}

int64_t crt_hip_compact_floats(crt_hip_scene *sc, int shard, int shard_count) {
    if (!sc || shard_count <= 0 || shard < 0 || shard >= shard_count) return set_error(CRT_E_INVALID, "bad shard");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_live_mask(sc);
    if (rc != CRT_OK) return rc;
    int64_t px = 0;
    compact_tiles(sc, shard, shard_count, &px);
    return 3 * px;
}

int64_t crt_hip_compact_stride(crt_hip_scene *sc, int shard_count) {
    if (!sc || shard_count <= 0) return set_error(CRT_E_INVALID, "bad shard count");
    int64_t m = 0;
    for (int s = 0; s < shard_count; ++s) {
        const int64_t f = crt_hip_compact_floats(sc, s, shard_count);
        if (f < 0) return f;
        m = std::max(m, f);
    }
    return std::max<int64_t>(64, (m + 63) / 64 * 64);
}

int crt_hip_render_shard_compact(crt_hip_scene *sc, const crt_renderer_settings *st, int shard, int shard_count,
                                 float *d_packed, void *stream) {
    return render_shard_t(sc, st, shard, shard_count, d_packed, stream, true);
}

int crt_hip_unpack_compact(crt_hip_scene *sc, int shard_count, const float *d_gathered, float *d_rgb, void *stream) {
    return unpack_shards_t<float>(sc, shard_count, d_gathered, d_rgb, stream, true);
}

int crt_hip_unpack_compact_rgb8(crt_hip_scene *sc, int shard_count, const uint8_t *d_gathered, uint8_t *d_rgb8,
                                void *stream) {
    return unpack_shards_t<uint8_t>(sc, shard_count, d_gathered, d_rgb8, stream, true);
}

int crt_hip_quantize_rgb8(const float *d_rgb, int64_t n, int32_t max_color_component, uint8_t *d_out, void *stream) {
    if ((n > 0 && (!d_rgb || !d_out)) || n < 0) return set_error(CRT_E_INVALID, "bad argument");
    if (max_color_component < 0 || max_color_component > 255)
        return set_error(CRT_E_UNSUPPORTED, "8-bit output needs max_color_component in 0..255");
    if (n == 0) return CRT_OK;
    const int64_t threads = (n + 3) / 4;
    hipLaunchKernelGGL(k_quantize, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_rgb, d_out, n, (float)max_color_component,
                       max_color_component);
    HIP_TRY(hipGetLastError());
    return CRT_OK;
}

int crt_hip_trace_batch(crt_hip_scene *sc, const float *rays, int64_t n, crt_hit *hits_out) {
    if (!sc || (n > 0 && (!rays || !hits_out)) || n < 0) return set_error(CRT_E_INVALID, "bad argument");
    if (n == 0) return CRT_OK;
    HIP_TRY(hipSetDevice(sc->device));
    float *d_rays = nullptr;
    crt_hit *d_hits = nullptr;
    HIP_TRY(hipMalloc(&d_rays, (size_t)n * 6 * sizeof(float)));
    hipError_t e = hipMalloc(&d_hits, (size_t)n * sizeof(crt_hit));
    if (e != hipSuccess) { (void)hipFree(d_rays); return set_error(CRT_E_HIP, hipGetErrorString(e)); }
    e = hipMemcpy(d_rays, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_trace_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, sc->stream, sc->ds, d_rays,
                           n, d_hits, sc->trace_walk);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(sc->stream);
    if (e == hipSuccess) e = hipMemcpy(hits_out, d_hits, (size_t)n * sizeof(crt_hit), hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    (void)hipFree(d_hits);
    if (e != hipSuccess) return set_error(CRT_E_HIP, hipGetErrorString(e));
    return CRT_OK;
}

int crt_hip_profile_waves(crt_hip_scene *sc, const crt_renderer_settings *st, uint64_t *stamps, int64_t cap,
                          int32_t *tile_xy) {
    if (!sc || !st) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    {
        const int rc = ensure_plans(sc, st, sc->stream);
        if (rc != CRT_OK) return rc;
    }
    const int nt = sc->full.ntiles;
    if (!stamps || !tile_xy) return nt;      /* query the size */
    if (cap < nt) return set_error(CRT_E_INVALID, "stamp buffer too small");
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    unsigned long long *d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)nt * 2 * sizeof(unsigned long long)));
    int rc = launch_render(sc, st, sc->full, sc->d_out, sc->stream, false, d);
    hipError_t e = rc == CRT_OK ? hipStreamSynchronize(sc->stream) : hipSuccess;
    if (rc == CRT_OK && e == hipSuccess)
        e = hipMemcpy(stamps, d, (size_t)nt * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::vector<Tile> tiles(nt);
    if (rc == CRT_OK && e == hipSuccess)
        e = hipMemcpy(tiles.data(), sc->full.d_tiles, (size_t)nt * sizeof(Tile), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (rc != CRT_OK) return rc;
    if (e != hipSuccess) return set_error(CRT_E_HIP, hipGetErrorString(e));
    for (int k = 0; k < nt; ++k) { tile_xy[2 * k] = tiles[k].x; tile_xy[2 * k + 1] = tiles[k].y; }
    return nt;
}

int crt_hip_plan_tiles(crt_hip_scene *sc, const crt_renderer_settings *st, int32_t *xywh, float *cost, int64_t cap) {
    if (!sc || !st) return set_error(CRT_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(sc->device));
    const int rc = ensure_plans(sc, st, sc->stream);
    if (rc != CRT_OK) return rc;
    const ShardPlan &p = sc->full;
    if (!xywh) return p.ntiles;
    if (cap < p.ntiles) return set_error(CRT_E_INVALID, "tile buffer too small");
    for (int k = 0; k < p.ntiles; ++k) {
        xywh[4 * k] = p.tiles[k].x;
        xywh[4 * k + 1] = p.tiles[k].y;
        xywh[4 * k + 2] = p.tiles[k].w;
        xywh[4 * k + 3] = p.tiles[k].h;
        if (cost) cost[k] = p.cost.empty() ? 0.f : p.cost[k];
    }
    return p.ntiles;
}

int crt_hip_count_work(crt_hip_scene *sc, const crt_renderer_settings *st, crt_work_counts *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    int rc = check_settings(st);
    if (rc != CRT_OK) return rc;
    HIP_TRY(hipSetDevice(sc->device));
    std::memset(out, 0, sizeof *out);
    if (sc->grid_empty) return CRT_OK;
    const size_t nfl = (size_t)sc->info.width * sc->info.height * 3;
    if (!sc->d_out) HIP_TRY(hipMalloc(&sc->d_out, nfl * sizeof(float)));
    if ((rc = ensure_plans(sc, st, sc->stream)) != CRT_OK) return rc;
    HIP_TRY(hipMemsetAsync(sc->d_counters, 0, 16 * sizeof(unsigned long long), sc->stream));
    rc = launch_render(sc, st, sc->full, sc->d_out, sc->stream, true);
    if (rc != CRT_OK) return rc;
    unsigned long long c[16];
    HIP_TRY(hipMemcpyAsync(c, sc->d_counters, sizeof c, hipMemcpyDeviceToHost, sc->stream));
    HIP_TRY(hipStreamSynchronize(sc->stream));
    out->traversals = c[0];
    out->node_tests = c[1];
    out->triangle_tests = c[2];
    out->hits = c[3];
    sc->wave_counts.node_steps = c[4];
    sc->wave_counts.triangle_steps = c[5];
    sc->wave_counts.edge_steps = c[6];
    sc->wave_counts.waves = c[7];
    sc->wave_counts.box_steps = c[8];
    sc->wave_counts.pass_steps = c[9];
    sc->wave_counts.window_waves = c[10];
    sc->wave_counts.window_steps = c[11];
    sc->wave_counts.window_slots = c[12];
    sc->wave_counts.window_reached = c[13];
    sc->wave_counts.window_tri_rounds = c[14];
    return CRT_OK;
}

int crt_hip_scene_set_option(crt_hip_scene *sc, const char *name, int value) {
    if (!sc || !name) return set_error(CRT_E_INVALID, "null argument");
    const std::string k(name);
    if (k == "traversal") {
        if (value != 7 && value != 8) return set_error(CRT_E_INVALID, "traversal must be 7 (reference order) or 8 (pruned)");
        sc->traversal = value;
        wf_graphs_clear(sc->wf);   /* captured wavefront frames bake in the level-0 walk */
    } else if (k == "secondary") {
        if (value != 0 && value != 4 && value != 10 && value != 14)
            return set_error(CRT_E_INVALID, "secondary must be 0, 4, 10 or 14");
        sc->secondary = value;
        wf_graphs_clear(sc->wf);   /* ... the levels' walk */
    } else if (k == "wavefront") {
        sc->wavefront = value != 0;
    } else if (k == "window") {
        sc->window_walk = value != 0;
    } else if (k == "gi_refill") {
        sc->gi_refill = value != 0;
    } else if (k == "gi_machine") {
        sc->gi_machine = value != 0;
    } else if (k == "calib_k_milli") {   /* a fixed split threshold k = value / 1000 (calibrate 2) */
        if (value <= 0) return set_error(CRT_E_INVALID, "calib_k_milli must be > 0");
        sc->calib_k = (float)value / 1000.0f;
        sc->calibrate = 2;
        sc->calib_walk = -1;
    } else if (k == "wf_graph") {
        sc->wf_graph = value != 0;
        wf_graphs_clear(sc->wf);
    } else if (k == "wf_replay") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "wf_replay must be 0, 1 or 2");
        sc->wf_replay = value;
        sc->wf.recs.clear();
        wf_graphs_clear(sc->wf);
    } else if (k == "wf_rpw") {
        if (value < 1 || value > 64) return set_error(CRT_E_INVALID, "wf_rpw must be 1..64");
        sc->wf_rays_per_wave = value;
        wf_graphs_clear(sc->wf);   /* ... and each level's rays per wave */
    } else if (k == "events") {
        sc->record_events = value != 0;
    } else if (k == "calibrate") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "calibrate must be 0 (estimate plan), 1 (tuned) or 2 (fixed k)");
        if (value != sc->calibrate) sc->calib_walk = sc->calibrate ? -1 : sc->calib_walk;   /* re-plan on next use */
        sc->calibrate = value;
        if (!sc->calibrate && !sc->calib.empty()) {   /* back to the estimate plan */
            HIP_TRY(hipDeviceSynchronize());
            sc->calib.clear();
            sc->calib_walk = -1;
            free_plans(sc);
            int64_t px = 0;
            const int rc = make_tile_plan(sc, shard_buckets(sc->info.width, sc->info.height, sc->info.bucket_size, 0, 1, &px),
                                          true, sc->full);
            if (rc != CRT_OK) return rc;
        }
    } else if (k == "calib_min") {   /* smallest side the calibrated plan splits tiles down to */
        if (value != 1 && value != 2 && value != 4 && value != 8) return set_error(CRT_E_INVALID, "calib_min must be 1, 2, 4 or 8");
        sc->calib_min = value;
        sc->calib_walk = -1;
    } else if (k == "shadows") {
        sc->shadows = value != 0;
    } else if (k == "trace_walk") {
        if (value < 0 || value > 2) return set_error(CRT_E_INVALID, "trace_walk must be 0, 1 or 2 (BVH)");
        sc->trace_walk = value;
    } else {
        return set_error(CRT_E_INVALID, "unknown option: " + k);
    }
    /* tile plans depend on the walk (tile splitting): rebuild on next use */
    return CRT_OK;
}

int crt_hip_wave_counts(crt_hip_scene *sc, crt_wave_counts *out) {
    if (!sc || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = sc->wave_counts;
    return CRT_OK;
}

}  // extern "C"
#endif  // CRT_SIDE_TU
