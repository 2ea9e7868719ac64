/*
 * crt_layout.h — the scene as it lives in HBM (shared by host prep and kernels).
 *
 * Reference data structures being replaced:
 *   AccelerationTreeNode { vector<Triangle> triangles; AABB bounds; int children[2]; int parent; }
 *       64 B + heap-allocated Triangle copies (crt_acceleration_tree.h:15-24)
 *   Triangle { const Vertex *v0,*v1,*v2; Vector face_normal; int material; flags }
 *       48 B with pointers into an AoS Vertex array (crt_triangle.h:19-23)
 *
 * Device layout:
 *   DNode[n]   32 B, in TRAVERSAL order = the order the reference's LIFO walk
 *              (crt_intersection.cpp:116-133: push child0, push child1, pop)
 *              visits nodes, i.e. preorder with child1 before child0.  A node
 *              whose box test passes continues at i+1 (its first visited
 *              child); a failed node or a leaf continues at `skip` — so the
 *              walk needs no stack and visits exactly the reference's node
 *              sequence.
 *   DTriGeo[m] 48 B per LEAF SLOT: every triangle copy a leaf holds
 *              (the reference's duplicated Triangle copies) stored contiguously
 *              in leaf order, so a leaf is one contiguous run of 48-B records.
 *   slot_tri[m] int32 global triangle id of each slot (final-hit attributes).
 *   slot_cull[m] uint8 back_face_culling flag (read only for back-face hits).
 *   DTriAttr[t] 16 B per triangle: vertex ids + material + smooth flag.
 *   vertex normals / uvs as float4 (16-B aligned loads).
 */
#pragma once
#include <stdint.h>

namespace crt_amd {

/* (lo, hi) of an axis sit in adjacent dwords: a scalar load puts each pair in
 * an aligned SGPR pair, the direct operand of the box test's packed ops. */
struct alignas(16) DNode {
    float lo_x, hi_x, lo_y, hi_y;
    float lo_z, hi_z;
    int32_t a;   /* interior: skip index (first node after the subtree) | leaf: count | depth << 24 */
    int32_t b;   /* interior: -(depth + 1)                               | leaf: first slot           */
};
static_assert(sizeof(DNode) == 32, "DNode must be 32 B");

/* Topology of the reference-order tree for the BVH walk's proof (crt_bvh.h
 * verify_topo), one 8-B record per DNode: the descent toward a hit point
 * needs only which children exist and where the second one starts — the
 * children's cells are the parent's halves (AABB::split, crt_aabb.h:24-35:
 * mid = (lo + hi) * 0.5f on axis depth % 3), computed in registers.
 *   interior: a = second child's index (-1: one child), b = -1 (first child,
 *             i + 1, is the lower half) or -2 (it is the upper half: the
 *             reference's LIFO walk visits child 1 first); a second child is
 *             the other half
 *   leaf:     a = triangle copies, b = first slot */
struct KTopo {
    int32_t a, b;
};
static_assert(sizeof(KTopo) == 8, "KTopo must be 8 B");

/* verify_topo's descent two levels a load: for node i, the KTopo records of
 * its children and grandchildren in heap order (the node is position 1,
 * position q's children are 2q and 2q + 1: first child i + 1, second child
 * KTopo::a), entry q - 2 for q = 2..7; absent ones {0, 0}.  64 B.  (Three
 * levels in one 128-B line took 30 more VGPRs in the camera kernel: one wave
 * less per SIMD.) */
struct alignas(64) KTopo2 {
    KTopo t[8];
};
static_assert(sizeof(KTopo2) == 64, "KTopo2 must be 64 B");

/* Node record of the pruned walks: the reference cell (the box the
 * reference's six-face test runs on — it decides which leaf copies are
 * eligible, crt_intersection.cpp:121) plus a conservative hull of every
 * triangle in the subtree, widened by a bound on the triangle test's rounding
 * (crt_scene_build.cpp: hull_margin).  A ray whose best hit so far is nearer
 * than the hull's entry distance cannot find a better (t, slot) key inside,
 * so the subtree is skipped without changing the result.  The node array is
 * stored 8 times, once per direction octant, each in preorder with the
 * near child (by the sign of d on the node's split axis, depth % 3) first;
 * `a` is the skip index within that octant's order, `b`/leaf fields as DNode.
 * Leaf slot numbers are the reference's visit order in every copy, so ties in
 * t are broken exactly as the reference's first-found rule does. */
struct alignas(16) PNode {
    float lo_x, hi_x, lo_y, hi_y;   /* cell, (lo, hi) pairs as DNode */
    float lo_z, hi_z;
    int32_t a, b;
    float tlo_x, thi_x, tlo_y, thi_y;   /* hull */
    float tlo_z, thi_z;
    int32_t depth;   /* tree depth (indexes the packet walk's reach mask) */
    int32_t count;   /* leaf: triangle copies, interior: 0 */
};
static_assert(sizeof(PNode) == 64, "PNode must be 64 B");

/* Node of the secondary-ray BVH (crt_bvh.h): a bounding volume hierarchy
 * over the scene's triangles (each triangle once, not the tree's duplicated
 * leaf copies), whose boxes are unions of the triangles' hulls (the same
 * conservative hulls as PNode's), stored like PNode once per direction octant
 * in preorder with the near child first.  `skip` is the first node after the
 * subtree in that order; `leaf` = first * 16 + count for a leaf (count 1..15,
 * triangles first .. first + count - 1 of the BVH triangle array), 0 for an
 * interior node. */
struct alignas(16) BNode {
    float lo_x, hi_x, lo_y, hi_y;
    float lo_z, hi_z;
    int32_t skip;
    int32_t leaf;
};
static_assert(sizeof(BNode) == 32, "BNode must be 32 B");

struct alignas(16) DTriGeo {
    float v0x, v0y, v0z, v1x;
    float v1y, v1z, v2x, v2y;
    float v2z, nx, ny, nz;
};
static_assert(sizeof(DTriGeo) == 48, "DTriGeo must be 48 B");

/* Camera-bin candidate (crt_bvh.h walk_bins, crt_bvh_build.cpp
 * build_camera_bins): a triangle listed in an 8x8-pixel cell of the frame
 * because a camera ray of that cell may hit it.  The hull box is the
 * triangle's conservative hull (BNode's boxes are unions of the same hulls);
 * dmin is a lower bound on the t of any hit the reference's triangle test
 * accepts for a camera ray (the cell's list is sorted by it); g and id are
 * the triangle as the BVH's triangle arrays hold it (id | culling << 31);
 * mask / rest let a pixel skip candidates it cannot hit and stop once none
 * is left. */
struct alignas(16) CamCand {
    float lo_x, hi_x, lo_y, hi_y;
    float lo_z, hi_z;
    float dmin;
    int32_t id;
    DTriGeo g;
    uint64_t mask;   /* pixels of the cell (bit 8 y + x) whose camera ray may hit it */
    uint64_t rest;   /* OR of mask over this and every later candidate of the cell */
};
static_assert(sizeof(CamCand) == 96, "CamCand must be 96 B");

/* Light bins of one light (crt_light_bins.cpp build_light_bins, crt_bvh.h
 * lbin_first_hit): a cube map of N x N cells a face around the light, each
 * cell listing (LightCand records) every triangle a shadow
 * ray whose origin lies in that cell's direction can hit on its way to the
 * light, sorted by dmin = the distance from the light to the hull, rounded
 * down; triangles whose hull comes within R0 of the light (and unbounded
 * hulls) are in a near list every ray tests.  Offsets
 * off[base] .. off[base + 6 N^2 + 1]: the near list, then the cells in order
 * (face = 2 axis + (w_axis < 0), row v, column u). */
/* A light-bin candidate (one 64-B line): dmin = the distance from the light
 * to the triangle's hull, rounded down; the triangle as the BVH holds it. */
struct alignas(16) LightCand {
    float dmin;
    int32_t id;      /* triangle id | back_face_culling << 31 */
    int32_t pad0, pad1;
    DTriGeo g;
};
static_assert(sizeof(LightCand) == 64, "LightCand must be 64 B");

struct DLightBin {
    double lx, ly, lz;      /* the light's position */
    double r0_sq;           /* R0^2 */
    double e_sq;            /* rays passing the light farther than e_max (e_sq = e_max^2) are not decided here */
    int32_t base;           /* first offset of this light */
    int32_t on;             /* 0: this light's rays take the BVH */
};
static_assert(sizeof(DLightBin) == 48, "DLightBin must be 48 B");

struct alignas(16) DTriAttr {
    int32_t i0, i1, i2;
    int32_t mat_flags;   /* material index | (smooth_shading << 31) */
};

struct alignas(16) DVec4 { float x, y, z, w; };

struct DMaterial {
    int32_t type;
    int32_t tex;
    float ior;
    int32_t pad;
};

struct DTexture {
    int32_t type;
    float c0x, c0y, c0z;
    float c1x, c1y, c1z;
    float scalar;
    int32_t w, h;
    int64_t texel_offset;   /* into the texel pool (float4 per texel), bitmap only */
};

struct DLight {
    float intensity;
    float px, py, pz;
};

/* The camera as the kernels see it (crt_camera.cpp:7-35): the frame's
 * constants, float(width) / height and std::tan(fov_radians * 0.5f) computed
 * on the host with the reference's libm. */
struct DCamera {
    float loc[3];
    float rot[9];           /* row-major, ray_dir = v * R (crt_matrix.h:66-74) */
    int32_t width, height;
    float aspect;           /* float(width) / height            (crt_camera.cpp:23) */
    float tan_half_fov;     /* std::tan(fov_radians * 0.5f)     (crt_camera.cpp:26-27) */
};

/* Everything a render kernel needs, passed by value. */
struct DeviceScene {
    const DNode *nodes;
    int32_t node_count;
    const PNode *pnodes;            /* 8 octant orders x (node_count + 1) (pruned walks; see pnode_order) */
    float prune_origin_max;         /* hull margins hold for rays with |o|_inf <= this */
    const DTriGeo *slots;
    const int32_t *slot_tri;
    const uint8_t *slot_cull;
    const uint32_t *slot_cull_bits;   /* same flags, 1 bit per slot (scalar-path reads) */
    /* secondary-ray BVH (crt_bvh.h): 8 octant orders x (bnode_count + 1) nodes,
     * its triangles in leaf order (geometry as the slots hold it, and the
     * global triangle id | back_face_culling << 31); null when not built */
    const BNode *bnodes;
    int32_t bnode_count;
    const DTriGeo *btri;
    const int32_t *btri_id;
    /* the proof's tree topology (KTopo, and per node its two levels below,
     * KTopo2); null when the tree lives on the device only */
    const KTopo *ktopo;
    const KTopo2 *ktopo2;
    /* camera bins (crt_bvh.h walk_bins), rebuilt on the device by every camera
     * frame (crt_bins.hip): per 8x8 cell of the frame (bin_tx cells a row),
     * candidates bins[bin_off[c] .. bin_off[c] + bin_len[c]), bin_len -1: the
     * cell's pixels walk the BVH; kBinSets sets taken in turn (the next
     * frames bin while frame k renders): a frame's per-cell entries at
     * set * ncell (set = frame % kBinSets),
     * its records anywhere in `bins` (offsets absolute); null when the scene
     * takes no bins */
    const CamCand *bins;
    const int32_t *bin_off;
    const int32_t *bin_len;
    int32_t bin_tx;
    const DTriAttr *tri_attr;
    const DVec4 *vnormal;
    const DVec4 *vuv;
    const DMaterial *materials;
    const DTexture *textures;
    const DVec4 *texels;
    const DLight *lights;
    int32_t light_count;
    /* light bins (DLightBin; built at the first shadow-ray frame, option
     * "light_bins"): per light its parameters, the offsets and the records;
     * lbin_n 0 when not built */
    const DLightBin *lbin_par;
    const int32_t *lbin_off;
    const LightCand *lbins;
    int32_t lbin_n;
    /* GI angle tables: (cosf, sinf) pairs of pi*u and of 2*pi*u for the 2^23 values of u */
    const float *gi_pi;
    const float *gi_2pi;
    /* powf(x, 5.0f) of the host's libm for every x = k * 2^-24 in [-1, 1]
     * (2^25 + 1 floats, index k + 2^24): the Fresnel term's exact values */
    const float *pow5;
    /* the camera frames are rendered with: a device scene record is one of a
     * ring of records (crt_host_render.hip sync_device_record), so a frame
     * keeps the camera it was issued with while the next frames move it */
    DCamera cam;
    int32_t planes_ok;      /* every node plane is 0 or |p| in [2^-40, 2^62] (crt_device.h coord_ok) */
    float background[3];
    int32_t gi_on, reflections_on, refractions_on;
};

/* Renderer settings as the kernels see them (crt_renderer.h:18-25). */
/* Deferred shadow rays of a frame without recursion (crt_shade.h
 * shade_hit_shadowed, k_shadow_vis, k_shadow_compose): per diffuse hit g a
 * group of light_count records, light-major in chunks of 64 groups
 * (sh_index): a wave of k_shadow_vis takes 64 neighbouring pixels' rays
 * towards one light, whose walks read the same lists. */
#if defined(__HIPCC__)
__host__ __device__ inline
#else
inline
#endif
int64_t sh_index(int64_t g, int l, int nl) { return ((g >> 6) * nl + l) * 64 + (g & 63); }
struct alignas(16) ShRay {
    float ox, oy, oz, r2;   /* origin p + n bias, |light - p|^2 */
    float dx, dy, dz;       /* normalised direction to the light */
    int32_t pix;            /* the pixel's index in the output image (3 floats a pixel); -1: no ray */
};
struct alignas(16) ShCon {
    float x, y, z;          /* the light's term (crt_renderer.cpp:90-95), added when the light is visible */
    uint32_t vis;           /* written by k_shadow_vis */
};

struct DSettings {
    uint32_t max_ray_depth;
    uint32_t diffuse_reflection_ray_count;
    float shadow_bias;
    float reflection_bias;
    float diffuse_reflection_bias;
    float refraction_bias;
    /* deferred shadow rays (null: traced inline) */
    ShRay *sh_rays;
    ShCon *sh_con;
    int32_t *sh_count;      /* groups taken this frame */
    int32_t sh_cap;         /* groups the buffers hold */
};

/* A bucket of the reference grid (crt_renderer.cpp:160-174). */
struct DBucket {
    int32_t x, y, w, h;
    int64_t packed_offset;   /* pixel offset of this bucket inside its shard's packed buffer */
};

}  // namespace crt_amd
