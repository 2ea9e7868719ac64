/*
 * crt_scene_build.cpp — host scene preparation (C++), no GPU.
 *
 *   mesh prep      vertex_array_extend / fill_triangles   crt_mesh.cpp:10-73,
 *                  Triangle ctor face normal              crt_triangle.h:25-33
 *   tree build     acceleration_tree::build/build_branch  crt_acceleration_tree.cpp:13-106,
 *                  AABB::split / intersects               crt_aabb.h:24-45
 *   camera consts  Camera::generate_ray                   crt_camera.cpp:7-35
 *
 * Every float operation that feeds the render is done in the reference's order
 * (fp32, no contraction — built with -ffp-contract=off) so vertex normals, face
 * normals and node bounds come out bit-identical to the reference's.  The
 * tree is rebuilt with an explicit work stack instead of recursion, producing
 * the same node numbering: a node's child0 is created and fully expanded
 * before its child1 is created.
 */
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "crt_device.h"
#include "crt_host.h"

namespace crt_amd {

static thread_local std::string g_last_error;

int set_error(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

namespace {

struct F3 { float x, y, z; };
inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline F3 cross3(F3 a, F3 b) { return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline float length3(F3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline F3 normalized3(F3 a) {
    const float l = length3(a);
    return f3(a.x / l, a.y / l, a.z / l);
}

struct Box6 { float lo[3], hi[3]; };

inline bool box_overlap(const Box6 &cell, const Box6 &b) {   /* crt_aabb.h:37-45 */
    for (int k = 0; k < 3; ++k) {
        if (b.lo[k] > cell.hi[k]) return false;
        if (b.hi[k] < cell.lo[k]) return false;
    }
    return true;
}

struct BuildNode {
    Box6 bounds;
    int32_t child[2] = {-1, -1};
    int32_t depth = 0;
    std::vector<int32_t> tris;   /* leaf contents (non-empty ⇔ leaf) */
};

constexpr int kMaxTreeDepth = 39;    /* crt_acceleration_tree.h:12 */
constexpr size_t kMaxLeafTris = 16;  /* crt_acceleration_tree.h:13 */

/* acceleration_tree::build, iteratively.  Work items: Expand(node, ids) and
 * MakeChild1(parent, bounds, ids).  Expand(n) creates child0 immediately and
 * queues MakeChild1 beneath Expand(child0) on the LIFO, so child0's whole
 * subtree is numbered before child1 exists — the reference's recursion order. */
void build_tree(const std::vector<Box6> &tri_boxes, const Box6 &root_box, std::vector<BuildNode> &nodes) {
    struct Work {
        bool make_child1;
        int32_t node;       /* Expand: node to expand | MakeChild1: parent */
        int32_t depth;      /* depth of the node being expanded / created */
        Box6 bounds;        /* MakeChild1 only */
        std::vector<int32_t> ids;
    };
    nodes.clear();
    BuildNode root;
    root.bounds = root_box;
    nodes.push_back(std::move(root));
    std::vector<Work> stack;
    {
        Work w{false, 0, 0, {}, {}};
        w.ids.resize(tri_boxes.size());
        for (size_t i = 0; i < tri_boxes.size(); ++i) w.ids[i] = (int32_t)i;
        stack.push_back(std::move(w));
    }
    while (!stack.empty()) {
        Work w = std::move(stack.back());
        stack.pop_back();
        int32_t idx = w.node;
        if (w.make_child1) {
            idx = (int32_t)nodes.size();
            BuildNode c;
            c.bounds = w.bounds;
            c.depth = w.depth;
            nodes.push_back(std::move(c));
            nodes[w.node].child[1] = idx;
        }
        const int depth = w.depth;
        if (depth > kMaxTreeDepth || w.ids.size() <= kMaxLeafTris) {   /* :32-35 */
            nodes[idx].tris = std::move(w.ids);
            continue;
        }
        const int axis = depth % 3;                                     /* :38 */
        Box6 c0 = nodes[idx].bounds, c1 = nodes[idx].bounds;
        const float mid = (c0.lo[axis] + c0.hi[axis]) * 0.5f;            /* crt_aabb.h:29 */
        c0.hi[axis] = mid;
        c1.lo[axis] = mid;
        std::vector<int32_t> left, right;
        left.reserve(w.ids.size());
        right.reserve(w.ids.size() / 2);
        for (int32_t id : w.ids) {                                      /* :44-58 */
            const bool in0 = box_overlap(c0, tri_boxes[id]);
            const bool in1 = box_overlap(c1, tri_boxes[id]);
            if (in0) left.push_back(id);
            if (in1) right.push_back(id);
        }
        std::vector<int32_t>().swap(w.ids);
        if (!right.empty()) {
            Work m{true, idx, depth + 1, c1, std::move(right)};
            stack.push_back(std::move(m));
        }
        if (!left.empty()) {
            const int32_t c = (int32_t)nodes.size();
            BuildNode n0;
            n0.bounds = c0;
            n0.depth = depth + 1;
            nodes.push_back(std::move(n0));
            nodes[idx].child[0] = c;
            Work e{false, c, depth + 1, {}, std::move(left)};
            stack.push_back(std::move(e));
        }
    }
}

/* ---- pruned-walk structures (crt_layout.h PNode) ------------------------
 *
 * Why a hull can bound the t the reference computes.  ray_intersect_triangle
 * (crt_intersection.cpp:47-93) accepts t = fl(op / rn) when the rounded
 * point p = o + d*t passes the three rounded edge tests.  With q = o + d*t in
 * exact arithmetic (the point the hull test sees):
 *   - height of q above the plane through v0 with normal N:
 *       N.(q - v0) = t*rn_exact - op_exact, and t*rn_computed = op_computed(1+e),
 *     so the height is a few ulps of |o|, |v0| and |q - o| — the division's
 *     error moves q along the (near-parallel) plane, not away from it;
 *   - in the plane, each rounded edge test admits points at most a few ulps of
 *     |p - v_i| outside its edge line; the three shifted lines bound the
 *     triangle scaled about its incentre, whose corners move by that shift
 *     times diam/inradius (slivers get wide margins).
 * So q lies within c * 2^-24 * (diam * kappa + |o| + |v| + |q|) of the
 * triangle's box, kappa = diam / inradius, c a small constant (< 100).  The
 * hull below uses 2^-14 * (diam * kappa + 2 G) for rays with |o|_inf <= G,
 * G = 4 max |vertex coordinate| — a margin of 2^10 over that bound — and the
 * device's slab test (rcp, one fma per plane: crt_device.h hull_alive) adds
 * errors far below it.  Triangles whose normal is not finite or whose area is 0 (no reliable
 * bound) get an unbounded hull: their subtrees are never pruned. */
/* round_down / round_up / HullD / triangle_hull: crt_device.h (shared with the
 * device build, crt_tree_build.hip, so both builds produce the same bits). */

/* G of the hull margins: 4 max |vertex coordinate| (rounded down: rays above
 * it are simply not pruned). */
void set_prune_origin_max(HostScene &hs) {
    double vmax = 0.0;
    for (float v : hs.vpos)
        if (std::isfinite(v)) vmax = std::max(vmax, (double)std::fabs(v));
    const double G = 4.0 * vmax;
    hs.prune_G = G;
    hs.prune_origin_max = (float)G;
    if ((double)hs.prune_origin_max > G) hs.prune_origin_max = round_down(G);
}

void build_pruned_nodes(const std::vector<BuildNode> &bn, HostScene &hs) {
    const int32_t n = (int32_t)bn.size();
    const double G = hs.prune_G;

    const size_t nt = hs.tri_attr.size();
    std::vector<HullD> th(nt);
    for (size_t t = 0; t < nt; ++t) {
        const DTriAttr &at = hs.tri_attr[t];
        th[t] = triangle_hull(&hs.vpos[3 * (size_t)at.i0], &hs.vpos[3 * (size_t)at.i1], &hs.vpos[3 * (size_t)at.i2],
                              &hs.face_normal[3 * t], G);
    }
    /* children are numbered after their parent (build_tree), so a reverse
     * sweep sees both children before the parent */
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<HullD> hull((size_t)n, HullD{{inf, inf, inf}, {-inf, -inf, -inf}});
    for (int32_t x = n - 1; x >= 0; --x) {
        HullD &h = hull[x];
        auto merge = [&](const HullD &o) {
            for (int k = 0; k < 3; ++k) {
                h.lo[k] = std::min(h.lo[k], o.lo[k]);
                h.hi[k] = std::max(h.hi[k], o.hi[k]);
            }
        };
        if (!bn[x].tris.empty()) {
            for (int32_t t : bn[x].tris) merge(th[t]);
        } else {
            for (int c = 0; c < 2; ++c)
                if (bn[x].child[c] != -1) merge(hull[bn[x].child[c]]);
        }
    }
    std::vector<int32_t> subtree((size_t)n, 1);
    for (int32_t x = n - 1; x >= 0; --x)
        if (bn[x].tris.empty())
            for (int c = 0; c < 2; ++c)
                if (bn[x].child[c] != -1) subtree[x] += subtree[bn[x].child[c]];
    /* leaf slot ranges follow the reference's order (prepare_scene's flatten) */
    std::vector<int32_t> first_slot((size_t)n, -1);
    {
        std::vector<int32_t> st{0};
        int32_t next = 0;
        while (!st.empty()) {
            const int32_t x = st.back();
            st.pop_back();
            if (!bn[x].tris.empty()) {
                first_slot[x] = next;
                next += (int32_t)bn[x].tris.size();
            } else {
                if (bn[x].child[0] != -1) st.push_back(bn[x].child[0]);
                if (bn[x].child[1] != -1) st.push_back(bn[x].child[1]);
            }
        }
    }
    hs.pnodes.assign((size_t)8 * (n + 1), PNode{});   /* + one zero record per order: successor prefetch of the last node */
    std::vector<int32_t> st;
    for (int oct = 0; oct < 8; ++oct) {
        PNode *out = hs.pnodes.data() + (size_t)oct * (n + 1);
        int32_t k = 0;
        st.assign(1, 0);
        while (!st.empty()) {
            const int32_t x = st.back();
            st.pop_back();
            PNode &o = out[k];
            o.lo_x = bn[x].bounds.lo[0]; o.lo_y = bn[x].bounds.lo[1]; o.lo_z = bn[x].bounds.lo[2];
            o.hi_x = bn[x].bounds.hi[0]; o.hi_y = bn[x].bounds.hi[1]; o.hi_z = bn[x].bounds.hi[2];
            o.tlo_x = round_down(hull[x].lo[0]); o.tlo_y = round_down(hull[x].lo[1]); o.tlo_z = round_down(hull[x].lo[2]);
            o.thi_x = round_up(hull[x].hi[0]); o.thi_y = round_up(hull[x].hi[1]); o.thi_z = round_up(hull[x].hi[2]);
            o.depth = bn[x].depth;
            o.count = (int32_t)bn[x].tris.size();
            if (bn[x].tris.empty()) {
                o.a = k + subtree[x];
                o.b = -(bn[x].depth + 1);
                /* near child first: on a negative direction along the split
                 * axis the upper half (child1) is entered first */
                const bool neg = ((oct >> (bn[x].depth % 3)) & 1) != 0;
                const int32_t near_c = bn[x].child[neg ? 1 : 0], far_c = bn[x].child[neg ? 0 : 1];
                if (far_c != -1) st.push_back(far_c);
                if (near_c != -1) st.push_back(near_c);
            } else {
                o.a = (int32_t)bn[x].tris.size() | (bn[x].depth << 24);
                o.b = first_slot[x];
            }
            ++k;
        }
    }
}

/* textures / materials / lights (crt_json.cpp:375-539, 220-247 as flattened
 * into crt_scene_desc) */
int add_shading(HostScene &hs, const crt_texture_desc *textures, int texture_count, const crt_material_desc *materials,
                int material_count, const crt_light_desc *lights, int light_count) {
    if ((texture_count > 0 && !textures) || (material_count > 0 && !materials) || (light_count > 0 && !lights))
        return set_error(CRT_E_INVALID, "null shading arrays");
    for (int i = 0; i < texture_count; ++i) {
        const crt_texture_desc &t = textures[i];
        DTexture x;
        std::memset(&x, 0, sizeof x);
        x.type = t.type;
        x.c0x = t.color0.x; x.c0y = t.color0.y; x.c0z = t.color0.z;
        x.c1x = t.color1.x; x.c1y = t.color1.y; x.c1z = t.color1.z;
        x.scalar = t.scalar;
        if (t.type < CRT_TEXTURE_ALBEDO || t.type > CRT_TEXTURE_BITMAP)
            return set_error(CRT_E_INVALID, "unknown texture type");
        if (t.type == CRT_TEXTURE_BITMAP) {
            if (!t.bitmap_rgb || t.bitmap_width <= 0 || t.bitmap_height <= 0)
                return set_error(CRT_E_INVALID, "bitmap texture without texels");
            x.w = t.bitmap_width;
            x.h = t.bitmap_height;
            x.texel_offset = (int64_t)hs.texels.size();
            for (int64_t k = 0; k < (int64_t)t.bitmap_width * t.bitmap_height; ++k)
                hs.texels.push_back(DVec4{t.bitmap_rgb[3 * k], t.bitmap_rgb[3 * k + 1], t.bitmap_rgb[3 * k + 2], 0.f});
        }
        hs.textures.push_back(x);
    }
    for (int i = 0; i < material_count; ++i) {
        const crt_material_desc &m = materials[i];
        if (m.type < CRT_MATERIAL_DIFFUSE || m.type > CRT_MATERIAL_CONSTANT)
            return set_error(CRT_E_INVALID, "unknown material type");
        if (m.type != CRT_MATERIAL_REFRACTIVE && (m.albedo_texture_index < 0 || m.albedo_texture_index >= texture_count))
            return set_error(CRT_E_INVALID, "material albedo texture index out of range");
        hs.materials.push_back(DMaterial{m.type, m.albedo_texture_index, m.ior, 0});
    }
    for (int i = 0; i < light_count; ++i)
        hs.lights.push_back(DLight{lights[i].intensity, lights[i].position.x, lights[i].position.y,
                                   lights[i].position.z});

    return CRT_OK;
}

/* The built tree (reference numbering) -> ref_* arrays, the traversal-ordered
 * DNode array with its leaf slots, and the pruned walks' PNode orders. */
int flatten_tree(const std::vector<BuildNode> &bn, HostScene &hs) {
    const int32_t n = (int32_t)bn.size();

    hs.ref_bounds.resize((size_t)n * 6);
    hs.ref_children.resize((size_t)n * 2);
    hs.ref_leaf_off.resize((size_t)n + 1);
    hs.ref_depth.resize((size_t)n);
    hs.ref_leaf_tris.clear();
    hs.leaf_count = 0;
    hs.max_depth = 0;
    hs.max_leaf_size = 0;
    for (int32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) {
            hs.ref_bounds[6 * i + k] = bn[i].bounds.lo[k];
            hs.ref_bounds[6 * i + 3 + k] = bn[i].bounds.hi[k];
        }
        hs.ref_children[2 * i] = bn[i].child[0];
        hs.ref_children[2 * i + 1] = bn[i].child[1];
        hs.ref_depth[i] = bn[i].depth;
        hs.ref_leaf_off[i] = (int64_t)hs.ref_leaf_tris.size();
        hs.ref_leaf_tris.insert(hs.ref_leaf_tris.end(), bn[i].tris.begin(), bn[i].tris.end());
        if (!bn[i].tris.empty()) {
            ++hs.leaf_count;
            hs.max_leaf_size = std::max(hs.max_leaf_size, (int32_t)bn[i].tris.size());
        }
        hs.max_depth = std::max(hs.max_depth, bn[i].depth);
    }
    hs.ref_leaf_off[n] = (int64_t)hs.ref_leaf_tris.size();

    /* ---- flatten to traversal order: preorder, child1 before child0 ---- */
    std::vector<int32_t> order;
    order.reserve(n);
    {
        std::vector<int32_t> st;
        st.push_back(0);
        while (!st.empty()) {
            const int32_t x = st.back();
            st.pop_back();
            order.push_back(x);
            if (bn[x].tris.empty()) {
                if (bn[x].child[0] != -1) st.push_back(bn[x].child[0]);
                if (bn[x].child[1] != -1) st.push_back(bn[x].child[1]);
            }
        }
    }
    std::vector<int32_t> pos(n), subtree(n, 1);
    for (int32_t k = 0; k < n; ++k) pos[order[k]] = k;
    for (int32_t k = n - 1; k >= 0; --k) {
        const int32_t x = order[k];
        if (bn[x].tris.empty())
            for (int c = 0; c < 2; ++c)
                if (bn[x].child[c] != -1) subtree[x] += subtree[bn[x].child[c]];
    }
    hs.nodes.resize(n);
    hs.slots.clear();
    hs.slot_tri.clear();
    hs.slot_cull.clear();
    hs.slots.reserve(hs.ref_leaf_tris.size());
    for (int32_t k = 0; k < n; ++k) {
        const int32_t x = order[k];
        DNode &o = hs.nodes[k];
        o.lo_x = bn[x].bounds.lo[0]; o.lo_y = bn[x].bounds.lo[1]; o.lo_z = bn[x].bounds.lo[2];
        o.hi_x = bn[x].bounds.hi[0]; o.hi_y = bn[x].bounds.hi[1]; o.hi_z = bn[x].bounds.hi[2];
        if (bn[x].tris.empty()) {
            o.a = k + subtree[x];
            o.b = -(bn[x].depth + 1);
        } else {
            if (bn[x].tris.size() >= (1u << 24) || bn[x].depth > 127)
                return set_error(CRT_E_UNSUPPORTED, "leaf too large for the node record");
            o.a = (int32_t)bn[x].tris.size() | (bn[x].depth << 24);
            o.b = (int32_t)hs.slots.size();
            for (int32_t t : bn[x].tris) {
                const DTriAttr &at = hs.tri_attr[t];
                DTriGeo g;
                g.v0x = hs.vpos[3 * (size_t)at.i0]; g.v0y = hs.vpos[3 * (size_t)at.i0 + 1]; g.v0z = hs.vpos[3 * (size_t)at.i0 + 2];
                g.v1x = hs.vpos[3 * (size_t)at.i1]; g.v1y = hs.vpos[3 * (size_t)at.i1 + 1]; g.v1z = hs.vpos[3 * (size_t)at.i1 + 2];
                g.v2x = hs.vpos[3 * (size_t)at.i2]; g.v2y = hs.vpos[3 * (size_t)at.i2 + 1]; g.v2z = hs.vpos[3 * (size_t)at.i2 + 2];
                g.nx = hs.face_normal[3 * (size_t)t]; g.ny = hs.face_normal[3 * (size_t)t + 1]; g.nz = hs.face_normal[3 * (size_t)t + 2];
                hs.slots.push_back(g);
                hs.slot_tri.push_back(t);
                hs.slot_cull.push_back(hs.tri_cull[t]);
            }
        }
    }
    if (hs.slots.size() > (size_t)std::numeric_limits<int32_t>::max())
        return set_error(CRT_E_UNSUPPORTED, "too many leaf triangle copies");
    (void)pos;
    build_pruned_nodes(bn, hs);
    return CRT_OK;
}

/* The BVH (crt_bvh.h): built on the host for every scene up to kHostBvhMax
 * triangles (camera rays take it too: walks 14 / 15).  Above that the host
 * never builds it (C5's 1 M triangles: 3.9 s); the upload builds it on the
 * device instead (crt_lbvh.hip), or, with create flag CRT_SCENE_NO_DEVICE_BVH,
 * there is none and every ray takes the exact kd walks. */
int maybe_build_bvh_(HostScene &hs);
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
int maybe_build_bvh(HostScene &hs) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = maybe_build_bvh_(hs);
    hs.bvh_ms = ms_since(t0);
    return rc;
}
int maybe_build_bvh_(HostScene &hs) {
    if (hs.tri_attr.size() > kHostBvhMax) return hs.nodes.empty() ? CRT_OK : build_proof_tables(hs);
    const int rc = build_bvh(hs);
    if (rc != CRT_OK || hs.nodes.empty()) return rc;   /* device-built tree: the proof descends it (verify_kd) */
    return build_proof_tables(hs);
}

}  // namespace

int prepare_scene_(const crt_scene_desc *d, HostScene &hs, bool build_tree_on_host);
int prepare_scene(const crt_scene_desc *d, HostScene &hs, bool build_tree_on_host) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = prepare_scene_(d, hs, build_tree_on_host);
    hs.prep_ms = ms_since(t0);
    return rc;
}

int prepare_scene_(const crt_scene_desc *d, HostScene &hs, bool build_tree_on_host) {
    if (!d) return set_error(CRT_E_INVALID, "null scene description");
    if (d->camera.width <= 0 || d->camera.height <= 0)
        return set_error(CRT_E_INVALID, "image width/height must be positive");
    if (d->bucket_size <= 0) return set_error(CRT_E_INVALID, "bucket_size must be positive");
    if (d->material_count < 0 || d->mesh_count < 0 || d->texture_count < 0 || d->light_count < 0)
        return set_error(CRT_E_INVALID, "negative element count");

    hs.background[0] = d->background_color.x;
    hs.background[1] = d->background_color.y;
    hs.background[2] = d->background_color.z;
    hs.cam_loc[0] = d->camera.location.x;
    hs.cam_loc[1] = d->camera.location.y;
    hs.cam_loc[2] = d->camera.location.z;
    std::memcpy(hs.cam_rot, d->camera.rotation, sizeof hs.cam_rot);
    hs.width = d->camera.width;
    hs.height = d->camera.height;
    /* crt_camera.h:20, crt_camera.cpp:23,26-27 — same float expressions, once. */
    hs.fov_radians = fov_degrees_to_radians(d->camera.fov_degrees);
    hs.aspect = float(hs.width) / hs.height;
    hs.tan_half_fov = std::tan(hs.fov_radians * 0.5f);
    hs.bucket_size = d->bucket_size;
    hs.gi_on = d->gi_on != 0;
    hs.reflections_on = d->reflections_on != 0;
    hs.refractions_on = d->refractions_on != 0;

    int rc = add_shading(hs, d->textures, d->texture_count, d->materials, d->material_count, d->lights,
                         d->light_count);
    if (rc != CRT_OK) return rc;

    /* ---- mesh prep (crt_mesh.cpp:10-73) ---- */
    int64_t nv = 0, nt = 0;
    for (int i = 0; i < d->mesh_count; ++i) {
        const crt_mesh_desc &m = d->meshes[i];
        if (m.vertex_count < 0 || m.index_count < 0 || m.index_count % 3 != 0 ||
            (m.vertex_count > 0 && !m.positions) || (m.index_count > 0 && !m.indices))
            return set_error(CRT_E_INVALID, "malformed mesh");
        if (m.material_index < 0 || m.material_index >= d->material_count)
            return set_error(CRT_E_INVALID, "mesh material index out of range");
        for (int64_t k = 0; k < m.index_count; ++k)
            if (m.indices[k] < 0 || m.indices[k] >= m.vertex_count)
                return set_error(CRT_E_INVALID, "mesh vertex index out of range");
        nv += m.vertex_count;
        nt += m.index_count / 3;
    }
    if (nt > (int64_t)std::numeric_limits<int32_t>::max() / 2)
        return set_error(CRT_E_UNSUPPORTED, "too many triangles");
    hs.vpos.resize((size_t)nv * 3);
    std::vector<F3> vnorm((size_t)nv, f3(0.f, 0.f, 0.f));
    hs.vuv.assign((size_t)nv, DVec4{0.f, 0.f, 0.f, 0.f});
    hs.tri_attr.resize((size_t)nt);
    hs.face_normal.resize((size_t)nt * 3);
    hs.tri_cull.resize((size_t)nt);
    int64_t vbase = 0, tbase = 0;
    for (int i = 0; i < d->mesh_count; ++i) {
        const crt_mesh_desc &m = d->meshes[i];
        const crt_material_desc &mat = d->materials[m.material_index];
        for (int64_t k = 0; k < m.vertex_count; ++k) {
            hs.vpos[3 * (vbase + k)] = m.positions[3 * k];
            hs.vpos[3 * (vbase + k) + 1] = m.positions[3 * k + 1];
            hs.vpos[3 * (vbase + k) + 2] = m.positions[3 * k + 2];
            if (m.uvs) hs.vuv[vbase + k] = DVec4{m.uvs[3 * k], m.uvs[3 * k + 1], m.uvs[3 * k + 2], 0.f};
        }
        for (int64_t k = 0; k < m.index_count; k += 3) {
            const int64_t t = tbase + k / 3;
            const int32_t a = (int32_t)(vbase + m.indices[k]);
            const int32_t b = (int32_t)(vbase + m.indices[k + 1]);
            const int32_t c = (int32_t)(vbase + m.indices[k + 2]);
            const F3 pa = f3(hs.vpos[3 * a], hs.vpos[3 * a + 1], hs.vpos[3 * a + 2]);
            const F3 pb = f3(hs.vpos[3 * b], hs.vpos[3 * b + 1], hs.vpos[3 * b + 2]);
            const F3 pc = f3(hs.vpos[3 * c], hs.vpos[3 * c + 1], hs.vpos[3 * c + 2]);
            const F3 fn = normalized3(cross3(pb - pa, pc - pa));
            hs.face_normal[3 * t] = fn.x;
            hs.face_normal[3 * t + 1] = fn.y;
            hs.face_normal[3 * t + 2] = fn.z;
            hs.tri_attr[t] = DTriAttr{a, b, c, m.material_index | (mat.smooth_shading ? (int32_t)0x80000000 : 0)};
            hs.tri_cull[t] = mat.back_face_culling ? 1 : 0;
            for (int32_t v : {a, b, c}) {
                vnorm[v].x += fn.x;
                vnorm[v].y += fn.y;
                vnorm[v].z += fn.z;
            }
        }
        vbase += m.vertex_count;
        tbase += m.index_count / 3;
        /* every vertex appended so far is re-normalised after each mesh (:27-29) */
        for (int64_t v = 0; v < vbase; ++v) vnorm[v] = normalized3(vnorm[v]);
    }
    hs.vnormal.resize((size_t)nv);
    for (int64_t v = 0; v < nv; ++v) hs.vnormal[v] = DVec4{vnorm[v].x, vnorm[v].y, vnorm[v].z, 0.f};

    /* ---- tree build (crt_acceleration_tree.cpp:87-106) ---- */
    set_prune_origin_max(hs);
    const float inf = std::numeric_limits<float>::infinity();
    Box6 root{{inf, inf, inf}, {-inf, -inf, -inf}};
    if (!build_tree_on_host) {
        /* root cell only (the same fold); the tree is built on the device */
        for (int64_t t = 0; t < nt; ++t)
            for (int32_t v : {hs.tri_attr[t].i0, hs.tri_attr[t].i1, hs.tri_attr[t].i2})
                for (int k = 0; k < 3; ++k) {
                    const float p = hs.vpos[3 * (size_t)v + k];
                    root.lo[k] = std::min(root.lo[k], p);
                    root.hi[k] = std::max(root.hi[k], p);
                }
        for (int k = 0; k < 3; ++k) {
            hs.root_box[k] = root.lo[k];
            hs.root_box[3 + k] = root.hi[k];
        }
        hs.tree_on_host = false;
        return maybe_build_bvh(hs);
    }
    const auto tb0 = std::chrono::steady_clock::now();
    std::vector<Box6> tri_boxes((size_t)nt);
    for (int64_t t = 0; t < nt; ++t) {
        Box6 b{{inf, inf, inf}, {-inf, -inf, -inf}};
        for (int32_t v : {hs.tri_attr[t].i0, hs.tri_attr[t].i1, hs.tri_attr[t].i2}) {
            for (int k = 0; k < 3; ++k) {
                const float p = hs.vpos[3 * (size_t)v + k];
                /* std::min(a,b) = (b < a) ? b : a, folded vertex by vertex (:13-22) */
                b.lo[k] = std::min(b.lo[k], p);
                b.hi[k] = std::max(b.hi[k], p);
                root.lo[k] = std::min(root.lo[k], p);
                root.hi[k] = std::max(root.hi[k], p);
            }
        }
        tri_boxes[t] = b;
    }
    for (int k = 0; k < 3; ++k) {
        hs.root_box[k] = root.lo[k];
        hs.root_box[3 + k] = root.hi[k];
    }
    std::vector<BuildNode> bn;
    build_tree(tri_boxes, root, bn);
    if ((rc = flatten_tree(bn, hs)) != CRT_OK) return rc;
    hs.tree_build_ms = ms_since(tb0);
    return maybe_build_bvh(hs);
}

/* The reference's built scene (crt_hip_scene_from_tree): vertices after
 * vertex_array_extend and the tree after acceleration_tree::build are taken as
 * they are.  Triangles get global ids in order of first appearance over the
 * leaves in the tree's own numbering (the copies of one triangle share its
 * vertex triple, material, flags and face normal — crt_acceleration_tree.cpp:
 * 44-58 copies the Triangle). */
int prepare_scene_from_tree(const crt_tree_scene_desc *d, HostScene &hs) {
    if (!d) return set_error(CRT_E_INVALID, "null scene description");
    if (d->width <= 0 || d->height <= 0) return set_error(CRT_E_INVALID, "image width/height must be positive");
    if (d->bucket_size <= 0) return set_error(CRT_E_INVALID, "bucket_size must be positive");
    if (d->material_count < 0 || d->texture_count < 0 || d->light_count < 0 || d->vertex_count < 0 ||
        d->node_count < 1 || d->node_count >= (int64_t)std::numeric_limits<int32_t>::max())
        return set_error(CRT_E_INVALID, "bad element count");
    if ((d->vertex_count > 0 && !d->vertices) || !d->node_bounds || !d->node_children || !d->leaf_offsets)
        return set_error(CRT_E_INVALID, "null scene arrays");
    hs.background[0] = d->background_color.x;
    hs.background[1] = d->background_color.y;
    hs.background[2] = d->background_color.z;
    hs.cam_loc[0] = d->camera_location.x;
    hs.cam_loc[1] = d->camera_location.y;
    hs.cam_loc[2] = d->camera_location.z;
    std::memcpy(hs.cam_rot, d->camera_rotation, sizeof hs.cam_rot);
    hs.width = d->width;
    hs.height = d->height;
    /* crt_camera.cpp:23,26-27 on the stored m_fov_radians */
    hs.fov_radians = d->fov_radians;
    hs.aspect = float(hs.width) / hs.height;
    hs.tan_half_fov = std::tan(hs.fov_radians * 0.5f);
    hs.bucket_size = d->bucket_size;
    hs.gi_on = d->gi_on != 0;
    hs.reflections_on = d->reflections_on != 0;
    hs.refractions_on = d->refractions_on != 0;
    int rc = add_shading(hs, d->textures, d->texture_count, d->materials, d->material_count, d->lights, d->light_count);
    if (rc != CRT_OK) return rc;

    const int64_t nv = d->vertex_count;
    hs.vpos.resize((size_t)nv * 3);
    hs.vnormal.resize((size_t)nv);
    hs.vuv.resize((size_t)nv);
    for (int64_t v = 0; v < nv; ++v) {
        const float *x = d->vertices + 9 * v;
        hs.vpos[3 * v] = x[0]; hs.vpos[3 * v + 1] = x[1]; hs.vpos[3 * v + 2] = x[2];
        hs.vnormal[v] = DVec4{x[3], x[4], x[5], 0.f};
        hs.vuv[v] = DVec4{x[6], x[7], x[8], 0.f};
    }

    const int32_t n = (int32_t)d->node_count;
    if (d->leaf_offsets[0] != 0) return set_error(CRT_E_INVALID, "leaf_offsets[0] must be 0");
    for (int32_t i = 0; i < n; ++i)
        if (d->leaf_offsets[i + 1] < d->leaf_offsets[i]) return set_error(CRT_E_INVALID, "leaf_offsets not ascending");
    const int64_t m = d->leaf_offsets[n];
    if (m > 0 && !d->leaf_triangles) return set_error(CRT_E_INVALID, "null leaf triangles");
    std::vector<BuildNode> bn((size_t)n);
    std::vector<uint8_t> seen((size_t)n, 0);
    seen[0] = 1;
    struct Key {
        int32_t v[3], mat, flags;
        bool operator<(const Key &o) const {
            return std::lexicographical_compare(&v[0], &v[0] + 5, &o.v[0], &o.v[0] + 5);
        }
    };
    static_assert(sizeof(Key) == 5 * sizeof(int32_t), "Key must be packed");
    std::map<Key, int32_t> ids;
    for (int32_t i = 0; i < n; ++i) {
        BuildNode &b = bn[i];
        for (int k = 0; k < 3; ++k) {
            b.bounds.lo[k] = d->node_bounds[6 * (size_t)i + k];
            b.bounds.hi[k] = d->node_bounds[6 * (size_t)i + 3 + k];
        }
        if (!seen[i]) return set_error(CRT_E_INVALID, "tree node unreachable from the root");
        const int64_t f = d->leaf_offsets[i], e = d->leaf_offsets[i + 1];
        for (int c = 0; c < 2; ++c) {
            const int32_t ch = d->node_children[2 * (size_t)i + c];
            if (ch == -1) continue;
            if (ch <= i || ch >= n || seen[ch])
                return set_error(CRT_E_INVALID, "tree children must be numbered after their parent, once");
            if (f != e) return set_error(CRT_E_INVALID, "a leaf (node with triangles) has children");
            seen[ch] = 1;
            b.child[c] = ch;
            bn[ch].depth = b.depth + 1;
            if (bn[ch].depth > 62)   /* the walks keep one reach bit per depth in 64-bit masks */
                return set_error(CRT_E_UNSUPPORTED, "tree deeper than 62 levels (the reference builds at most 40)");
        }
        if (f == e && b.child[0] == -1 && b.child[1] == -1 && n > 1)
            return set_error(CRT_E_INVALID, "interior node without children");
        for (int64_t k = f; k < e; ++k) {
            const crt_tree_triangle &t = d->leaf_triangles[k];
            for (int j = 0; j < 3; ++j)
                if (t.v[j] < 0 || t.v[j] >= nv) return set_error(CRT_E_INVALID, "triangle vertex index out of range");
            if (t.material_index < 0 || t.material_index >= d->material_count)
                return set_error(CRT_E_INVALID, "triangle material index out of range");
            const Key key{{t.v[0], t.v[1], t.v[2]}, t.material_index, t.flags & 3};
            auto it = ids.find(key);
            int32_t id;
            if (it == ids.end()) {
                id = (int32_t)hs.tri_attr.size();
                ids.emplace(key, id);
                hs.tri_attr.push_back(DTriAttr{t.v[0], t.v[1], t.v[2],
                                               t.material_index | ((t.flags & 1) ? (int32_t)0x80000000 : 0)});
                hs.face_normal.insert(hs.face_normal.end(), t.face_normal, t.face_normal + 3);
                hs.tri_cull.push_back((t.flags & 2) ? 1 : 0);
            } else {
                id = it->second;
            }
            b.tris.push_back(id);
        }
    }
    set_prune_origin_max(hs);
    for (int k = 0; k < 3; ++k) {
        hs.root_box[k] = bn[0].bounds.lo[k];
        hs.root_box[3 + k] = bn[0].bounds.hi[k];
    }
    if ((rc = flatten_tree(bn, hs)) != CRT_OK) return rc;
    return maybe_build_bvh(hs);
}

DCamera host_camera(const HostScene &hs) {
    DCamera c{};
    std::memcpy(c.loc, hs.cam_loc, sizeof c.loc);
    std::memcpy(c.rot, hs.cam_rot, sizeof c.rot);
    c.width = hs.width;
    c.height = hs.height;
    c.aspect = hs.aspect;
    c.tan_half_fov = hs.tan_half_fov;
    return c;
}

bool make_camera(const float loc[3], const float rot[9], float fov_radians, int32_t width, int32_t height,
                 DCamera &out) {
    if (width <= 0 || height <= 0) return false;
    std::memcpy(out.loc, loc, sizeof out.loc);
    std::memcpy(out.rot, rot, sizeof out.rot);
    out.width = width;
    out.height = height;
    /* crt_camera.cpp:23,26-27 — the same float expressions prepare_scene uses */
    out.aspect = float(width) / height;
    out.tan_half_fov = std::tan(fov_radians * 0.5f);
    return true;
}

std::vector<float> tile_work_estimate(const HostScene &hs, int tiles_x, int tiles_y) {
    return tile_work_estimate_of(host_camera(hs), hs.ref_bounds, hs.ref_children, hs.ref_leaf_off, tiles_x, tiles_y);
}

std::vector<float> tile_work_estimate_of(const DCamera &cam, const std::vector<float> &ref_bounds,
                                         const std::vector<int32_t> &ref_children,
                                         const std::vector<int64_t> &ref_leaf_off, int tiles_x, int tiles_y) {
    std::vector<float> w((size_t)tiles_x * tiles_y, 0.f);
    const size_t n = ref_children.size() / 2;
    if (ref_leaf_off.size() < n + 1 || ref_bounds.size() < 6 * n) return w;
    const float *R = cam.rot;
    const float sx = cam.aspect * cam.tan_half_fov, sy = cam.tan_half_fov;
    for (size_t i = 0; i < n; ++i) {
        const int64_t cnt = ref_leaf_off[i + 1] - ref_leaf_off[i];
        if (cnt == 0) continue;
        const float *b = &ref_bounds[6 * i];
        float x0 = 1e30f, x1 = -1e30f, y0 = 1e30f, y1 = -1e30f;
        bool behind = false;
        for (int c = 0; c < 8; ++c) {
            const float v[3] = {b[(c & 1) ? 3 : 0] - cam.loc[0], b[(c & 2) ? 4 : 1] - cam.loc[1],
                                b[(c & 4) ? 5 : 2] - cam.loc[2]};
            /* camera space = world * R^T (ray dir = cam * R, crt_camera.cpp:31) */
            const float cx = v[0] * R[0] + v[1] * R[1] + v[2] * R[2];
            const float cy = v[0] * R[3] + v[1] * R[4] + v[2] * R[5];
            const float cz = v[0] * R[6] + v[1] * R[7] + v[2] * R[8];
            if (!(cz < -1e-6f)) { behind = true; break; }
            const float px = (cx / -cz / sx + 1.0f) * 0.5f * cam.width;
            const float py = (1.0f - cy / -cz / sy) * 0.5f * cam.height;
            x0 = std::min(x0, px); x1 = std::max(x1, px);
            y0 = std::min(y0, py); y1 = std::max(y1, py);
        }
        int tx0 = 0, tx1 = tiles_x - 1, ty0 = 0, ty1 = tiles_y - 1;
        if (!behind) {
            if (x1 < 0 || y1 < 0 || x0 >= cam.width || y0 >= cam.height) continue;
            tx0 = std::max(0, (int)(x0 / 8)); tx1 = std::min(tiles_x - 1, (int)(x1 / 8));
            ty0 = std::max(0, (int)(y0 / 8)); ty1 = std::min(tiles_y - 1, (int)(y1 / 8));
        }
        const float add = (float)cnt;
        for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) w[(size_t)ty * tiles_x + tx] += add;
    }
    return w;
}

std::vector<DBucket> shard_buckets(int32_t width, int32_t height, int32_t bucket_size, int shard,
                                   int shard_count, int64_t *packed_pixels) {
    std::vector<DBucket> out;
    /* crt_renderer.cpp:160-174: counts round half up, the last row/column absorbs the rest */
    const int nx = static_cast<int>(float(width) / bucket_size + 0.5);
    const int ny = static_cast<int>(float(height) / bucket_size + 0.5);
    int64_t off = 0;
    int64_t k = 0;
    for (int by = 0; by < ny; ++by) {
        const int y = by * bucket_size;
        const int h = by == ny - 1 ? height - y : bucket_size;
        for (int bx = 0; bx < nx; ++bx, ++k) {
            const int x = bx * bucket_size;
            const int w = bx == nx - 1 ? width - x : bucket_size;
            if (k % shard_count != shard) continue;
            if (w <= 0 || h <= 0) continue;
            out.push_back(DBucket{x, y, w, h, off});
            off += (int64_t)w * h;
        }
    }
    if (packed_pixels) *packed_pixels = off;
    return out;
}

/* Live tiles of a shard: each bucket of the shard cut into 8x8 tiles from the
 * bucket's origin (the render plan's own tiling), kept when some pixel of the
 * tile is live (mask null: all live), packed back to back.  Dead tiles are the
 * frame's background by construction (see crt_hip_compact_*). */
std::vector<DBucket> shard_live_tiles(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                                      const uint8_t *live, int64_t *packed_pixels, std::vector<DBucket> *dead) {
    std::vector<DBucket> out;
    int64_t px = 0, off = 0;
    for (const DBucket &b : shard_buckets(width, height, bucket_size, shard, shard_count, &px)) {
        for (int ty = 0; ty < b.h; ty += 8)
            for (int tx = 0; tx < b.w; tx += 8) {
                const int x = b.x + tx, y = b.y + ty, w = std::min(8, b.w - tx), h = std::min(8, b.h - ty);
                bool any = live == nullptr;
                for (int yy = 0; yy < h && !any; ++yy)
                    for (int xx = 0; xx < w && !any; ++xx) any = live[(size_t)(y + yy) * width + x + xx] != 0;
                if (any) {
                    out.push_back(DBucket{x, y, w, h, off});
                    off += (int64_t)w * h;
                } else if (dead) {
                    dead->push_back(DBucket{x, y, w, h, -1});
                }
            }
    }
    if (packed_pixels) *packed_pixels = off;
    return out;
}

}  // namespace crt_amd

using namespace crt_amd;

extern "C" {

const char *crt_hip_last_error(void) { return g_last_error.c_str(); }
int crt_hip_abi_version(void) { return CRT_HIP_ABI_VERSION; }

void crt_renderer_settings_default(crt_renderer_settings *out) {
    if (!out) return;
    out->max_ray_depth = 3;                      /* crt_renderer.h:10 */
    out->diffuse_reflection_ray_count = 4;       /* :11 */
    out->shadow_bias = 1e-2f;                    /* :13-16 */
    out->reflection_bias = 1e-2f;
    out->diffuse_reflection_bias = 1e-2f;
    out->refraction_bias = 1e-2f;
}

int crt_host_scene_create(const crt_scene_desc *desc, crt_host_scene **out) {
    if (!out) return set_error(CRT_E_INVALID, "null output");
    *out = nullptr;
    std::unique_ptr<HostScene> hs(new HostScene());
    const int rc = prepare_scene(desc, *hs);
    if (rc != CRT_OK) return rc;
    *out = reinterpret_cast<crt_host_scene *>(hs.release());
    return CRT_OK;
}

int crt_host_scene_info(const crt_host_scene *h, crt_scene_info *out) {
    if (!h || !out) return set_error(CRT_E_INVALID, "null argument");
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    std::memset(out, 0, sizeof *out);
    out->triangle_count = (int64_t)hs.tri_attr.size();
    out->vertex_count = (int64_t)hs.vnormal.size();
    out->node_count = (int64_t)hs.nodes.size();
    out->leaf_count = hs.leaf_count;
    out->leaf_ref_count = (int64_t)hs.slots.size();
    out->max_depth = hs.max_depth;
    out->max_leaf_size = hs.max_leaf_size;
    out->width = hs.width;
    out->height = hs.height;
    out->bucket_size = hs.bucket_size;
    out->gi_on = hs.gi_on;
    out->reflections_on = hs.reflections_on;
    out->refractions_on = hs.refractions_on;
    out->tree_build_ms = hs.tree_build_ms;
    out->prep_ms = hs.prep_ms;
    out->bvh_ms = hs.bvh_ms;
    return CRT_OK;
}

int crt_host_scene_tree(const crt_host_scene *h, float *bounds, int32_t *children, int64_t *leaf_offsets,
                        int32_t *leaf_tris) {
    if (!h) return set_error(CRT_E_INVALID, "null argument");
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    if (bounds) std::memcpy(bounds, hs.ref_bounds.data(), hs.ref_bounds.size() * sizeof(float));
    if (children) std::memcpy(children, hs.ref_children.data(), hs.ref_children.size() * sizeof(int32_t));
    if (leaf_offsets) std::memcpy(leaf_offsets, hs.ref_leaf_off.data(), hs.ref_leaf_off.size() * sizeof(int64_t));
    if (leaf_tris) std::memcpy(leaf_tris, hs.ref_leaf_tris.data(), hs.ref_leaf_tris.size() * sizeof(int32_t));
    return CRT_OK;
}

int crt_host_scene_vertex_normals(const crt_host_scene *h, float *out) {
    if (!h || !out) return set_error(CRT_E_INVALID, "null argument");
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    for (size_t i = 0; i < hs.vnormal.size(); ++i) {
        out[3 * i] = hs.vnormal[i].x; out[3 * i + 1] = hs.vnormal[i].y; out[3 * i + 2] = hs.vnormal[i].z;
    }
    return CRT_OK;
}

int crt_host_scene_face_normals(const crt_host_scene *h, float *out) {
    if (!h || !out) return set_error(CRT_E_INVALID, "null argument");
    const HostScene &hs = *reinterpret_cast<const HostScene *>(h);
    std::memcpy(out, hs.face_normal.data(), hs.face_normal.size() * sizeof(float));
    return CRT_OK;
}

int crt_host_scene_from_tree(const crt_tree_scene_desc *desc, crt_host_scene **out) {
    if (!out) return set_error(CRT_E_INVALID, "null output");
    *out = nullptr;
    std::unique_ptr<HostScene> hs(new HostScene());
    const int rc = prepare_scene_from_tree(desc, *hs);
    if (rc != CRT_OK) return rc;
    *out = reinterpret_cast<crt_host_scene *>(hs.release());
    return CRT_OK;
}

void crt_host_scene_destroy(crt_host_scene *h) { delete reinterpret_cast<HostScene *>(h); }

int64_t crt_shard_compact_plan(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                               const uint8_t *live_mask, int64_t *tiles_out, int64_t cap) {
    if (width <= 0 || height <= 0 || bucket_size <= 0 || shard_count <= 0 || shard < 0 || shard >= shard_count)
        return set_error(CRT_E_INVALID, "bad shard plan arguments");
    int64_t px = 0;
    const std::vector<DBucket> t = shard_live_tiles(width, height, bucket_size, shard, shard_count, live_mask, &px,
                                                    nullptr);
    for (size_t i = 0; i < t.size() && (int64_t)i < cap && tiles_out; ++i) {
        int64_t *o = tiles_out + 5 * i;
        o[0] = t[i].x; o[1] = t[i].y; o[2] = t[i].w; o[3] = t[i].h; o[4] = t[i].packed_offset;
    }
    return (int64_t)t.size();
}

int64_t crt_shard_plan(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                       int64_t *buckets_out, int64_t cap) {
    if (width <= 0 || height <= 0 || bucket_size <= 0 || shard_count <= 0 || shard < 0 || shard >= shard_count)
        return set_error(CRT_E_INVALID, "bad shard plan arguments");
    int64_t px = 0;
    const std::vector<DBucket> b = shard_buckets(width, height, bucket_size, shard, shard_count, &px);
    const int nx = static_cast<int>(float(width) / bucket_size + 0.5);
    for (size_t i = 0; i < b.size() && (int64_t)i < cap; ++i) {
        int64_t *o = buckets_out + 6 * i;
        o[0] = b[i].x; o[1] = b[i].y; o[2] = b[i].w; o[3] = b[i].h; o[4] = b[i].packed_offset;
        o[5] = (int64_t)(b[i].y / bucket_size) * nx + b[i].x / bucket_size;
    }
    return (int64_t)b.size();
}

}  // extern "C"
