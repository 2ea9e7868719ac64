/*
 * crt_oracle.cpp — CPU ORACLE (test infrastructure, NOT product code).
 *
 * A from-scratch C++ restatement of the reference render path of
 * bvpav/chaos-ray-tracing-course-2025 @ HEAD, written to reproduce its fp32
 * results bit for bit.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * Pinning: tests/test_oracle_ref.py checks this restatement against the
 * reference's own translation units (crt_intersection.cpp, crt_acceleration_tree.cpp,
 * crt_mesh.cpp, crt_camera.cpp, crt_matrix.cpp, crt_vector.cpp, crt_image_ppm.cpp)
 * compiled from /root/reference by oracle/Makefile into oracle/_ref/ (tree
 * topology, per-ray intersections, camera rays, vertex normals, PPM bytes),
 * and against the committed fixtures in tests/golden/ (which were produced
 * the same way, so they also pin it where /root/reference is absent).
 * crt_renderer.cpp and crt_texture.cpp need C++23 std::unreachable, which the
 * container's libstdc++ 11 lacks: they are not built, so shade_ray below is
 * pinned only through the hot path it calls and the coverage masks of the
 * reference's committed PNGs (parity of the shading arithmetic itself is
 * by line-by-line restatement).
 *
 * Build: g++ -O3 -std=c++17 -ffp-contract=off (x86-64 SSE2, no FMA — like the
 * reference's Release build, Makefile:7,13, CMakeLists.txt:5-7).
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

#include "../include/crt_hip.h"

namespace oracle {

/* ---- crt_vector.h:7-137 -------------------------------------------- */
struct V3 { float x, y, z; };

static inline V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 scale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
/* crt_vector.h:76-78 — the reference's Vector*Vector multiplies y twice. */
static inline V3 mul_quirk(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y * a.y, a.z * b.z); }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float len_sq(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float len(V3 a) { return std::sqrt(len_sq(a)); }              /* crt_vector.cpp:7-9 */
static inline V3 unit(V3 a) { return divs(a, len(a)); }                      /* crt_vector.h:98-105 */
static inline float comp(V3 a, int k) { return k == 0 ? a.x : (k == 1 ? a.y : a.z); }

/* crt_matrix.h:66-74: row vector times row-major matrix, accumulated from 0. */
static inline V3 vec_mat(V3 v, const float m[9]) {
    float r[3];
    const float in[3] = {v.x, v.y, v.z};
    for (int i = 0; i < 3; ++i) {
        float acc = 0.0f;
        for (int j = 0; j < 3; ++j) acc += in[j] * m[j * 3 + i];
        r[i] = acc;
    }
    return v3(r[0], r[1], r[2]);
}

/* ---- scene types (crt_vertex.h, crt_triangle.h, crt_aabb.h) ---------- */
struct Vert { V3 pos, nrm, uv; };
struct Tri {
    int32_t i0, i1, i2;   /* global vertex ids (the reference keeps pointers) */
    V3 fn;                /* crt_triangle.h:25-33 */
    int32_t mat;
    bool smooth, cull;
    int32_t id;           /* global triangle id */
};
struct Box { V3 lo, hi; };
struct Node {
    std::vector<int32_t> tris;   /* triangle ids; leaf iff non-empty (crt_acceleration_tree.h:21-23) */
    Box bounds;
    int32_t child[2];
    int32_t parent;
    int32_t depth;
};

struct Texture {
    int32_t type;
    V3 c0, c1;
    float s;
    int32_t w, h;
    std::vector<V3> texels;
};
struct Material { int32_t type, tex; float ior; };
struct Light { float intensity; V3 pos; };

struct Scene {
    V3 background;
    V3 cam_loc;
    float cam_rot[9];
    int32_t width, height;
    float fov_rad;
    int32_t bucket;
    bool gi, refl, refr;
    std::vector<Vert> verts;
    std::vector<Tri> tris;
    std::vector<Node> nodes;
    std::vector<Texture> textures;
    std::vector<Material> materials;
    std::vector<Light> lights;
    /* oracle_set_shadows: trace each light's shadow ray (the course's earlier
     * renderer; dead code at HEAD, crt_renderer.cpp:29-44) */
    bool shadows = false;
};

struct Counters { uint64_t traversals = 0, nodes = 0, tris = 0, hits = 0; };

struct Hit {
    float t;
    V3 p, n, uv;
    float bu, bv;
    int32_t mat;
    int32_t tri;
};

struct Ray { V3 o, d; int depth; };

/* ---- mesh prep: crt_mesh.cpp:10-73 ------------------------------------ */
static void append_mesh(Scene &sc, const crt_mesh_desc &m, const crt_material_desc &mat) {
    const int32_t base = (int32_t)sc.verts.size();
    for (int64_t i = 0; i < m.vertex_count; ++i) {
        Vert v;
        v.pos = v3(m.positions[3 * i], m.positions[3 * i + 1], m.positions[3 * i + 2]);
        v.nrm = v3(0.f, 0.f, 0.f);
        v.uv = m.uvs ? v3(m.uvs[3 * i], m.uvs[3 * i + 1], m.uvs[3 * i + 2]) : v3(0.f, 0.f, 0.f);
        sc.verts.push_back(v);
    }
    for (int64_t k = 0; k + 2 < m.index_count; k += 3) {
        Tri t;
        t.i0 = base + m.indices[k];
        t.i1 = base + m.indices[k + 1];
        t.i2 = base + m.indices[k + 2];
        const V3 a = sc.verts[t.i0].pos, b = sc.verts[t.i1].pos, c = sc.verts[t.i2].pos;
        t.fn = unit(cross(sub(b, a), sub(c, a)));
        t.mat = m.material_index;
        t.smooth = mat.smooth_shading != 0;
        t.cull = mat.back_face_culling != 0;
        t.id = (int32_t)sc.tris.size();
        sc.tris.push_back(t);
        /* accumulate the unweighted face normal into each corner (crt_mesh.cpp:19-23) */
        for (int32_t vi : {t.i0, t.i1, t.i2}) {
            V3 &n = sc.verts[vi].nrm;
            n.x += t.fn.x; n.y += t.fn.y; n.z += t.fn.z;
        }
    }
    /* every vertex so far is re-normalised after each mesh (crt_mesh.cpp:27-29) */
    for (Vert &v : sc.verts) v.nrm = unit(v.nrm);
}

/* ---- tree build: crt_acceleration_tree.cpp:13-106, crt_aabb.h:17-45 ---- */
static const int kMaxDepth = 39;
static const size_t kMaxLeaf = 16;

static Box tri_box(const Scene &sc, const Tri &t) {
    const float inf = std::numeric_limits<float>::infinity();
    Box b{v3(inf, inf, inf), v3(-inf, -inf, -inf)};
    for (int32_t vi : {t.i0, t.i1, t.i2}) {
        const V3 p = sc.verts[vi].pos;
        b.lo.x = std::min(b.lo.x, p.x); b.lo.y = std::min(b.lo.y, p.y); b.lo.z = std::min(b.lo.z, p.z);
        b.hi.x = std::max(b.hi.x, p.x); b.hi.y = std::max(b.hi.y, p.y); b.hi.z = std::max(b.hi.z, p.z);
    }
    return b;
}

static float &axis_ref(V3 &v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

static bool boxes_touch(const Box &cell, const Box &b) {     /* crt_aabb.h:37-45 */
    for (int k = 0; k < 3; ++k) {
        if (comp(b.lo, k) > comp(cell.hi, k)) return false;
        if (comp(b.hi, k) < comp(cell.lo, k)) return false;
    }
    return true;
}

static void build_node(Scene &sc, int32_t idx, std::vector<int32_t> ids, int depth) {
    sc.nodes[idx].depth = depth;
    if (depth > kMaxDepth || ids.size() <= kMaxLeaf) {
        sc.nodes[idx].tris = std::move(ids);
        return;
    }
    const int axis = depth % 3;
    Box lo_cell = sc.nodes[idx].bounds, hi_cell = sc.nodes[idx].bounds;
    const float mid = (comp(lo_cell.lo, axis) + comp(lo_cell.hi, axis)) * 0.5f;
    axis_ref(lo_cell.hi, axis) = mid;
    axis_ref(hi_cell.lo, axis) = mid;

    std::vector<int32_t> left, right;
    for (int32_t id : ids) {
        const Box tb = tri_box(sc, sc.tris[id]);
        const bool in_l = boxes_touch(lo_cell, tb);
        const bool in_r = boxes_touch(hi_cell, tb);
        if (in_l) left.push_back(id);
        if (in_r) right.push_back(id);
    }
    if (!left.empty()) {
        const int32_t c = (int32_t)sc.nodes.size();
        sc.nodes.push_back(Node{{}, lo_cell, {-1, -1}, idx, depth + 1});
        sc.nodes[idx].child[0] = c;
        build_node(sc, c, std::move(left), depth + 1);
    }
    if (!right.empty()) {
        const int32_t c = (int32_t)sc.nodes.size();
        sc.nodes.push_back(Node{{}, hi_cell, {-1, -1}, idx, depth + 1});
        sc.nodes[idx].child[1] = c;
        build_node(sc, c, std::move(right), depth + 1);
    }
}

static void build_tree(Scene &sc) {
    const float inf = std::numeric_limits<float>::infinity();
    Box root{v3(inf, inf, inf), v3(-inf, -inf, -inf)};
    std::vector<int32_t> ids(sc.tris.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        ids[i] = (int32_t)i;
        /* vertex by vertex, as union_triangle_aabb folds (crt_acceleration_tree.cpp:13-22,89-94) */
        const Tri &t = sc.tris[i];
        for (int32_t vi : {t.i0, t.i1, t.i2}) {
            const V3 p = sc.verts[vi].pos;
            root.lo.x = std::min(root.lo.x, p.x); root.lo.y = std::min(root.lo.y, p.y);
            root.lo.z = std::min(root.lo.z, p.z); root.hi.x = std::max(root.hi.x, p.x);
            root.hi.y = std::max(root.hi.y, p.y); root.hi.z = std::max(root.hi.z, p.z);
        }
    }
    sc.nodes.clear();
    sc.nodes.push_back(Node{{}, root, {-1, -1}, -1, 0});
    build_node(sc, 0, std::move(ids), 0);
}

/* ---- hot path: crt_intersection.cpp ----------------------------------- */
static inline V3 ray_at(const Ray &r, float t) { return add(r.o, scale(r.d, t)); }   /* crt_ray.h:13-15 */

/* crt_intersection.cpp:14-45 — six face planes, first containing face wins. */
static bool hits_box(const Ray &r, const Box &b) {
    static const int U[3] = {1, 2, 0}, W[3] = {2, 0, 1};
    for (int e = 0; e < 2; ++e) {
        const V3 plane = e == 0 ? b.lo : b.hi;
        for (int a = 0; a < 3; ++a) {
            const float da = comp(r.d, a);
            if (std::fabs(da) < 1e-6f) continue;
            const float t = (comp(plane, a) - comp(r.o, a)) / da;
            if (t < 0.0f) continue;
            const V3 p = ray_at(r, t);
            const int u = U[a], w = W[a];
            if (comp(p, u) >= comp(b.lo, u) && comp(p, u) <= comp(b.hi, u) &&
                comp(p, w) >= comp(b.lo, w) && comp(p, w) <= comp(b.hi, w))
                return true;
        }
    }
    return false;
}

/* crt_intersection.cpp:47-93 */
static bool hit_triangle(const Scene &sc, const Ray &r, const Tri &t, Hit &out) {
    const Vert &A = sc.verts[t.i0], &B = sc.verts[t.i1], &C = sc.verts[t.i2];
    const V3 e0 = sub(B.pos, A.pos), e1 = sub(C.pos, B.pos), e2 = sub(A.pos, C.pos);
    const float rn = dot(t.fn, r.d);
    if (std::fabs(rn) < 1e-6f) return false;
    const float op = dot(t.fn, sub(A.pos, r.o));
    const bool front = op < 0.0f;
    if (!(front || !t.cull)) return false;
    const float dist = op / rn;
    if (dist < 0.0f) return false;
    const V3 p = ray_at(r, dist);
    const V3 ap = sub(p, A.pos), bp = sub(p, B.pos), cp = sub(p, C.pos);
    if (!(dot(t.fn, cross(e0, ap)) >= 0.0f && dot(t.fn, cross(e1, bp)) >= 0.0f &&
          dot(t.fn, cross(e2, cp)) >= 0.0f))
        return false;
    const V3 ab = e0, ac = neg(e2);
    const float bu = len(cross(ap, ac)) / len(cross(ab, ac));
    const float bv = len(cross(ab, ap)) / len(cross(ab, ac));
    const V3 sn = add(add(scale(B.nrm, bu), scale(C.nrm, bv)), scale(A.nrm, 1 - bu - bv));
    out.t = dist;
    out.p = p;
    out.n = t.smooth ? sn : t.fn;
    out.uv = add(add(scale(B.uv, bu), scale(C.uv, bv)), scale(A.uv, 1.0f - bu - bv));
    out.bu = bu;
    out.bv = bv;
    out.mat = t.mat;
    out.tri = t.id;
    return true;
}

/* crt_intersection.cpp:109-136 (+ span scan :95-107): LIFO walk from the root,
 * child0 pushed before child1, no pruning, strict '<' keeps the first found. */
static bool closest_hit(const Scene &sc, const Ray &r, Hit &best, Counters &cnt) {
    bool found = false;
    ++cnt.traversals;
    if (sc.nodes.empty()) return false;
    std::vector<int32_t> todo;
    todo.reserve(64);
    todo.push_back(0);
    while (!todo.empty()) {
        const Node &nd = sc.nodes[todo.back()];
        todo.pop_back();
        ++cnt.nodes;
        if (!hits_box(r, nd.bounds)) continue;
        if (!nd.tris.empty()) {
            bool leaf_found = false;
            Hit leaf_best{};
            for (int32_t id : nd.tris) {
                Hit h;
                ++cnt.tris;
                if (hit_triangle(sc, r, sc.tris[id], h) && (!leaf_found || h.t < leaf_best.t)) {
                    leaf_best = h;
                    leaf_found = true;
                }
            }
            if (leaf_found && (!found || leaf_best.t < best.t)) {
                best = leaf_best;
                found = true;
            }
        } else {
            if (nd.child[0] != -1) todo.push_back(nd.child[0]);
            if (nd.child[1] != -1) todo.push_back(nd.child[1]);
        }
    }
    if (found) ++cnt.hits;
    return found;
}

/* ---- camera: crt_camera.cpp:7-35 ------------------------------------- */
static Ray camera_ray(const Scene &sc, int x, int y) {
    V3 d = v3(x + 0.5f, y + 0.5f, 0.0f);
    d.x /= sc.width;
    d.y /= sc.height;
    d.x = (2.0f * d.x) - 1.0f;
    d.y = 1.0f - (2.0f * d.y);
    d.x *= float(sc.width) / sc.height;
    d.x *= std::tan(sc.fov_rad * 0.5f);
    d.y *= std::tan(sc.fov_rad * 0.5f);
    d.z = -1.0f;
    d = vec_mat(d, sc.cam_rot);
    d = unit(d);
    Ray r;
    r.o = sc.cam_loc;
    r.d = d;
    r.depth = 0;
    return r;
}

/* ---- RNG: crt_random.h:10-43 ----------------------------------------- */
struct Pcg {
    uint64_t state, inc;
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    float uniform() {
        const uint32_t bits = 0x3f800000u | (next() >> 9);
        float f;
        std::memcpy(&f, &bits, 4);
        return f - 1.0f;
    }
};
static Pcg pixel_rng(uint32_t x, uint32_t y) {
    const uint64_t seed = ((uint64_t)x << 32) | y;
    Pcg g;
    g.state = 0;
    g.inc = (seed << 1) | 1;
    (void)g.next();
    g.state += seed;
    (void)g.next();
    return g;
}

/* ---- texture: crt_texture.cpp:9-49 ------------------------------------ */
static int x86_trunc(float f) {      /* cvttss2si: out of range / NaN → INT_MIN */
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int)f;
    return std::numeric_limits<int>::min();
}
static V3 sample(const Texture &tx, V3 uv, float bu, float bv) {
    switch (tx.type) {
    case CRT_TEXTURE_ALBEDO: return tx.c0;
    case CRT_TEXTURE_EDGES:
        if (bu <= tx.s || bv <= tx.s || (1.0f - bu - bv) <= tx.s) return tx.c0;
        return tx.c1;
    case CRT_TEXTURE_CHECKER: {
        const int row = x86_trunc(uv.x / tx.s);
        const int col = x86_trunc(uv.y / tx.s);
        return ((row + col) & 1) ? tx.c1 : tx.c0;
    }
    default: {
        int rx = x86_trunc(uv.x * tx.w) % tx.w;
        int ry = x86_trunc((1.0f - uv.y) * tx.h) % tx.h;
        if (rx < 0) rx += tx.w;      /* reference reads out of bounds here (UB) */
        if (ry < 0) ry += tx.h;
        return tx.texels[(size_t)ry * tx.w + rx];
    }
    }
}

/* ---- shading: crt_renderer.cpp:46-145 --------------------------------- */
static V3 rotation_y_mul(V3 v, float ang) {    /* crt_matrix.cpp:14-20 then crt_matrix.h:66-74 */
    const float c = std::cos(ang), s = std::sin(ang);
    const float m[9] = {c, 0.0f, -s, 0.0f, 1.0f, 0.0f, s, 0.0f, c};
    return vec_mat(v, m);
}

static V3 shade(const Scene &sc, const Ray &ray, const crt_renderer_settings &st, Pcg &rng,
                Counters &cnt) {
    if ((uint32_t)ray.depth > st.max_ray_depth) return v3(0.f, 0.f, 0.f);
    Hit h;
    if (!closest_hit(sc, ray, h, cnt)) return sc.background;
    const Material &m = sc.materials[h.mat];
    V3 n = h.n;
    switch (m.type) {
    case CRT_MATERIAL_DIFFUSE: {
        V3 acc = v3(0.f, 0.f, 0.f);
        if (sc.gi) {
            for (int i = 0; i < (int)st.diffuse_reflection_ray_count; ++i) {
                const V3 right = unit(cross(ray.d, n));
                const V3 fwd = cross(right, n);
                const float basis[9] = {right.x, right.y, right.z, n.x, n.y, n.z, fwd.x, fwd.y, fwd.z};
                const float a_xy = 3.14159265358979323846f * rng.uniform();
                V3 dir = v3(std::cos(a_xy), std::sin(a_xy), 0.0f);
                const float a_xz = 2.0f * 3.14159265358979323846f * rng.uniform();
                dir = rotation_y_mul(dir, a_xz);
                dir = vec_mat(dir, basis);
                Ray child;
                child.o = add(h.p, scale(n, st.diffuse_reflection_bias));
                child.d = dir;
                child.depth = ray.depth + 1;
                const V3 c = shade(sc, child, st, rng, cnt);
                acc.x += c.x; acc.y += c.y; acc.z += c.z;
            }
        }
        const V3 alb = sample(sc.textures[m.tex], h.uv, h.bu, h.bv);
        for (const Light &L : sc.lights) {
            V3 ld = sub(L.pos, h.p);
            const float r2 = len_sq(ld);
            ld = unit(ld);
            const float dn = dot(ld, n);
            const float cos_law = (0.0f < dn) ? dn : 0.0f;       /* std::max(0.0f, dn) */
            const float area = 4 * 3.14159265358979323846f * r2;
            /* shadow ray: trace_ray_with_refractions never loops (crt_renderer.cpp:29-44),
             * so at HEAD every light counts as unoccluded.  With sc.shadows the loop
             * body runs: it always intersects the unchanged shadow ray, so the
             * result is that ray's closest hit (:90-92). */
            if (sc.shadows) {
                Ray sr;
                sr.o = add(h.p, scale(n, st.shadow_bias));
                sr.d = ld;
                sr.depth = 0;
                Hit sh;
                if (closest_hit(sc, sr, sh, cnt) && !(sh.t * sh.t > r2)) continue;
            }
            const V3 term = scale(divs(scale(alb, L.intensity), area), cos_law);
            acc.x += term.x; acc.y += term.y; acc.z += term.z;
        }
        const float k = (float)(st.diffuse_reflection_ray_count + 1);
        acc.x /= k; acc.y /= k; acc.z /= k;
        return acc;
    }
    case CRT_MATERIAL_REFLECTIVE: {
        Ray rr;
        rr.o = add(h.p, scale(n, st.reflection_bias));
        rr.d = sub(ray.d, scale(scale(n, 2.0f), dot(ray.d, n)));
        rr.depth = ray.depth + 1;
        const V3 alb = sample(sc.textures[m.tex], h.uv, h.bu, h.bv);
        return sc.refl ? mul_quirk(alb, shade(sc, rr, st, rng, cnt)) : alb;
    }
    case CRT_MATERIAL_REFRACTIVE: {
        if (!sc.refr) return v3(0.f, 0.f, 0.f);
        float n_out = 1.0f, n_in = m.ior;
        if (dot(ray.d, n) > 0.0f) {
            n = neg(n);
            std::swap(n_in, n_out);
        }
        /* Ray::refracted_at → refract_at with its default 1e-2f bias (crt_ray.h:30-35,40-50) */
        bool has_refr = false;
        Ray tr;
        {
            V3 d = ray.d;
            const float ca = -dot(d, n);
            const float sa = std::sqrt(1.0f - ca * ca);
            if (!(sa > n_in / n_out)) {             /* crt_vector.cpp:11-27 */
                const float sb = sa * n_out / n_in;
                const float cb = std::sqrt(1.0f - sb * sb);
                d = add(d, scale(n, ca));
                d = unit(d);
                d = scale(d, sb);
                d = add(d, scale(neg(n), cb));
                tr.o = add(h.p, scale(neg(n), 1e-2f));
                tr.d = d;
                tr.depth = ray.depth + 1;
                has_refr = true;
            }
        }
        Ray rr;
        rr.o = add(h.p, scale(n, st.reflection_bias));
        rr.d = sub(ray.d, scale(scale(n, 2.0f), dot(ray.d, n)));
        rr.depth = ray.depth + 1;
        const V3 cr = shade(sc, rr, st, rng, cnt);
        if (!has_refr) return cr;
        const V3 ct = shade(sc, tr, st, rng, cnt);
        const float f = 0.5f * std::pow((1.0f + dot(ray.d, n)), 5.0f);
        return add(scale(cr, f), scale(ct, 1.0f - f));
    }
    default:  /* Constant */
        return sample(sc.textures[m.tex], h.uv, h.bu, h.bv);
    }
}

/* ---- render_image: crt_renderer.cpp:147-199 ---------------------------- */
struct Bucket { int x, y, w, h; };

static std::vector<Bucket> bucket_grid(const Scene &sc) {
    std::vector<Bucket> out;
    const int nx = (int)(float(sc.width) / sc.bucket + 0.5);
    const int ny = (int)(float(sc.height) / sc.bucket + 0.5);
    for (int by = 0; by < ny; ++by) {
        const int y = by * sc.bucket;
        const int h = by == ny - 1 ? sc.height - y : sc.bucket;
        for (int bx = 0; bx < nx; ++bx) {
            const int x = bx * sc.bucket;
            const int w = bx == nx - 1 ? sc.width - x : sc.bucket;
            out.push_back(Bucket{x, y, w, h});
        }
    }
    return out;
}

static void render(const Scene &sc, const crt_renderer_settings &st, float *out, int nthreads,
                   Counters *total) {
    const std::vector<Bucket> grid = bucket_grid(sc);
    size_t next = 0;
    std::mutex mu;
    std::vector<Counters> per(nthreads);
    auto worker = [&](int tid) {
        for (;;) {
            Bucket b;
            {
                std::lock_guard<std::mutex> g(mu);
                if (next >= grid.size()) return;
                b = grid[next++];
            }
            for (int y = b.y; y < b.y + b.h; ++y)
                for (int x = b.x; x < b.x + b.w; ++x) {
                    Pcg rng = pixel_rng((uint32_t)x, (uint32_t)y);
                    const Ray r = camera_ray(sc, x, y);
                    const V3 c = shade(sc, r, st, rng, per[tid]);
                    float *px = out + 3 * ((size_t)y * sc.width + x);
                    px[0] = c.x; px[1] = c.y; px[2] = c.z;
                }
        }
    };
    std::vector<std::thread> pool;
    for (int i = 0; i < nthreads; ++i) pool.emplace_back(worker, i);
    for (auto &t : pool) t.join();
    if (total) {
        for (const Counters &c : per) {
            total->traversals += c.traversals; total->nodes += c.nodes;
            total->tris += c.tris; total->hits += c.hits;
        }
    }
}

static Scene *make_scene(const crt_scene_desc *d) {
    Scene *sc = new Scene();
    sc->background = v3(d->background_color.x, d->background_color.y, d->background_color.z);
    sc->cam_loc = v3(d->camera.location.x, d->camera.location.y, d->camera.location.z);
    std::memcpy(sc->cam_rot, d->camera.rotation, sizeof(sc->cam_rot));
    sc->width = d->camera.width;
    sc->height = d->camera.height;
    sc->fov_rad = d->camera.fov_degrees * 3.14159265358979323846f / 180.0f;   /* crt_camera.h:20 */
    sc->bucket = d->bucket_size;
    sc->gi = d->gi_on != 0;
    sc->refl = d->reflections_on != 0;
    sc->refr = d->refractions_on != 0;
    for (int i = 0; i < d->texture_count; ++i) {
        const crt_texture_desc &t = d->textures[i];
        Texture tx;
        tx.type = t.type;
        tx.c0 = v3(t.color0.x, t.color0.y, t.color0.z);
        tx.c1 = v3(t.color1.x, t.color1.y, t.color1.z);
        tx.s = t.scalar;
        tx.w = t.bitmap_width;
        tx.h = t.bitmap_height;
        if (t.type == CRT_TEXTURE_BITMAP && t.bitmap_rgb)
            for (int64_t k = 0; k < (int64_t)t.bitmap_width * t.bitmap_height; ++k)
                tx.texels.push_back(v3(t.bitmap_rgb[3 * k], t.bitmap_rgb[3 * k + 1], t.bitmap_rgb[3 * k + 2]));
        sc->textures.push_back(tx);
    }
    for (int i = 0; i < d->material_count; ++i)
        sc->materials.push_back(Material{d->materials[i].type, d->materials[i].albedo_texture_index,
                                         d->materials[i].ior});
    for (int i = 0; i < d->light_count; ++i)
        sc->lights.push_back(Light{d->lights[i].intensity,
                                   v3(d->lights[i].position.x, d->lights[i].position.y, d->lights[i].position.z)});
    size_t nv = 0;
    for (int i = 0; i < d->mesh_count; ++i) nv += (size_t)d->meshes[i].vertex_count;
    sc->verts.reserve(nv);
    for (int i = 0; i < d->mesh_count; ++i)
        append_mesh(*sc, d->meshes[i], d->materials[d->meshes[i].material_index]);
    build_tree(*sc);
    return sc;
}

}  // namespace oracle

using namespace oracle;

extern "C" {

struct oracle_scene { Scene *sc; };

oracle_scene *oracle_scene_create(const crt_scene_desc *d) {
    oracle_scene *o = new oracle_scene();
    o->sc = make_scene(d);
    return o;
}

void oracle_set_shadows(oracle_scene *o, int shadows) { o->sc->shadows = shadows != 0; }

void oracle_scene_destroy(oracle_scene *o) {
    if (!o) return;
    delete o->sc;
    delete o;
}

/* out: W*H*3 floats. counts may be NULL. */
int oracle_render(oracle_scene *o, const crt_renderer_settings *st, float *out, int nthreads,
                  crt_work_counts *counts) {
    if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
    if (nthreads <= 0) nthreads = 1;
    Counters c;
    render(*o->sc, *st, out, nthreads, &c);
    if (counts) {
        counts->traversals = c.traversals; counts->node_tests = c.nodes;
        counts->triangle_tests = c.tris; counts->hits = c.hits;
    }
    return 0;
}

/* Render only pixels [first, first+count) in row-major order, single thread
 * (bounded CPU-baseline samples). */
int oracle_render_pixels(oracle_scene *o, const crt_renderer_settings *st, int64_t first,
                         int64_t count, float *out, crt_work_counts *counts) {
    const Scene &sc = *o->sc;
    Counters c;
    for (int64_t i = 0; i < count; ++i) {
        const int64_t p = first + i;
        const int x = (int)(p % sc.width), y = (int)(p / sc.width);
        Pcg rng = pixel_rng((uint32_t)x, (uint32_t)y);
        const V3 col = shade(sc, camera_ray(sc, x, y), *st, rng, c);
        out[3 * i] = col.x; out[3 * i + 1] = col.y; out[3 * i + 2] = col.z;
    }
    if (counts) {
        counts->traversals = c.traversals; counts->node_tests = c.nodes;
        counts->triangle_tests = c.tris; counts->hits = c.hits;
    }
    return 0;
}

/* Closest hit of n rays (6 floats each) + per-ray node/triangle test counts. */
int oracle_trace(oracle_scene *o, const float *rays, int64_t n, crt_hit *hits, int64_t *node_tests,
                 int64_t *tri_tests) {
    const Scene &sc = *o->sc;
    for (int64_t i = 0; i < n; ++i) {
        Ray r;
        r.o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        r.d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        r.depth = 0;
        Counters c;
        Hit h;
        crt_hit &out = hits[i];
        std::memset(&out, 0, sizeof(out));
        out.triangle_index = -1;
        if (closest_hit(sc, r, h, c)) {
            out.hit = 1;
            out.distance = h.t;
            out.point[0] = h.p.x; out.point[1] = h.p.y; out.point[2] = h.p.z;
            out.normal[0] = h.n.x; out.normal[1] = h.n.y; out.normal[2] = h.n.z;
            out.uv[0] = h.uv.x; out.uv[1] = h.uv.y; out.uv[2] = h.uv.z;
            out.bary_u = h.bu; out.bary_v = h.bv;
            out.material_index = h.mat;
            out.triangle_index = h.tri;
        }
        if (node_tests) node_tests[i] = (int64_t)c.nodes;
        if (tri_tests) tri_tests[i] = (int64_t)c.tris;
    }
    return 0;
}

/* Camera rays for (x,y) pairs → n*6 floats. */
int oracle_camera_rays(oracle_scene *o, const int32_t *xy, int64_t n, float *rays) {
    for (int64_t i = 0; i < n; ++i) {
        const Ray r = camera_ray(*o->sc, xy[2 * i], xy[2 * i + 1]);
        rays[6 * i] = r.o.x; rays[6 * i + 1] = r.o.y; rays[6 * i + 2] = r.o.z;
        rays[6 * i + 3] = r.d.x; rays[6 * i + 4] = r.d.y; rays[6 * i + 5] = r.d.z;
    }
    return 0;
}

int64_t oracle_node_count(oracle_scene *o) { return (int64_t)o->sc->nodes.size(); }
int64_t oracle_triangle_count(oracle_scene *o) { return (int64_t)o->sc->tris.size(); }
int64_t oracle_vertex_count(oracle_scene *o) { return (int64_t)o->sc->verts.size(); }

/* Tree in the reference's preorder numbering: bounds n*6, children n*2,
 * leaf_offsets n+1 (prefix sums of leaf sizes), leaf_tris (triangle ids). */
int oracle_tree_dump(oracle_scene *o, float *bounds, int32_t *children, int64_t *leaf_offsets,
                     int32_t *leaf_tris) {
    const Scene &sc = *o->sc;
    int64_t off = 0;
    for (size_t i = 0; i < sc.nodes.size(); ++i) {
        const Node &nd = sc.nodes[i];
        if (bounds) {
            bounds[6 * i] = nd.bounds.lo.x; bounds[6 * i + 1] = nd.bounds.lo.y; bounds[6 * i + 2] = nd.bounds.lo.z;
            bounds[6 * i + 3] = nd.bounds.hi.x; bounds[6 * i + 4] = nd.bounds.hi.y; bounds[6 * i + 5] = nd.bounds.hi.z;
        }
        if (children) { children[2 * i] = nd.child[0]; children[2 * i + 1] = nd.child[1]; }
        if (leaf_offsets) leaf_offsets[i] = off;
        for (int32_t id : nd.tris) {
            if (leaf_tris) leaf_tris[off] = id;
            ++off;
        }
    }
    if (leaf_offsets) leaf_offsets[sc.nodes.size()] = off;
    return 0;
}

int oracle_vertex_normals(oracle_scene *o, float *out) {
    const Scene &sc = *o->sc;
    for (size_t i = 0; i < sc.verts.size(); ++i) {
        out[3 * i] = sc.verts[i].nrm.x; out[3 * i + 1] = sc.verts[i].nrm.y; out[3 * i + 2] = sc.verts[i].nrm.z;
    }
    return 0;
}

int oracle_face_normals(oracle_scene *o, float *out) {
    const Scene &sc = *o->sc;
    for (size_t i = 0; i < sc.tris.size(); ++i) {
        out[3 * i] = sc.tris[i].fn.x; out[3 * i + 1] = sc.tris[i].fn.y; out[3 * i + 2] = sc.tris[i].fn.z;
    }
    return 0;
}

}  // extern "C"
