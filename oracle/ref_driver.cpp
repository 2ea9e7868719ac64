/*
 * ref_driver.cpp — TEST INFRASTRUCTURE: a C-ABI shim over the reference's own
 * compiled translation units (built by oracle/Makefile from
 * /root/reference/src/core into oracle/_ref/; never copied into this repo).
 *
 * It builds a crt::Scene-equivalent exactly the way crt_json.cpp does
 * (vertices reserved up front :177, vertex_array_extend per object :211/213,
 * acceleration_tree::build :606, Camera{w,h,fov,Transform} :134-142) and then
 * calls the reference's hot-path functions directly:
 *   crt::intersection::ray_intersect_acceleration_tree (crt_intersection.cpp:109)
 *   crt::Camera::generate_ray                         (crt_camera.cpp:7)
 *   crt::write_ppm                                    (crt_image_ppm.cpp:9)
 * It is used only to pin oracle/crt_oracle.cpp and to generate tests/golden/.
 */
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <tuple>
#include <vector>

#include "core/crt_acceleration_tree.h"
#include "core/crt_camera.h"
#include "core/crt_image.h"
#include "core/crt_image_ppm.h"
#include "core/crt_intersection.h"
#include "core/crt_mesh.h"
#include "core/crt_transform.h"

#include "../include/crt_hip.h"

struct ref_scene {
    std::vector<crt::Vertex> vertices;
    std::vector<crt::Triangle> triangles;     /* pre-build order = global ids */
    crt::AccelerationTree tree;
    crt::Camera *camera = nullptr;
    std::map<std::tuple<const void *, const void *, const void *>, int32_t> tri_ids;
};

extern "C" {

ref_scene *ref_scene_create(const crt_scene_desc *d) {
    ref_scene *s = new ref_scene();
    size_t nv = 0, nt = 0;
    for (int i = 0; i < d->mesh_count; ++i) {
        nv += (size_t)d->meshes[i].vertex_count;
        nt += (size_t)d->meshes[i].index_count / 3;
    }
    s->vertices.reserve(nv);
    s->triangles.reserve(nt);
    for (int i = 0; i < d->mesh_count; ++i) {
        const crt_mesh_desc &m = d->meshes[i];
        std::vector<crt::Vector> pos((size_t)m.vertex_count), uvs;
        for (int64_t k = 0; k < m.vertex_count; ++k)
            pos[k] = crt::Vector{m.positions[3 * k], m.positions[3 * k + 1], m.positions[3 * k + 2]};
        std::vector<int> idx(m.indices, m.indices + m.index_count);
        const crt_material_desc &mat = d->materials[m.material_index];
        crt::TriangleFlags flags{};
        flags.smooth_shading = mat.smooth_shading ? 1 : 0;
        flags.back_face_culling = mat.back_face_culling ? 1 : 0;
        if (m.uvs) {
            uvs.resize((size_t)m.vertex_count);
            for (int64_t k = 0; k < m.vertex_count; ++k)
                uvs[k] = crt::Vector{m.uvs[3 * k], m.uvs[3 * k + 1], m.uvs[3 * k + 2]};
            crt::vertex_array_extend(s->vertices, s->triangles, pos, uvs, idx, m.material_index, flags);
        } else {
            crt::vertex_array_extend(s->vertices, s->triangles, pos, idx, m.material_index, flags);
        }
    }
    for (size_t i = 0; i < s->triangles.size(); ++i) {
        const crt::Triangle &t = s->triangles[i];
        s->tri_ids.emplace(std::make_tuple((const void *)t.v0, (const void *)t.v1, (const void *)t.v2), (int32_t)i);
    }
    s->tree = crt::acceleration_tree::build(s->triangles);
    crt::Transform tf;
    tf.location = crt::Vector{d->camera.location.x, d->camera.location.y, d->camera.location.z};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) tf.rotation.data[r][c] = d->camera.rotation[3 * r + c];
    s->camera = new crt::Camera(d->camera.width, d->camera.height, d->camera.fov_degrees, tf);
    return s;
}

void ref_scene_destroy(ref_scene *s) {
    if (!s) return;
    delete s->camera;
    delete s;
}

int64_t ref_node_count(ref_scene *s) { return (int64_t)s->tree.size(); }

int ref_tree_dump(ref_scene *s, float *bounds, int32_t *children, int64_t *leaf_offsets, int32_t *leaf_tris) {
    int64_t off = 0;
    for (size_t i = 0; i < s->tree.size(); ++i) {
        const crt::AccelerationTreeNode &n = s->tree[i];
        if (bounds) {
            bounds[6 * i] = n.bounds.min.x; bounds[6 * i + 1] = n.bounds.min.y; bounds[6 * i + 2] = n.bounds.min.z;
            bounds[6 * i + 3] = n.bounds.max.x; bounds[6 * i + 4] = n.bounds.max.y; bounds[6 * i + 5] = n.bounds.max.z;
        }
        if (children) { children[2 * i] = n.children_indices[0]; children[2 * i + 1] = n.children_indices[1]; }
        if (leaf_offsets) leaf_offsets[i] = off;
        for (const crt::Triangle &t : n.triangles) {
            if (leaf_tris) {
                auto it = s->tri_ids.find(std::make_tuple((const void *)t.v0, (const void *)t.v1, (const void *)t.v2));
                leaf_tris[off] = it == s->tri_ids.end() ? -1 : it->second;
            }
            ++off;
        }
    }
    if (leaf_offsets) leaf_offsets[s->tree.size()] = off;
    return 0;
}

int64_t ref_vertex_count(ref_scene *s) { return (int64_t)s->vertices.size(); }

/* Scene::vertices as the reference holds them after vertex_array_extend:
 * position, normal, uv (crt_vertex.h:7-11), 9 floats per vertex. */
int ref_vertex_dump(ref_scene *s, float *out) {
    for (size_t i = 0; i < s->vertices.size(); ++i) {
        const crt::Vertex &v = s->vertices[i];
        const float x[9] = {v.position.x, v.position.y, v.position.z, v.normal.x, v.normal.y,
                            v.normal.z, v.uv.x, v.uv.y, v.uv.z};
        std::memcpy(out + 9 * i, x, sizeof x);
    }
    return 0;
}

/* The leaves' Triangle copies in tree order (ref_tree_dump's leaf_offsets):
 * vertex indices = the Vertex pointers minus the array base, the copy's
 * face_normal, material_index and TriangleFlags (crt_triangle.h:19-23). */
int ref_leaf_triangles(ref_scene *s, crt_tree_triangle *out) {
    int64_t k = 0;
    const crt::Vertex *base = s->vertices.data();
    for (const crt::AccelerationTreeNode &n : s->tree) {
        for (const crt::Triangle &t : n.triangles) {
            crt_tree_triangle &o = out[k++];
            o.v[0] = (int32_t)(t.v0 - base);
            o.v[1] = (int32_t)(t.v1 - base);
            o.v[2] = (int32_t)(t.v2 - base);
            o.face_normal[0] = t.face_normal.x;
            o.face_normal[1] = t.face_normal.y;
            o.face_normal[2] = t.face_normal.z;
            o.material_index = t.material_index;
            o.flags = (t.flags.smooth_shading ? 1 : 0) | (t.flags.back_face_culling ? 2 : 0);
        }
    }
    return 0;
}

int ref_trace(ref_scene *s, const float *rays, int64_t n, crt_hit *hits) {
    for (int64_t i = 0; i < n; ++i) {
        crt::Ray r{};
        r.origin = crt::Vector{rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]};
        r.direction = crt::Vector{rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]};
        crt_hit &o = hits[i];
        std::memset(&o, 0, sizeof(o));
        o.triangle_index = -1;
        if (auto h = crt::intersection::ray_intersect_acceleration_tree(r, s->tree)) {
            o.hit = 1;
            o.distance = h->distance;
            o.point[0] = h->point.x; o.point[1] = h->point.y; o.point[2] = h->point.z;
            o.normal[0] = h->normal.x; o.normal[1] = h->normal.y; o.normal[2] = h->normal.z;
            o.uv[0] = h->uv.x; o.uv[1] = h->uv.y; o.uv[2] = h->uv.z;
            o.bary_u = h->bary_u; o.bary_v = h->bary_v;
            o.material_index = h->material_index;
        }
    }
    return 0;
}

int ref_camera_rays(ref_scene *s, const int32_t *xy, int64_t n, float *rays) {
    for (int64_t i = 0; i < n; ++i) {
        const crt::Ray r = s->camera->generate_ray(xy[2 * i], xy[2 * i + 1]);
        rays[6 * i] = r.origin.x; rays[6 * i + 1] = r.origin.y; rays[6 * i + 2] = r.origin.z;
        rays[6 * i + 3] = r.direction.x; rays[6 * i + 4] = r.direction.y; rays[6 * i + 5] = r.direction.z;
    }
    return 0;
}

int ref_vertex_normals(ref_scene *s, float *out) {
    for (size_t i = 0; i < s->vertices.size(); ++i) {
        out[3 * i] = s->vertices[i].normal.x; out[3 * i + 1] = s->vertices[i].normal.y;
        out[3 * i + 2] = s->vertices[i].normal.z;
    }
    return 0;
}

int ref_face_normals(ref_scene *s, float *out) {
    for (size_t i = 0; i < s->triangles.size(); ++i) {
        out[3 * i] = s->triangles[i].face_normal.x; out[3 * i + 1] = s->triangles[i].face_normal.y;
        out[3 * i + 2] = s->triangles[i].face_normal.z;
    }
    return 0;
}

int ref_write_ppm(const float *rgb, int32_t w, int32_t h, const char *path) {
    crt::Image img(w, h);
    for (int64_t i = 0; i < (int64_t)w * h; ++i)
        img.buffer[i] = crt::Vector{rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]};
    std::ofstream os(path, std::ios::out | std::ios::binary);
    if (!os) return -1;
    crt::write_ppm(img, os, 255);
    return 0;
}

}  // extern "C"
