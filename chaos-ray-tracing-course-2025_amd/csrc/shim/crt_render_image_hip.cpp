/*
 * crt_render_image_hip.cpp — drop-in definition of the reference's renderer
 * entry point over the C-ABI of this repo (include/crt_hip.h):
 *
 *   crt::Image crt::render_image(const crt::Scene &, const crt::RendererSettings &)
 *       declared src/core/crt_renderer.h:27, defined src/core/crt_renderer.cpp:157-199
 *
 * Compiled against the reference's OWN headers (-I<reference>/src), it
 * replaces crt_renderer.cpp in the reference's crt_core library; the two
 * callers (src/standalone/main.cpp:38, src/python/py_crt_module.cpp:100) and
 * through _crt the Blender add-on are unchanged.  Build + link recipe:
 * INTEGRATION.md §1 (the package Makefile's `shim` target compiles it here).
 *
 * What crosses: the Scene the reference already built is handed over as it
 * is — Scene::vertices (after vertex_array_extend, crt_mesh.cpp:32-73) and
 * Scene::acceleration_tree (after acceleration_tree::build,
 * crt_acceleration_tree.cpp:87-106), node for node with every leaf's Triangle
 * copies as (vertex index, face normal, material, flags) — through
 * crt_hip_scene_from_tree; nothing is rebuilt.  The device scene is cached
 * per Scene object and reused while the flattened description is byte-equal
 * to the cached one (frames of an unchanged scene pay only the render).
 *
 * Errors: the reference's render_image cannot fail; a HIP failure here throws
 * std::runtime_error with crt_hip_last_error() (the CLI reports it and exits
 * 1; a CPython caller should translate it — INTEGRATION.md §2).
 * Device: CRT_HIP_DEVICE (default 0).
 */
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "core/crt_renderer.h"
#include "core/crt_scene.h"
#include "crt_hip.h"

namespace {

/* Camera keeps fov and transform private (crt_camera.h:64-67) and exposes no
 * accessor; the device needs the same m_fov_radians and m_transform that
 * Camera::generate_ray uses (crt_camera.cpp:7-35).  Access through explicit
 * template instantiation, which the standard exempts from access checking
 * ([temp.spec.general]/6). */
template <class Tag, typename Tag::type M>
struct Grant {
    friend typename Tag::type member(Tag) { return M; }
};
struct CamFov {
    using type = float crt::Camera::*;
    friend type member(CamFov);
};
struct CamTransform {
    using type = crt::Transform crt::Camera::*;
    friend type member(CamTransform);
};
template struct Grant<CamFov, &crt::Camera::m_fov_radians>;
template struct Grant<CamTransform, &crt::Camera::m_transform>;

static_assert(sizeof(crt::Vector) == 3 * sizeof(float), "crt::Vector must be three packed floats");
static_assert(sizeof(crt::Vertex) == 9 * sizeof(float), "crt::Vertex must be position, normal, uv");

/* crt_tree_scene_desc of a Scene plus the arrays it points into. */
struct Flat {
    crt_tree_scene_desc desc{};
    std::vector<float> bounds;
    std::vector<int32_t> children;
    std::vector<int64_t> offsets;
    std::vector<crt_tree_triangle> tris;
    std::vector<crt_material_desc> materials;
    std::vector<crt_texture_desc> textures;
    std::vector<crt_light_desc> lights;
};

crt_vec3 v3(const crt::Vector &v) { return crt_vec3{v.x, v.y, v.z}; }

void flatten(const crt::Scene &s, Flat &f) {
    const crt::Vertex *base = s.vertices.data();
    const size_t n = s.acceleration_tree.size();
    f.bounds.resize(6 * n);
    f.children.resize(2 * n);
    f.offsets.resize(n + 1);
    f.tris.clear();
    for (size_t i = 0; i < n; ++i) {
        const crt::AccelerationTreeNode &nd = s.acceleration_tree[i];
        const float b[6] = {nd.bounds.min.x, nd.bounds.min.y, nd.bounds.min.z,
                            nd.bounds.max.x, nd.bounds.max.y, nd.bounds.max.z};
        std::memcpy(&f.bounds[6 * i], b, sizeof b);
        f.children[2 * i] = nd.children_indices[0];
        f.children[2 * i + 1] = nd.children_indices[1];
        f.offsets[i] = (int64_t)f.tris.size();
        for (const crt::Triangle &t : nd.triangles) {
            crt_tree_triangle o;
            o.v[0] = (int32_t)(t.v0 - base);
            o.v[1] = (int32_t)(t.v1 - base);
            o.v[2] = (int32_t)(t.v2 - base);
            o.face_normal[0] = t.face_normal.x;
            o.face_normal[1] = t.face_normal.y;
            o.face_normal[2] = t.face_normal.z;
            o.material_index = t.material_index;
            o.flags = (t.flags.smooth_shading ? 1 : 0) | (t.flags.back_face_culling ? 2 : 0);
            f.tris.push_back(o);
        }
    }
    f.offsets[n] = (int64_t)f.tris.size();

    f.materials.clear();
    for (const crt::Material &m : s.materials)
        f.materials.push_back(crt_material_desc{(int32_t)m.type, m.albedo_map_texture_index, m.ior, 0, 0});
    f.textures.clear();
    for (const crt::Texture &t : s.textures) {
        crt_texture_desc o{};
        o.type = (int32_t)t.type;
        switch (t.type) {   /* crt_texture.h:8-51 */
        case crt::TextureType::Albedo: o.color0 = v3(t.as_albedo_tex.albedo); break;
        case crt::TextureType::Edges:
            o.color0 = v3(t.as_edges_tex.edge_color);
            o.color1 = v3(t.as_edges_tex.inner_color);
            o.scalar = t.as_edges_tex.edge_width;
            break;
        case crt::TextureType::Checker:
            o.color0 = v3(t.as_checker_tex.color_a);
            o.color1 = v3(t.as_checker_tex.color_b);
            o.scalar = t.as_checker_tex.square_size;
            break;
        case crt::TextureType::Bitmap: {
            const crt::Image *img = t.as_bitmap_tex.image;
            o.bitmap_width = img ? img->width : 0;
            o.bitmap_height = img ? img->height : 0;
            o.bitmap_rgb = img ? reinterpret_cast<const float *>(img->buffer.data()) : nullptr;
            break;
        }
        }
        f.textures.push_back(o);
    }
    f.lights.clear();
    for (const crt::Light &l : s.lights) f.lights.push_back(crt_light_desc{l.intensity, v3(l.position)});

    crt_tree_scene_desc &d = f.desc;
    std::memset(&d, 0, sizeof d);
    d.background_color = v3(s.background_color);
    const crt::Transform &tf = s.camera.*member(CamTransform{});
    d.camera_location = v3(tf.location);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) d.camera_rotation[3 * r + c] = tf.rotation.data[r][c];
    d.width = s.camera.resolution_x();
    d.height = s.camera.resolution_y();
    d.fov_radians = s.camera.*member(CamFov{});
    d.bucket_size = s.bucket_size;
    d.gi_on = s.gi_on;
    d.reflections_on = s.reflections_on;
    d.refractions_on = s.refractions_on;
    d.vertices = reinterpret_cast<const float *>(s.vertices.data());
    d.vertex_count = (int64_t)s.vertices.size();
    d.node_bounds = f.bounds.data();
    d.node_children = f.children.data();
    d.leaf_offsets = f.offsets.data();
    d.leaf_triangles = f.tris.data();
    d.node_count = (int64_t)n;
    d.materials = f.materials.data();
    d.material_count = (int32_t)f.materials.size();
    d.textures = f.textures.data();
    d.texture_count = (int32_t)f.textures.size();
    d.lights = f.lights.data();
    d.light_count = (int32_t)f.lights.size();
}

[[noreturn]] void fail(const char *what) {
    throw std::runtime_error(std::string("crt_hip ") + what + ": " + crt_hip_last_error());
}

}  // namespace

namespace crt {

Image render_image(const Scene &scene, const RendererSettings &settings) {
    Image result{scene.camera.resolution_x(), scene.camera.resolution_y()};
    Flat flat;
    flatten(scene, flat);
    const crt_renderer_settings st{settings.max_ray_depth, settings.diffuse_reflection_ray_count, settings.shadow_bias,
                                   settings.reflection_bias, settings.diffuse_reflection_bias, settings.refraction_bias};
    /* the device-scene cache and the render: csrc/shim/crt_shim_core.cpp */
    if (crt_hip_render_image_tree(&flat.desc, &st, reinterpret_cast<float *>(result.buffer.data())) != CRT_OK)
        fail("render_image");
    return result;
}

}  // namespace crt
