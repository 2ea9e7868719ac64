/*
 * crt_shim_core.cpp — the body of the crt::render_image drop-in
 * (crt_render_image_hip.cpp), over this repo's own C-ABI types only, so it is
 * part of lib/libcrt_hip.so and runs wherever the library does (the GPU tests
 * drive it with the reference's built trees, tests/golden/reftree_*.npz).
 * The reference-header half of the shim only reads the crt::Scene's fields
 * into a crt_tree_scene_desc and calls crt_hip_render_image_tree.
 *
 * render_image (crt_renderer.cpp:157-199) renders whatever Scene it is
 * handed; a long-running caller (_crt, the Blender add-on) hands a new Scene
 * per frame, mostly the same geometry with the camera moved.  So the device
 * scenes of the two most recently rendered scenes stay cached
 * (crt_scene_lru.h), found by content without the camera; a scene equal but
 * for its camera moves the cached device scene's camera
 * (crt_hip_scene_set_camera_rad) instead of uploading it again.
 */
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../../include/crt_hip.h"
#include "../crt_host.h"
#include "crt_scene_lru.h"

namespace {

/* A tree scene description with every array it points to copied (the
 * caller's Scene goes away after the call), and its device scene. */
struct Owned {
    crt_tree_scene_desc desc{};
    std::vector<float> vertices, bounds;
    std::vector<int32_t> children;
    std::vector<int64_t> offsets;
    std::vector<crt_tree_triangle> tris;
    std::vector<crt_material_desc> materials;
    std::vector<crt_texture_desc> textures;
    std::vector<std::vector<float>> texels;
    std::vector<crt_light_desc> lights;
    crt_hip_scene *scene = nullptr;
    ~Owned() { crt_hip_scene_destroy(scene); }
};

template <class T>
bool same(const std::vector<T> &a, const T *b, size_t n) {
    return a.size() == n && (n == 0 || (b && std::memcmp(a.data(), b, n * sizeof(T)) == 0));
}

size_t texel_count(const crt_texture_desc &t) {
    return t.type == CRT_TEXTURE_BITMAP && t.bitmap_rgb ? (size_t)t.bitmap_width * t.bitmap_height * 3 : 0;
}

/* Byte-equality of everything but the camera and the large arrays (vertices,
 * tree, leaf triangles, texels): scalars, counts, materials, lights, texture
 * records.  A cached entry that passes is the candidate; slice_same then
 * compares the large arrays on the image copy's host threads while the
 * candidate's frame renders (crt_api.hip render_checked). */
bool cheap_same(const Owned &a, const crt_tree_scene_desc &b) {
    const crt_tree_scene_desc &x = a.desc;
    if (std::memcmp(&x.background_color, &b.background_color, sizeof x.background_color) != 0 ||
        x.bucket_size != b.bucket_size || x.gi_on != b.gi_on || x.reflections_on != b.reflections_on ||
        x.refractions_on != b.refractions_on || x.vertex_count != b.vertex_count || x.node_count != b.node_count ||
        x.material_count != b.material_count || x.texture_count != b.texture_count || x.light_count != b.light_count)
        return false;
    const size_t n = (size_t)b.node_count;
    if (a.offsets.size() != n + 1 || (n && a.offsets[n] != b.leaf_offsets[n])) return false;
    if (!same(a.materials, b.materials, (size_t)b.material_count) || !same(a.lights, b.lights, (size_t)b.light_count))
        return false;
    for (int32_t i = 0; i < b.texture_count; ++i) {
        crt_texture_desc p = a.textures[(size_t)i], q = b.textures[i];
        p.bitmap_rgb = q.bitmap_rgb = nullptr;
        if (std::memcmp(&p, &q, sizeof p) != 0) return false;
        if (a.texels[(size_t)i].size() != texel_count(b.textures[i])) return false;
    }
    return true;
}

/* Slice i of n of every large array (by bytes), after cheap_same. */
struct SliceArgs {
    const Owned *a;
    const crt_tree_scene_desc *b;
};

template <class T>
bool same_slice(const std::vector<T> &a, const T *b, int i, int n) {
    const size_t bytes = a.size() * sizeof(T), lo = bytes * (size_t)i / (size_t)n, hi = bytes * (size_t)(i + 1) / (size_t)n;
    return hi == lo || std::memcmp(reinterpret_cast<const char *>(a.data()) + lo, reinterpret_cast<const char *>(b) + lo,
                                   hi - lo) == 0;
}

bool slice_same(void *arg, int i, int n) {
    const SliceArgs &s = *static_cast<const SliceArgs *>(arg);
    const Owned &a = *s.a;
    const crt_tree_scene_desc &b = *s.b;
    if (!same_slice(a.vertices, b.vertices, i, n) || !same_slice(a.bounds, b.node_bounds, i, n) ||
        !same_slice(a.children, b.node_children, i, n) || !same_slice(a.offsets, b.leaf_offsets, i, n) ||
        !same_slice(a.tris, b.leaf_triangles, i, n))
        return false;
    for (int32_t t = 0; t < b.texture_count; ++t)
        if (!same_slice(a.texels[(size_t)t], b.textures[t].bitmap_rgb, i, n)) return false;
    return true;
}

bool same_but_camera(const Owned &a, const crt_tree_scene_desc &b) {
    if (!cheap_same(a, b)) return false;
    SliceArgs s{&a, &b};
    return slice_same(&s, 0, 1);
}

bool same_camera(const crt_tree_scene_desc &x, const crt_tree_scene_desc &b) {
    return std::memcmp(&x.camera_location, &b.camera_location, sizeof x.camera_location) == 0 &&
           std::memcmp(x.camera_rotation, b.camera_rotation, sizeof x.camera_rotation) == 0 && x.width == b.width &&
           x.height == b.height && x.fov_radians == b.fov_radians;
}

void set_camera_fields(crt_tree_scene_desc &x, const crt_tree_scene_desc &b) {
    x.camera_location = b.camera_location;
    std::memcpy(x.camera_rotation, b.camera_rotation, sizeof x.camera_rotation);
    x.width = b.width;
    x.height = b.height;
    x.fov_radians = b.fov_radians;
}

std::unique_ptr<Owned> copy_of(const crt_tree_scene_desc &b) {
    std::unique_ptr<Owned> o(new Owned());
    const size_t n = (size_t)b.node_count;
    o->vertices.assign(b.vertices, b.vertices + (size_t)b.vertex_count * 9);
    o->bounds.assign(b.node_bounds, b.node_bounds + 6 * n);
    o->children.assign(b.node_children, b.node_children + 2 * n);
    o->offsets.assign(b.leaf_offsets, b.leaf_offsets + n + 1);
    if (n) o->tris.assign(b.leaf_triangles, b.leaf_triangles + b.leaf_offsets[n]);
    o->materials.assign(b.materials, b.materials + b.material_count);
    o->lights.assign(b.lights, b.lights + b.light_count);
    o->textures.assign(b.textures, b.textures + b.texture_count);
    for (crt_texture_desc &t : o->textures) {
        const size_t nt = texel_count(t);
        o->texels.emplace_back(t.bitmap_rgb, t.bitmap_rgb + nt);
        t.bitmap_rgb = nt ? o->texels.back().data() : nullptr;
    }
    o->desc = b;
    o->desc.vertices = o->vertices.data();
    o->desc.node_bounds = o->bounds.data();
    o->desc.node_children = o->children.data();
    o->desc.leaf_offsets = o->offsets.data();
    o->desc.leaf_triangles = o->tris.data();
    o->desc.materials = o->materials.data();
    o->desc.textures = o->textures.data();
    o->desc.lights = o->lights.data();
    return o;
}

std::mutex g_mu;
crt_shim::SceneLru<Owned> g_cache(2);
int64_t g_creates = 0, g_moves = 0, g_reuses = 0;

}  // namespace

extern "C" {

int crt_hip_render_image_tree(const crt_tree_scene_desc *desc, const crt_renderer_settings *settings, float *rgb_out) {
    if (!desc || !settings || !rgb_out) return CRT_E_INVALID;
    if ((desc->vertex_count > 0 && !desc->vertices) || !desc->node_bounds || !desc->node_children ||
        !desc->leaf_offsets || desc->node_count < 0)
    {   /* malformed: the scene validation reports why */
        crt_hip_scene *tmp = nullptr;
        const int rc = crt_hip_scene_from_tree(desc, 0, &tmp);
        crt_hip_scene_destroy(tmp);
        return rc != CRT_OK ? rc : CRT_E_INVALID;
    }
    std::lock_guard<std::mutex> lock(g_mu);
    /* the most recent entry equal in everything but the camera and the large
     * arrays: render it, its large arrays compared with the caller's while the
     * frame renders (render_checked) — a repeat frame pays no serial compare */
    const Owned *tried = nullptr;
    if (Owned *c = g_cache.find([&](const Owned &e) { return cheap_same(e, *desc); })) {
        const bool moved = !same_camera(c->desc, *desc);
        if (moved) {
            const int rc = crt_hip_scene_set_camera_rad(c->scene, &desc->camera_location, desc->camera_rotation,
                                                        desc->fov_radians, desc->width, desc->height);
            if (rc != CRT_OK) return rc;
            set_camera_fields(c->desc, *desc);
        }
        SliceArgs args{c, desc};
        bool mismatch = false;
        const int rc = crt_amd::render_checked(c->scene, settings, rgb_out, nullptr, slice_same, &args, &mismatch);
        if (rc != CRT_OK || !mismatch) {
            if (rc == CRT_OK) ++(moved ? g_moves : g_reuses);
            return rc;
        }
        tried = c;   /* same shape, other content */
    }
    Owned *c = g_cache.find([&](const Owned &e) { return &e != tried && same_but_camera(e, *desc); });
    if (!c) {
        std::unique_ptr<Owned> fresh = copy_of(*desc);
        /* as many GPUs as the frame pays for (crt_hip_scene_from_tree_auto;
         * CRT_HIP_GPUS=N sets the count), as render_image spans every hardware
         * thread (crt_renderer.cpp:176-196); CRT_HIP_DEVICE=K pins one device */
        const char *dev = std::getenv("CRT_HIP_DEVICE");
        const int rc = dev ? crt_hip_scene_from_tree(&fresh->desc, std::atoi(dev), &fresh->scene)
                           : crt_hip_scene_from_tree_auto(&fresh->desc, settings, &fresh->scene);
        if (rc != CRT_OK) return rc;
        c = g_cache.insert(std::move(fresh));
        ++g_creates;
    } else if (!same_camera(c->desc, *desc)) {
        const int rc = crt_hip_scene_set_camera_rad(c->scene, &desc->camera_location, desc->camera_rotation,
                                                    desc->fov_radians, desc->width, desc->height);
        if (rc != CRT_OK) return rc;
        set_camera_fields(c->desc, *desc);
        ++g_moves;
    } else {
        ++g_reuses;
    }
    return crt_hip_render(c->scene, settings, rgb_out, nullptr);
}

int crt_hip_render_image_tree_stats(int64_t *creates, int64_t *camera_moves, int64_t *reuses) {
    std::lock_guard<std::mutex> lock(g_mu);
    if (creates) *creates = g_creates;
    if (camera_moves) *camera_moves = g_moves;
    if (reuses) *reuses = g_reuses;
    return CRT_OK;
}

void crt_hip_render_image_tree_reset(void) {
    std::lock_guard<std::mutex> lock(g_mu);
    g_cache.clear();
}

}  // extern "C"
