/*
 * crt_hip.h — C-ABI drop-in boundary for the MI355X (gfx950) render path.
 *
 * Replaces (reference = bvpav/chaos-ray-tracing-course-2025):
 *   crt::Image crt::render_image(const crt::Scene&, const crt::RendererSettings&)
 *       src/core/crt_renderer.h:27, defined at src/core/crt_renderer.cpp:157-199
 *   and, below it, the per-ray hot path
 *       crt::intersection::ray_intersect_acceleration_tree   src/core/crt_intersection.cpp:109-136
 *       crt::intersection::ray_intersect_aabb_p              src/core/crt_intersection.cpp:14-45
 *       crt::intersection::ray_intersect_triangle(_span)     src/core/crt_intersection.cpp:47-107
 *
 * Plain C: pointers + sizes, no C++/torch types.  Every entry point returns 0 on
 * success or a negative CRT_E_* status; crt_hip_last_error() then holds a
 * thread-local message.  The reference's render_image cannot fail; its callers
 * (CLI main.cpp:22-26, _crt py_crt_module.cpp:91-94) map failures to exit code
 * 1 / ValueError, and the shims in this repo do the same.
 */
#ifndef CRT_HIP_H
#define CRT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRT_HIP_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------- */
#define CRT_OK              0
#define CRT_E_INVALID     (-1)   /* bad argument / malformed scene            */
#define CRT_E_PARSE       (-2)   /* scene JSON rejected (crt_json.cpp:541-647) */
#define CRT_E_UNSUPPORTED (-3)   /* feature outside this build's scope        */
#define CRT_E_HIP         (-4)   /* HIP runtime error                         */
#define CRT_E_NOMEM       (-5)
#define CRT_E_IO          (-6)
#define CRT_E_STATE       (-7)   /* an earlier asynchronous frame was rendered wrongly (see the message) */

/* ---- scene description (the reference's crt::Scene inputs, flat) ---- */
typedef struct crt_vec3 { float x, y, z; } crt_vec3;

/* crt_material.h:5-10 */
enum { CRT_MATERIAL_DIFFUSE = 0, CRT_MATERIAL_REFLECTIVE = 1,
       CRT_MATERIAL_REFRACTIVE = 2, CRT_MATERIAL_CONSTANT = 3 };
/* crt_texture.h:8-13 */
enum { CRT_TEXTURE_ALBEDO = 0, CRT_TEXTURE_EDGES = 1,
       CRT_TEXTURE_CHECKER = 2, CRT_TEXTURE_BITMAP = 3 };

/* crt_texture.h:15-51 (tagged union flattened) */
typedef struct crt_texture_desc {
    int32_t  type;
    crt_vec3 color0;          /* Albedo: albedo | Edges: edge_color | Checker: color_A */
    crt_vec3 color1;          /* Edges: inner_color | Checker: color_B                 */
    float    scalar;          /* Edges: edge_width  | Checker: square_size             */
    int32_t  bitmap_width;    /* Bitmap: decoded texels, rgb fp32, top row first      */
    int32_t  bitmap_height;
    const float *bitmap_rgb;
} crt_texture_desc;

/* crt_material.h:12-16 + per-material TriangleFlags (crt_json.cpp:535) */
typedef struct crt_material_desc {
    int32_t type;
    int32_t albedo_texture_index;   /* -1 for refractive (crt_json.cpp:493) */
    float   ior;
    int32_t smooth_shading;
    int32_t back_face_culling;
} crt_material_desc;

/* one scene "object" (crt_json.cpp:150-218 → vertex_array_extend, crt_mesh.cpp:32-73) */
typedef struct crt_mesh_desc {
    const float   *positions;     /* vertex_count * 3                      */
    const float   *uvs;           /* vertex_count * 3, or NULL (uv = 0)   */
    int64_t        vertex_count;
    const int32_t *indices;       /* index_count, multiple of 3, mesh-local */
    int64_t        index_count;
    int32_t        material_index;
} crt_mesh_desc;

/* crt_light.h:10-16 */
typedef struct crt_light_desc { float intensity; crt_vec3 position; } crt_light_desc;

/* crt_camera.h:13-25 + crt_transform.h:8-10 */
typedef struct crt_camera_desc {
    crt_vec3 location;
    float    rotation[9];         /* row-major 3x3, ray_dir = v * R (crt_matrix.h:66-74) */
    int32_t  width, height;
    float    fov_degrees;         /* 90 when the scene file has none (crt_camera.h:13-15) */
} crt_camera_desc;

/* crt_scene.h:18-30 */
typedef struct crt_scene_desc {
    crt_vec3 background_color;
    crt_camera_desc camera;
    int32_t  bucket_size;                         /* default 24 (crt_scene.h:16) */
    int32_t  gi_on, reflections_on, refractions_on;
    const crt_mesh_desc     *meshes;    int32_t mesh_count;
    const crt_material_desc *materials; int32_t material_count;
    const crt_texture_desc  *textures;  int32_t texture_count;
    const crt_light_desc    *lights;    int32_t light_count;
} crt_scene_desc;

/* crt_renderer.h:18-25 (same six fields, same defaults) */
typedef struct crt_renderer_settings {
    uint32_t max_ray_depth;                 /* 3    */
    uint32_t diffuse_reflection_ray_count;  /* 4    */
    float    shadow_bias;                   /* 1e-2 */
    float    reflection_bias;               /* 1e-2 */
    float    diffuse_reflection_bias;       /* 1e-2 */
    float    refraction_bias;               /* 1e-2 */
} crt_renderer_settings;

/* crt_intersection.h:13-20 plus hit flag / triangle id (test hook only) */
typedef struct crt_hit {
    float   distance;
    float   point[3];
    float   normal[3];
    float   uv[3];
    float   bary_u, bary_v;
    int32_t material_index;
    int32_t hit;              /* 0 = std::nullopt */
    int32_t triangle_index;   /* scene-global triangle id, -1 on miss */
} crt_hit;

typedef struct crt_scene_info {
    int64_t triangle_count;
    int64_t vertex_count;
    int64_t node_count;        /* crt_acceleration_tree.cpp:87-106 node count */
    int64_t leaf_count;
    int64_t leaf_ref_count;    /* triangle copies held by leaves              */
    int32_t max_depth;
    int32_t max_leaf_size;
    int64_t device_bytes;      /* bytes resident in HBM for this scene        */
    int32_t width, height;
    int32_t bucket_size;
    int32_t gi_on, reflections_on, refractions_on;
    int32_t tree_on_device;    /* 1: tree built by crt_tree_build.hip on the GPU   */
    double  tree_build_ms;     /* wall time of the tree build (host: build + flatten into the device layout) */
    /* scene-create cost (wall ms; host scenes: the host parts only) */
    double  prep_ms;           /* host preparation in all: mesh prep, host tree build, BVH */
    double  bvh_ms;            /* the secondary-ray BVH and proof tables (host; + the device build, bvh_on_device) */
    double  bins_ms;           /* camera-bins setup: templates, buffers, the sizing pass (device) */
    double  upload_ms;         /* upload to every device (incl. device tree build and bins setup) */
    double  create_ms;         /* the whole crt_hip_scene_create* call */
    int32_t wf_sets;           /* wavefront frame buffer sets holding buffers (1 for a caller that waits for
                                * each frame; up to 12 for frames issued back to back) */
    int32_t pad0;
    int64_t camera_moves;      /* crt_hip_scene_set_camera calls that changed the camera */
    int64_t view_rebuilds;     /* ... of them that rebuilt the view's plans / buffers (new resolution, camera
                                * bins built or dropped for the new camera) with the device drained */
    int64_t records_written;   /* device scene records written (one per camera, plus table pointers) */
    int32_t multi_probe;       /* handles over >= 2 distinct GPUs: 1 the probe frame matched, -1 it differed and
                                * -2 it failed (the handle then renders on one GPU), 0 not run */
    int32_t pad1;
    double  multi_probe_ms;    /* wall time of that probe (two 64x36 frames and two view rebuilds) */
    int64_t bins_binnings;     /* camera-bins binnings run (frames, plus the test hooks') */
    int64_t bins_reuses;       /* frames that rendered the last binning's lists (same camera; option "bins_reuse") */
    int32_t bvh_on_device;     /* 1: the BVH was built on the device (crt_lbvh.hip, > 2^18 triangles; its
                                * time is in bvh_ms) */
    int32_t bvh_depth;         /* ... its deepest node (root 0), 0 for the host build */
    int64_t light_bin_records; /* light bins' candidate records (built at the first shadow-ray frame; 0: none) */
    double  light_bins_ms;     /* wall time of that build and upload */
} crt_scene_info;

typedef struct crt_render_stats {
    double   kernel_ms;        /* device time of the render kernel(s)      */
    double   total_ms;         /* host wall time of the whole call         */
    int32_t  width, height;
} crt_render_stats;

/* Work counters of one frame (instrumented kernel, §8(d) algorithmic bytes). */
typedef struct crt_work_counts {
    uint64_t traversals;       /* calls of ray_intersect_acceleration_tree */
    uint64_t node_tests;       /* ray_intersect_aabb_p calls               */
    uint64_t triangle_tests;   /* ray_intersect_triangle calls             */
    uint64_t hits;             /* traversals returning an intersection     */
} crt_work_counts;

/* ---- host: scene file loader (crt_json.cpp:541-647) ------------------ */
typedef struct crt_scene_file crt_scene_file;
/* Parse .crtscene JSON text. Same accept/reject rules and defaults as the
 * reference loader.  Bitmap textures are read from asset_root /
 * relative_path(file_path) (crt_json.cpp:349-368) and decoded by
 * crt_image_decode_rgb8; a file that cannot be read or decoded makes texture
 * parsing fail exactly as a failed read_stb would (crt_json.cpp:582-588). */
int  crt_scene_file_parse(const char *json_text, size_t len, const char *asset_root,
                          crt_scene_file **out);
int  crt_scene_file_load(const char *path, crt_scene_file **out);
const crt_scene_desc *crt_scene_file_desc(const crt_scene_file *f);
/* Override image size (the reference CLI has no flags; BASELINE configs need it). */
int  crt_scene_file_set_resolution(crt_scene_file *f, int32_t width, int32_t height);
void crt_scene_file_destroy(crt_scene_file *f);

/* Replaces read_stb (src/core/crt_image_stbi.cpp:16-40, stbi_load with
 * STBI_rgb): decode an image file held in memory into 8-bit RGB, top row
 * first.  JPEG (baseline + progressive, stb_image's integer IDCT, upsampling
 * and colour conversion — csrc/crt_image_decode.cpp).  *file_components is the
 * file's component count as stbi_load reports it (the loader requires 3).
 * With rgb_out NULL only the size is returned; otherwise cap >= w*h*3. */
int  crt_image_decode_rgb8(const uint8_t *bytes, size_t len, int32_t *width, int32_t *height,
                           int32_t *file_components, uint8_t *rgb_out, size_t cap);

/* ---- host: scene preparation (no GPU needed) ------------------------- */
typedef struct crt_host_scene crt_host_scene;

/* Mesh prep (vertex_array_extend, crt_mesh.cpp:10-73) and the exact
 * acceleration-tree build (crt_acceleration_tree.cpp:13-106), flattened into
 * the device layout.  The caller keeps ownership of every array in `desc`. */
int  crt_host_scene_create(const crt_scene_desc *desc, crt_host_scene **out);
int  crt_host_scene_info(const crt_host_scene *hs, crt_scene_info *out);
/* Tree in the reference's own preorder numbering: bounds n*6 (min xyz, max xyz),
 * children n*2 (-1 = none), leaf_offsets n+1, leaf_tris (global triangle ids,
 * leaf order).  Any pointer may be NULL. */
int  crt_host_scene_tree(const crt_host_scene *hs, float *bounds, int32_t *children,
                         int64_t *leaf_offsets, int32_t *leaf_tris);
int  crt_host_scene_vertex_normals(const crt_host_scene *hs, float *out);   /* 3 per vertex */
int  crt_host_scene_face_normals(const crt_host_scene *hs, float *out);     /* 3 per triangle */
void crt_host_scene_destroy(crt_host_scene *hs);

/* ---- device scene ---------------------------------------------------- */
typedef struct crt_hip_scene crt_hip_scene;

/* crt_host_scene_create + crt_hip_scene_upload (tree build chosen as
 * CRT_SCENE_TREE_AUTO, see crt_hip_scene_create_ex). */
int  crt_hip_scene_create(const crt_scene_desc *desc, int device, crt_hip_scene **out);

/* Where the acceleration tree (crt_acceleration_tree.cpp:13-106) is built:
 * AUTO = on the device from CRT_SCENE_DEVICE_BUILD_MIN triangles up (the env
 * variable CRT_TREE_BUILD=host|device overrides), HOST = crt_scene_build.cpp,
 * DEVICE = crt_tree_build.hip.  Both builds produce identical bits. */
#define CRT_SCENE_TREE_AUTO   0
#define CRT_SCENE_TREE_HOST   1
#define CRT_SCENE_TREE_DEVICE 2
#define CRT_SCENE_DEVICE_BUILD_MIN 65536
/* further flag bits of the create calls that take flags (_ex, _on, _mask, _auto) */
#define CRT_SCENE_NO_DEVICE_BVH        (1 << 4)   /* no device-built BVH above 2^18 triangles (kd walks for every ray) */
#define CRT_SCENE_PROBE_OFF            (1 << 5)   /* multi-device creates: no probe frame */
#define CRT_SCENE_PROBE_FORCE          (1 << 6)   /* ... the probe even over repeated devices */
#define CRT_SCENE_PROBE_TEST_MISMATCH  (1 << 7)   /* test hook: the probe's sharded image gets a differing bit */
int  crt_hip_scene_create_ex(const crt_scene_desc *desc, int device, int flags, crt_hip_scene **out);

/* ---- device scene from the reference's already-built crt::Scene -------
 * For a caller that holds the reference's own data structures (crt_scene.h:
 * 18-30): the vertex array after vertex_array_extend (crt_mesh.cpp:32-73)
 * and the acceleration tree after acceleration_tree::build
 * (crt_acceleration_tree.cpp:87-106), node for node in its preorder
 * numbering.  Nothing is rebuilt: the tree, its leaf triangle copies and
 * their face normals are taken as given and flattened into the device
 * layout.  Used by the crt::render_image shim (csrc/shim/). */

/* One Triangle copy held by a leaf (crt_triangle.h:19-23): vertex indices
 * into the vertex array (the reference's Vertex pointers minus the array's
 * base), its face normal, material and TriangleFlags. */
typedef struct crt_tree_triangle {
    int32_t  v[3];
    float    face_normal[3];
    int32_t  material_index;
    int32_t  flags;           /* bit 0 smooth_shading, bit 1 back_face_culling */
} crt_tree_triangle;

typedef struct crt_tree_scene_desc {
    crt_vec3 background_color;
    /* Camera (crt_camera.h:16-21): the stored m_fov_radians, m_transform */
    crt_vec3 camera_location;
    float    camera_rotation[9];      /* row-major, Matrix::data */
    int32_t  width, height;
    float    fov_radians;
    int32_t  bucket_size;
    int32_t  gi_on, reflections_on, refractions_on;
    /* Scene::vertices: 9 floats per vertex — position, normal, uv (crt_vertex.h:7-11) */
    const float *vertices;       int64_t vertex_count;
    /* Scene::acceleration_tree in its own numbering: node_bounds n*6 (min xyz,
     * max xyz), node_children n*2 (-1 = none), leaf_offsets n+1 into
     * leaf_triangles (interior nodes: empty ranges) */
    const float   *node_bounds;
    const int32_t *node_children;
    const int64_t *leaf_offsets;
    const crt_tree_triangle *leaf_triangles;
    int64_t node_count;
    /* materials (smooth / culling fields ignored: flags are per triangle here),
     * textures, lights as in crt_scene_desc */
    const crt_material_desc *materials; int32_t material_count;
    const crt_texture_desc  *textures;  int32_t texture_count;
    const crt_light_desc    *lights;    int32_t light_count;
} crt_tree_scene_desc;

/* Validates the tree (children numbered after their parent, leaves hold
 * triangles, interior nodes none; indices in range) and uploads it. */
int  crt_hip_scene_from_tree(const crt_tree_scene_desc *desc, int device, crt_hip_scene **out);
/* Host-only part of the same (tree flatten; no GPU). */
int  crt_host_scene_from_tree(const crt_tree_scene_desc *desc, crt_host_scene **out);

/* crt::render_image (crt_renderer.h:27) for the reference's built Scene, as
 * the shim (csrc/shim/crt_render_image_hip.cpp) calls it once it has read
 * the Scene's fields into a crt_tree_scene_desc: the device scenes of the two
 * most recently rendered scenes stay cached by content (vertices, tree,
 * materials, textures with their texels, lights, flags); a scene equal to a
 * cached one but for its camera moves that scene's camera
 * (crt_hip_scene_set_camera_rad) instead of uploading it again; then the
 * blocking render into rgb_out (W*H*3 fp32, top row first).  A new scene is
 * created over crt_auto_gpus_tree GPUs (CRT_HIP_DEVICE=K: device K alone).
 * Thread-safe (one render at a time).  _stats: calls that created a device
 * scene, moved a cached scene's camera, reused one as it was; _reset drops
 * the cache. */
int  crt_hip_render_image_tree(const crt_tree_scene_desc *desc, const crt_renderer_settings *settings,
                               float *rgb_out);
int  crt_hip_render_image_tree_stats(int64_t *creates, int64_t *camera_moves, int64_t *reuses);
void crt_hip_render_image_tree_reset(void);

/* The scene's tree in the reference's preorder numbering, as
 * crt_host_scene_tree (sizes from crt_hip_scene_info). */
int  crt_hip_scene_tree(const crt_hip_scene *scene, float *bounds, int32_t *children, int64_t *leaf_offsets,
                        int32_t *leaf_tris);
/* The secondary-ray BVH (crt_bvh.h; test hook): its node count N (returned;
 * 0 without a BVH) and, when the pointers are non-null, the 8 octant orders
 * of N + 1 32-B records each (crt_layout.h BNode: 6 floats lo_x hi_x lo_y hi_y
 * lo_z hi_z, skip, leaf = first * 16 + count) and the triangle id of every
 * leaf position (id | back_face_culling << 31; triangle_count entries). */
int64_t crt_hip_scene_bvh(const crt_hip_scene *scene, void *nodes_out, int32_t *tri_ids_out);
/* Copy a prepared scene into HBM of `device` (the host scene may be destroyed after). */
int  crt_hip_scene_upload(const crt_host_scene *hs, int device, crt_hip_scene **out);
int  crt_hip_scene_info(const crt_hip_scene *scene, crt_scene_info *out);
void crt_hip_scene_destroy(crt_hip_scene *scene);

/* ---- several GPUs behind one scene handle ----------------------------
 * The reference's render_image spans every hardware thread of the host
 * (crt_renderer.cpp:176-196); a scene created on several devices spans every
 * listed GPU.  The scene is prepared once and replicated on each device; a
 * frame (crt_hip_render / crt_hip_render_device) deals the reference's
 * bucket grid to the replicas (bucket k -> replica k % count, compact shards:
 * only 8x8 tiles with a live pixel), each replica renders its shard on its
 * own stream, the shards are copied peer to peer (xGMI) into the first
 * device and unpacked there.  The image is bit-identical for any count.  A
 * device may be listed more than once (several replicas on it: how a one-GPU
 * host runs the split).  The shard / trace / count entry points act on the
 * first replica. */
int  crt_hip_device_count(void);          /* visible HIP devices; 0 without a GPU */
int  crt_hip_scene_create_on(const crt_scene_desc *desc, const int32_t *devices, int32_t count, int flags,
                             crt_hip_scene **out);
int  crt_hip_scene_from_tree_on(const crt_tree_scene_desc *desc, const int32_t *devices, int32_t count,
                                crt_hip_scene **out);
/* gpu_mask: bit i = HIP device i; 0 = the first N devices for the environment
 * variable CRT_HIP_GPUS=N, else every visible device. */
int  crt_hip_scene_create_mask(const crt_scene_desc *desc, uint64_t gpu_mask, int flags, crt_hip_scene **out);
int  crt_hip_scene_from_tree_mask(const crt_tree_scene_desc *desc, uint64_t gpu_mask, crt_hip_scene **out);
/* The GPU count a frame is spread over when the caller leaves the choice
 * (the CLI, _crt and the crt::render_image shim): 1 unless the frame estimated
 * from the scene and settings (pixels, GI fan-out, recursion, triangles) takes
 * >= 2 ms on one GPU, else about one GPU per 0.6 ms of it, at most `visible`
 * (C2 / C3 stay on one GPU, C4 / C5 spread).  CRT_HIP_GPUS=N
 * overrides.  No GPU needed. */
int  crt_auto_gpus(const crt_scene_desc *desc, const crt_renderer_settings *settings, int visible);
int  crt_auto_gpus_tree(const crt_tree_scene_desc *desc, const crt_renderer_settings *settings, int visible);
/* crt_hip_scene_create_mask / _from_tree_mask over the first crt_auto_gpus devices. */
int  crt_hip_scene_create_auto(const crt_scene_desc *desc, const crt_renderer_settings *settings, int flags,
                               crt_hip_scene **out);
int  crt_hip_scene_from_tree_auto(const crt_tree_scene_desc *desc, const crt_renderer_settings *settings,
                                  crt_hip_scene **out);
/* The multi-GPU probe's decision (run by the create of a handle over >= 2
 * distinct devices, crt_scene_info.multi_probe): 0 keep the replicas, 1 the
 * replicas' probe frame differs from device 0's, 2 a probe render failed
 * (render_status != 0) — both fall back to one GPU.  No GPU needed. */
int  crt_multi_probe_verdict(const float *multi, const float *single, int64_t n, int render_status);
/* Replica devices (devices may be NULL); returns the replica count. */
int  crt_hip_scene_devices(const crt_hip_scene *scene, int32_t *devices, int32_t cap);
/* Kernel ms of each replica's shard in the last render (blocks until done). */
int  crt_hip_last_replica_ms(crt_hip_scene *scene, double *ms, int32_t cap);

/* ---- moving the camera ------------------------------------------------
 * The reference renders whatever camera its Scene holds on every call
 * (render_image, crt_renderer.cpp:157-199; the Blender add-on hands a new
 * scene dict per frame, bl_crt_engine.py:12-31).  A device scene keeps its
 * geometry, trees, BVH, textures and lights and takes a new camera here: the
 * camera's per-frame constants (float(W)/H, std::tan(fov * 0.5f),
 * crt_camera.cpp:23,26-27) are recomputed on the host with the reference's
 * libm, frames already issued keep the camera they were issued with (each
 * frame reads its own device scene record and its own binning camera), and
 * the next frames take the new one — no upload, no host wait.  A new
 * resolution, or a camera for which the camera bins must be built or dropped
 * (the bins need the camera inside the hull margins' origin bound), rebuilds
 * the view's tile plan and buffers with the device drained
 * (crt_scene_info.view_rebuilds).  Every replica of a multi-GPU handle takes
 * the camera.  set_camera converts fov_degrees as the scene loader does
 * (crt_camera.h:20: deg * pi / 180 in float); _rad takes the reference
 * Camera's stored m_fov_radians (crt_tree_scene_desc). */
int  crt_hip_scene_set_camera(crt_hip_scene *scene, const crt_camera_desc *camera);
int  crt_hip_scene_set_camera_rad(crt_hip_scene *scene, const crt_vec3 *location, const float *rotation,
                                  float fov_radians, int32_t width, int32_t height);
/* The current camera (either pointer may be NULL; fov_degrees = fov_radians * 180 / pi). */
int  crt_hip_scene_camera(const crt_hip_scene *scene, crt_camera_desc *camera, float *fov_radians);

/* Blocking drop-in for render_image: rgb_out is caller-allocated W*H*3 fp32,
 * row-major, top row first, unclamped (crt_image.h:11-27). */
int  crt_hip_render(crt_hip_scene *scene, const crt_renderer_settings *settings,
                    float *rgb_out, crt_render_stats *stats);

/* Asynchronous: render the whole frame into device memory d_rgb (W*H*3 fp32)
 * on `stream` (a hipStream_t, NULL = the scene's own stream).
 *
 * Concurrency: a scene holds one set of per-frame scratch state (refill
 * counter, wavefront queues, work counters, timing events).  At most one
 * render of a scene may be in flight at a time: successive asynchronous calls
 * on one scene must be issued on the same stream (or ordered by the caller
 * with events).  Different scenes are independent. */
int  crt_hip_render_device(crt_hip_scene *scene, const crt_renderer_settings *settings,
                           float *d_rgb, void *stream);

/* Multi-GPU: the reference bucket grid (crt_renderer.cpp:160-174) is dealt
 * to shards round-robin (bucket k → shard k % shard_count).  A shard renders
 * its buckets packed, bucket after bucket, each bucket row-major.
 * crt_hip_shard_floats gives the packed size (floats) of one shard;
 * crt_hip_shard_stride the size every shard's slot is padded to for gathers. */
int64_t crt_hip_shard_floats(const crt_hip_scene *scene, int shard, int shard_count);
int64_t crt_hip_shard_stride(const crt_hip_scene *scene, int shard_count);
int  crt_hip_render_shard(crt_hip_scene *scene, const crt_renderer_settings *settings,
                          int shard, int shard_count, float *d_packed, void *stream);
/* Host-side plan of one shard (no GPU): writes up to `cap` buckets as 6 int64
 * each {x, y, w, h, packed_pixel_offset, bucket_index}; returns the number of
 * buckets of the shard (or a negative status). */
int64_t crt_shard_plan(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                       int64_t *buckets_out, int64_t cap);
/* d_gathered holds shard_count slots of crt_hip_shard_stride floats each. */
int  crt_hip_unpack_shards(crt_hip_scene *scene, int shard_count, const float *d_gathered,
                           float *d_rgb, void *stream);
/* Same for 8-bit shards (crt_hip_quantize_rgb8 of each packed shard):
 * d_gathered holds shard_count slots of crt_hip_shard_stride BYTES each. */
int  crt_hip_unpack_shards_rgb8(crt_hip_scene *scene, int shard_count, const uint8_t *d_gathered,
                                uint8_t *d_rgb8, void *stream);

/* Compact shards: the same bucket deal, each bucket cut into 8x8 tiles from its
 * origin, and only LIVE tiles rendered and packed — a tile is live when some
 * pixel's camera ray passes the reference's six-face test on the root cell
 * (node 0 is tested first, crt_intersection.cpp:114-121; a ray failing it is
 * a miss and shade_ray returns the background colour, crt_renderer.cpp:142-144).
 * Lossless: unpacking writes the background into the dead tiles.  The mask is
 * computed once per scene on the device (crt_hip_live_mask: W*H bytes, 1 =
 * live).  On 14-01/scene1 at 1920x1080, 28% of the tiles are live, so a gather
 * moves 3.5x fewer bytes than the full shards.  crt_shard_compact_plan lists a
 * shard's live tiles (5 int64 each: x, y, w, h, packed pixel offset) for a
 * given mask, without a GPU. */
int     crt_hip_live_mask(crt_hip_scene *scene, uint8_t *mask_out);
int64_t crt_hip_compact_floats(crt_hip_scene *scene, int shard, int shard_count);
int64_t crt_hip_compact_stride(crt_hip_scene *scene, int shard_count);
int     crt_hip_render_shard_compact(crt_hip_scene *scene, const crt_renderer_settings *settings, int shard,
                                     int shard_count, float *d_packed, void *stream);
int     crt_hip_unpack_compact(crt_hip_scene *scene, int shard_count, const float *d_gathered, float *d_rgb,
                               void *stream);
int     crt_hip_unpack_compact_rgb8(crt_hip_scene *scene, int shard_count, const uint8_t *d_gathered,
                                    uint8_t *d_rgb8, void *stream);
int64_t crt_shard_compact_plan(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                               const uint8_t *live_mask, int64_t *tiles_out, int64_t cap);

/* write_ppm's per-component conversion on the device (crt_image_ppm.cpp:15-18):
 * d_out[i] = clamp(static_cast<int>(d_rgb[i] * max), 0, max) for n floats
 * (x86 cvttss2si semantics for the cast).  max_color_component <= 255.  Runs
 * on `stream` (NULL = the null stream) of the current device.  Element order
 * is kept, so it applies to whole frames and to packed shards alike. */
int  crt_hip_quantize_rgb8(const float *d_rgb, int64_t n, int32_t max_color_component, uint8_t *d_out,
                           void *stream);

/* Test hook for the a1–a4 known-answer tests: closest hit of n rays
 * (rays = n * 6 floats: origin xyz, direction xyz), host buffers. */
int  crt_hip_trace_batch(crt_hip_scene *scene, const float *rays, int64_t n, crt_hit *hits_out);

/* Test hooks of the camera bins (per 8x8 cell of the frame, the triangles a
 * camera ray of the cell may hit, sorted by a lower bound of the hit
 * distance).  crt_hip_camera_bins runs one frame's device
 * binning (crt_bins.hip) and returns its lists; crt_host_camera_bins the host
 * checker's (build_camera_bins, no GPU).  len_out (cells = ceil(W/8) x
 * ceil(H/8), row-major) gets each cell's list length (-1: more than the cell
 * cap — that cell's pixels walk the BVH); recs_out (96-B records,
 * csrc/crt_layout.h CamCand) the lists back to back in cell order, at most cap
 * records.  Either may be NULL.  Returns the record count (0 and every length 0
 * when the scene takes no camera bins). */
int64_t crt_hip_camera_bins(crt_hip_scene *scene, int32_t *len_out, void *recs_out, int64_t cap);
int64_t crt_host_camera_bins(const crt_host_scene *hs, int32_t *len_out, void *recs_out, int64_t cap);
/* Diagnostics: device ms of one frame's camera binning alone (the two kernels
 * every camera-bins frame runs before its render kernel), averaged over
 * `frames` back-to-back frames on the scene's stream; 0 without camera bins. */
int  crt_hip_bins_time(crt_hip_scene *scene, int32_t frames, double *ms);

/* Work counters of one frame (instrumented variant of the render kernel). */
int  crt_hip_count_work(crt_hip_scene *scene, const crt_renderer_settings *settings,
                        crt_work_counts *out);

/* Wave-level steps of the last crt_hip_count_work frame, for the packet walks
 * (a wave pays once per node / triangle of the union of its lanes' visit sets):
 * node_steps / triangle_steps = wave iterations, edge_steps = triangle steps
 * where some lane ran the edge stage, waves = waves launched.  For wavefront
 * levels >= 1 (cooperative walks): node_steps = loop rounds summed over waves,
 * edge_steps = the longest wave's rounds, waves = waves of those levels.
 * Zero for walks without wave-uniform steps. */
typedef struct crt_wave_counts {
    uint64_t node_steps, triangle_steps, edge_steps, waves;
    uint64_t box_steps;      /* packet walks: node steps where some lane ran the six-face test */
    uint64_t pass_steps;     /* ... where some lane passed it */
    uint64_t window_waves;   /* waves that ran the window walk (their node_steps count every window record) */
    uint64_t window_steps;   /* window walk: windows evaluated */
    uint64_t window_slots;   /* ... lane slots of those windows (records x rays) */
    uint64_t window_reached; /* ... slots whose ray reached the record and kept it alive (hull) */
    uint64_t window_tri_rounds; /* ... rounds of the leaf phase (one triangle per lane group each) */
} crt_wave_counts;
int  crt_hip_wave_counts(crt_hip_scene *scene, crt_wave_counts *out);

/* Options (results are identical for every setting; work and speed differ):
 *   "traversal"  camera walk: 7 = packet walk in the reference's node order
 *                (work counters equal the reference's) | 8 = exact t-pruned
 *                packet walks | 14 = BVH walk + proof on the reference's tree
 *                (default where the scene has a BVH: host-built trees up to
 *                2^18 triangles), camera frames without recursion then take
 *                the camera bins ("bins")
 *   "bins"       0/1 (default 1): camera frames of scenes without reflective /
 *                refractive materials or GI walk per-8x8-cell candidate lists
 *                 where they were built
 *   "bins_split" >= 1 (default 48): cells with this many candidates run as
 *                four 4x4-pixel waves
 *   "bins_quad"  0/1 (default 1): those waves walk the list with four lanes
 *                per pixel
 *   "bins_slack" 0..1000 (default 100): the grid's waves per kind of cell are
 *                the sizing pass's count plus this percentage (room for a
 *                moved camera; cells beyond take a wave's further entries)
 *   "bins_reuse" 0/1 (default 1): a frame whose camera and plan are the last
 *                binning's renders that binning's lists (no binning); 0 bins
 *                every frame (crt_scene_info.bins_binnings / bins_reuses)
 *   "secondary"  walk of secondary rays: 0 = by frame (default: 14 where the
 *                scene has a BVH), 4 = cooperative walk in the reference's
 *                order, 10 = pruned cooperative, 14 = BVH + proof
 *   "wavefront"  0/1 (default 1): level-by-level recursion when GI is off
 *   "window"     0/1 (default 1): the plan's split tiles of <= 16 camera rays
 *                take the window walk
 *   "calibrate"  0 = estimate plan | 1 = measured-cost tile plan, split
 *                threshold tuned by timing candidate plans (long-running
 *                hosts, bench.py) | 2 = measured-cost plan with a fixed
 *                threshold (default; a one-shot caller's first frame of a walk
 *                renders with the estimate plan and the second calibrates)
 *   "calib_k_milli" k x 1000: a fixed split threshold (sets "calibrate" 2)
 *   "calib_min"  1/2/4/8: smallest side a calibrated plan splits tiles to
 *   "gi_refill"  0/1 (default 1): GI frames run persistent waves that refill
 *                finished lanes with the next pixel of the tile list
 *   "gi_machine" 0/1 (default 1): ... as per-lane state machines (k_render_gi)
 *   "wf_rpw"     1..64 (default 48): cap on the rays per wave of wavefront
 *                levels >= 1 with a cooperative walk; a level of n rays takes
 *                min(cap, max(8, n / 4096)) and the other lanes start idle and
 *                take donated pieces
 *   "wf_replay"  1 (default): a wavefront frame whose settings and tile list
 *                were rendered before launches every level with the recorded
 *                level sizes, no host read-back | 0: read every level's size
 *                back | 2: tests only, recorded sizes minus one (overflow path)
 *   "wf_graph"   0/1 (default 1): such frames run as a HIP graph captured on
 *                their first replay (per tile list, settings, output, stream)
 *   "wf_dynamic" 1 (default): a wavefront frame with no recorded sizes (a new
 *                camera, tile list or settings) sizes its levels on the device
 *                — no read-back; queues of 2 x the camera rays, "wf_dyn_ids"
 *                (default 4) x the camera rays of ray ids, grids of at most
 *                "wf_dyn_waves" (default 8192) waves striding over a level —
 *                and its sizes are recorded behind it; a level past those
 *                capacities is reported like a recorded-size overflow and the
 *                next frame reads its sizes back | 0: read-backs
 *   "trace_walk" 0 = reference order, 1 = pruned per-ray walk, 2 = BVH + proof
 *                (crt_hip_trace_batch)
 *   "events"     0/1 (default 1): start/stop events around every render
 *   "shadows"    0/1 (default 0): trace the shadow rays — NOT HEAD's image.
 *                At HEAD trace_ray_with_refractions never runs its loop
 *                (crt_renderer.cpp:29-44) and every light is unoccluded; the
 *                course's earlier renderer traced them (:90-92: a light counts
 *                when the shadow ray's closest hit is absent or farther than
 *                the light), which its committed renders 09-02/scene3 and
 *                09-03/scene5 show at every pixel.  A separate report
 *                (bench.py --shadows), never the HEAD-parity headline; the
 *                frame runs the frame-stack kernel with per-lane shadow walks,
 *                and crt_hip_count_work counts the shadow rays as traversals.
 * Environment overrides of these (CRT_TRAVERSAL, ...) exist in A/B builds only
 * (-DCRT_AB_OPTIONS). */
int  crt_hip_scene_set_option(crt_hip_scene *scene, const char *name, int value);

/* Diagnostics: the full-frame tile plan in dispatch order (x, y, w, h per
 * tile) and each tile's measured walk cost (wave steps; 0 without a
 * calibrated plan).  With NULL xywh returns the tile count. */
int  crt_hip_plan_tiles(crt_hip_scene *scene, const crt_renderer_settings *settings, int32_t *xywh, float *cost,
                        int64_t cap);

/* The full-frame tile plan in use.  A calibrated plan splits a tile whose
 * measured cost exceeds calib_k x the mean cost per wave slot into 4x4 / 2x2
 * tiles (window walk); k is tuned per scene by timing the candidate plans'
 * frames (or fixed: "calibrate" 2 with env CRT_CALIB_K / "calib_k_milli"). */
typedef struct crt_plan_info {
    double  calib_k;       /* 0: no calibrated plan */
    int32_t tiles;         /* waves of the full-frame plan */
    int32_t small_tiles;   /* split tiles of <= 16 pixels */
} crt_plan_info;
int  crt_hip_plan_info(const crt_hip_scene *scene, crt_plan_info *out);

/* Diagnostics: render one full frame with per-wave s_memrealtime stamps
 * (100 MHz ticks; stamps = 2 per wave of the render grid: start, end;
 * tile_xy = the origin of the wave's tile, in dispatch order, -1 for a wave
 * with nothing to do — an unused camera-bins priority slot, stamps 0).  With
 * NULL buffers returns the wave count. */

int  crt_hip_profile_waves(crt_hip_scene *scene, const crt_renderer_settings *settings, uint64_t *stamps,
                           int64_t cap, int32_t *tile_xy);

/* Device-side stats of the last crt_hip_render_device launch on `scene`:
 * device time in ms between the launch's start/stop events (blocks). */
int  crt_hip_last_kernel_ms(crt_hip_scene *scene, double *ms);

/* Defaults of crt_renderer.h:10-16. */
void crt_renderer_settings_default(crt_renderer_settings *out);

/* ---- host output (crt_image_ppm.cpp:9-23) ---------------------------- */
int  crt_write_ppm(const char *path, const float *rgb, int32_t width, int32_t height,
                   int32_t max_color_component);

const char *crt_hip_last_error(void);
int  crt_hip_abi_version(void);
/* Hash of the library's sources and build flags (measurements name the build). */
const char *crt_hip_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* CRT_HIP_H */
