/*
 * crt_host.h — host-side (C++) scene preparation shared by the C-ABI layer.
 */
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/crt_hip.h"
#include "crt_layout.h"

namespace crt_amd {

/* Thread-local error channel behind crt_hip_last_error(). Returns `code`. */
int set_error(int code, const std::string &msg);

/* Owned storage behind a crt_scene_file (the parsed .crtscene). */
struct SceneFile {
    crt_scene_desc desc;
    struct Mesh {
        std::vector<float> positions, uvs;
        bool has_uvs = false;
        std::vector<int32_t> indices;
        int32_t material_index = 0;
    };
    std::vector<Mesh> meshes_storage;
    std::vector<crt_mesh_desc> meshes;
    std::vector<crt_material_desc> materials;
    std::vector<crt_texture_desc> textures;
    std::vector<crt_light_desc> lights;
    /* decoded bitmap texels (rgb fp32, byte / 255.0f), indexed like textures */
    std::vector<std::vector<float>> bitmaps;
    std::string warning;
    void relink();
};

int parse_scene_json(const char *text, size_t len, const char *asset_root, SceneFile &out);

/* read_stb (crt_image_stbi.cpp:16-40) without stb: decode an image file's
 * bytes into 8-bit RGB (crt_image_decode.cpp).  comps = the file's component
 * count as stbi_load reports it; false (with why) where read_stb fails. */
bool decode_image_rgb8(const uint8_t *bytes, size_t len, int &w, int &h, int &comps, std::vector<uint8_t> &rgb,
                       std::string &why);

/* The scene after mesh prep and tree build, in device layout (crt_layout.h). */
struct HostScene {
    /* camera / settings */
    float background[3];
    float cam_loc[3];
    float cam_rot[9];
    int32_t width = 0, height = 0;
    float fov_radians = 0.f;
    float aspect = 0.f, tan_half_fov = 0.f;
    int32_t bucket_size = 24;
    bool gi_on = false, reflections_on = true, refractions_on = true;

    /* geometry (global ids: vertex/triangle order of crt_mesh.cpp) */
    std::vector<float> vpos;            /* 3 per vertex */
    std::vector<DVec4> vnormal, vuv;
    std::vector<DTriAttr> tri_attr;
    std::vector<float> face_normal;     /* 3 per triangle */
    std::vector<uint8_t> tri_cull;

    /* tree, reference numbering (preorder, child0 subtree first) */
    std::vector<float> ref_bounds;      /* 6 per node */
    std::vector<int32_t> ref_children;  /* 2 per node */
    std::vector<int64_t> ref_leaf_off;  /* n+1 */
    std::vector<int32_t> ref_leaf_tris;
    std::vector<int32_t> ref_depth;

    /* tree, device layout (traversal order) */
    std::vector<DNode> nodes;
    std::vector<DTriGeo> slots;
    std::vector<int32_t> slot_tri;
    std::vector<uint8_t> slot_cull;

    /* pruned walks (crt_layout.h PNode): 8 octant orders x (nodes.size() + 1) */
    std::vector<PNode> pnodes;
    float prune_origin_max = 0.f;
    double prune_G = 0.0;           /* the G of the hull margins (crt_scene_build.cpp) */

    /* secondary-ray BVH (crt_bvh_build.cpp, crt_layout.h BNode): 8 octant
     * orders x (bnode_count + 1) nodes, triangles in leaf order */
    std::vector<BNode> bnodes;
    int32_t bnode_count = 0;
    std::vector<DTriGeo> btri;
    std::vector<int32_t> btri_id;   /* triangle id | back_face_culling << 31 */
    /* the BVH proof's tree topology (crt_layout.h KTopo; build_proof_tables) */
    std::vector<KTopo> ktopo;
    std::vector<KTopo2> ktopo2;   /* per node: its children and grandchildren (verify_topo) */


    /* root cell (crt_acceleration_tree.cpp:89-94); tree_on_host = false when
     * prepare_scene skipped the tree (built on the device, crt_tree_build.h) */
    float root_box[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool tree_on_host = true;
    bool device_bvh = true;             /* scenes above kHostBvhMax triangles: BVH built on the device
                                         * (create flag CRT_SCENE_NO_DEVICE_BVH: none) */

    /* shading */
    std::vector<DMaterial> materials;
    std::vector<DTexture> textures;
    std::vector<DVec4> texels;
    std::vector<DLight> lights;

    /* stats */
    double tree_build_ms = 0.0, bvh_ms = 0.0, prep_ms = 0.0;   /* wall time of the host builds */
    int64_t leaf_count = 0;
    int32_t max_depth = 0;
    int32_t max_leaf_size = 0;
};

/* The camera of hs as the kernels see it (crt_layout.h DCamera). */
DCamera host_camera(const HostScene &hs);
/* A camera from the reference's Camera fields (crt_camera.h:16-21: location,
 * rotation, the stored m_fov_radians, resolution), with the per-frame
 * constants float(W)/H and std::tan(fov * 0.5f) of crt_camera.cpp:23,26-27
 * computed once by this process's libm.  false: non-positive resolution. */
bool make_camera(const float loc[3], const float rot[9], float fov_radians, int32_t width, int32_t height,
                 DCamera &out);
/* crt_camera.h:20 (crt_json.cpp camera "fov"): m_fov_radians from degrees, float ops. */
inline float fov_degrees_to_radians(float deg) { return deg * 3.14159265358979323846f / 180.0f; }

/* The secondary-ray BVH over hs's triangles (crt_bvh_build.cpp); needs the
 * mesh prep and prune_G. */
int build_bvh(HostScene &hs);
/* scenes above this many triangles get the device-built BVH (crt_lbvh.hip) */
constexpr size_t kHostBvhMax = (size_t)1 << 18;

/* The topology records of the flattened tree hs.nodes (crt_layout.h KTopo)
 * for crt_bvh.h verify_topo (crt_bvh_build.cpp); none (verify_kd then) if a
 * child cell is not its parent's half. */
int build_proof_tables(HostScene &hs);

/* Camera bins of hs's camera and resolution (crt_bins.h; the host checker of
 * the device binning, crt_bins.hip): for each 8x8 cell of the frame
 * (row-major, (width + 7) / 8 a row), every triangle a camera ray of the cell
 * may hit, sorted by (dmin, id): cell c holds bins[off[c] .. off[c + 1]); a
 * cell with more than kBinCellCap candidates holds none and is marked in
 * *over (its pixels walk the BVH).  Leaves everything empty (the scene then
 * walks the BVH) when bin_camera fails or the lists would be too long. */
struct BinCamera;
int build_camera_bins(const HostScene &hs, std::vector<CamCand> &bins, std::vector<int32_t> &off,
                      std::vector<uint8_t> *over = nullptr);
/* The projection constants of hs's camera (false: no bins — the camera is too
 * far for the hull margins, its matrix singular or the field of view bad). */
bool bin_camera(const HostScene &hs, BinCamera &cam);
/* Same for any camera of a scene (prune_origin_max: the hull margins' origin
 * bound, crt_scene_build.cpp). */
bool bin_camera_of(const DCamera &c, float prune_origin_max, BinCamera &cam);
/* Per-triangle static part of the candidate records (hull box, id, geometry). */
void bin_templates(const HostScene &hs, std::vector<CamCand> &tpl);

/* Light bins (crt_layout.h DLightBin, crt_light_bins.cpp) of every light over
 * the triangles' templates: N x N cells a cube face, for rays passing their
 * light within e_max.  False (out empty) when no light takes bins. */
struct LightBinsHost {
    int n = 0;
    std::vector<DLightBin> par;
    std::vector<int32_t> off;
    std::vector<LightCand> recs;
};
bool build_light_bins(const CamCand *tpl, int nt, const DLight *lights, int nl, double e_max, int N,
                      LightBinsHost &out);

/* Mesh prep + (build_tree) the exact tree build and its flattening. */
int prepare_scene(const crt_scene_desc *desc, HostScene &out, bool build_tree = true);
/* The reference's built scene (vertices + tree) flattened as it is. */
int prepare_scene_from_tree(const crt_tree_scene_desc *desc, HostScene &out);

/* Screen-space work estimate: every leaf cell is projected through the camera
 * and its triangle count added to the 8x8 tiles its image overlaps.  Used only
 * to dispatch expensive tiles first (results do not depend on it). */
std::vector<float> tile_work_estimate(const HostScene &hs, int tiles_x, int tiles_y);
/* Same from the tree in the reference's numbering, for any camera. */
std::vector<float> tile_work_estimate_of(const DCamera &c, const std::vector<float> &ref_bounds,
                                         const std::vector<int32_t> &ref_children,
                                         const std::vector<int64_t> &ref_leaf_off, int tiles_x, int tiles_y);

/* The reference bucket grid (crt_renderer.cpp:160-174) dealt round-robin to
 * shard_count shards; returns the buckets of `shard` with packed offsets and
 * the shard's packed pixel count. */
std::vector<DBucket> shard_buckets(int32_t width, int32_t height, int32_t bucket_size, int shard,
                                   int shard_count, int64_t *packed_pixels);

/* The shard's buckets cut into 8x8 tiles from each bucket origin, keeping the
 * tiles with a live pixel (live: W*H bytes, null = all live), packed in order;
 * the other tiles are appended to *dead (packed_offset -1) when given. */
std::vector<DBucket> shard_live_tiles(int32_t width, int32_t height, int32_t bucket_size, int shard, int shard_count,
                                      const uint8_t *live, int64_t *packed_pixels, std::vector<DBucket> *dead);

/* Host half of the compact image copy (crt_host_copy.cpp, crt_api.hip
 * image_to_host).  fill_background: n pixels of the colour bg from dst on;
 * store_fence() orders a thread's stores before a handover to another. */
void fill_background(float *dst, int64_t n, const float bg[3]);
void store_fence();

/* crt_hip_render with a check that the image copy's host threads run while
 * the frame renders (crt_shim_core.cpp: the cached scene's content against
 * the caller's Scene): check(arg, i, n) for i < n; if any returns false,
 * *mismatch is set and the image in rgb_out is not to be used. */
int render_checked(crt_hip_scene *sc, const crt_renderer_settings *st, float *rgb_out, crt_render_stats *stats,
                   bool (*check)(void *, int, int), void *check_arg, bool *mismatch);

/* Persistent host threads that run the bands of a host-side image copy with
 * the calling thread: task i of n runs on thread i mod (workers + 1), the
 * caller taking i = 0, T, 2T...  Workers spin for a while after each job (a
 * frame's copy follows the previous one closely) and then sleep. */
class HostPool {
public:
    static HostPool &get();
    int threads() const;                                    /* workers + the caller */
    void run(int n, void (*fn)(void *, int), void *arg);   /* returns when all n tasks ran */
    ~HostPool();

private:
    explicit HostPool(int workers);
    struct Impl;
    Impl *impl_;
};

}  // namespace crt_amd
