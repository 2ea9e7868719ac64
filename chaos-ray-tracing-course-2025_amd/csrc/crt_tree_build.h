/*
 * crt_tree_build.h — device-side exact build of the acceleration tree and of
 * the layouts the walks read (crt_tree_build.hip).
 *
 * Replaces, on the GPU: acceleration_tree::build / build_branch
 * (crt_acceleration_tree.cpp:13-106), AABB::split / intersects
 * (crt_aabb.h:24-45), and the host flattening of crt_scene_build.cpp
 * (traversal-ordered DNode array, 8 octant PNode orders with hulls, leaf slots).
 */
#pragma once
#include <stdint.h>

#include <vector>

#include "crt_host.h"
#include "crt_layout.h"

namespace crt_amd {

/* Device arrays of a built tree (all allocated with hipMalloc, listed in
 * `allocs`; the caller frees them). */
struct DeviceTree {
    DNode *nodes = nullptr;            /* node_count, reference LIFO visit order */
    PNode *pnodes = nullptr;           /* 8 x (node_count + 1), pnode_order */
    DTriGeo *slots = nullptr;          /* slot_count, reference visit order */
    int32_t *slot_tri = nullptr;
    uint8_t *slot_cull = nullptr;
    uint32_t *slot_cull_bits = nullptr;
    /* the tree in the reference's own numbering (crt_hip_scene_tree) */
    float *ref_bounds = nullptr;       /* 6 per node */
    int32_t *ref_children = nullptr;   /* 2 per node */
    int64_t *ref_leaf_off = nullptr;   /* node_count + 1 */
    int32_t *ref_leaf_tris = nullptr;  /* slot_count */
    int32_t node_count = 0;
    int64_t slot_count = 0;
    int64_t leaf_count = 0;
    int32_t max_depth = 0;
    int32_t max_leaf_size = 0;
    int32_t planes_ok = 1;             /* crt_device.h coord_ok on every node plane */
    int32_t levels = 0;
    double build_ms = 0.0;             /* host wall time of the whole build */
    std::vector<void *> allocs;
};

/* Build from a HostScene whose mesh prep is done (vpos, tri_attr,
 * face_normal, tri_cull, root_box, prune_origin_max) on the current device,
 * on `stream` (a hipStream_t); blocks until done.  Returns CRT_OK or a
 * CRT_E_* status (crt_hip_last_error). */
int build_tree_device(const HostScene &hs, void *stream, DeviceTree &out);

}  // namespace crt_amd
