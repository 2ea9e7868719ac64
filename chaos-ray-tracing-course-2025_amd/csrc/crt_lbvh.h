/*
 * crt_lbvh.h — device build of the secondary-ray BVH (crt_bvh.h, crt_layout.h
 * BNode) for scenes too large for the host SAH build (crt_bvh_build.cpp,
 * > 2^18 triangles): a linear BVH over 30-bit Morton codes of the triangles'
 * box centres (crt_lbvh.hip).
 *
 * Same contract as the host build: every triangle once, each box the union of
 * its triangles' conservative hulls (crt_device.h triangle_hull, rounded
 * outwards), 8 octant orders in preorder with the near child first and skip
 * links, leaves of at most kLbvhLeaf triangles; only the tree's shape differs
 * (the walk's exactness rests on the boxes alone, crt_bvh.h).
 */
#pragma once
#include <stdint.h>

#include <vector>

#include "crt_host.h"
#include "crt_layout.h"

namespace crt_amd {

struct DeviceBvh {
    BNode *bnodes = nullptr;     /* 8 x (node_count + 1) */
    DTriGeo *btri = nullptr;     /* triangles in leaf order */
    int32_t *btri_id = nullptr;  /* triangle id | back_face_culling << 31 */
    int32_t node_count = 0;
    int32_t max_depth = 0;       /* deepest node (root 0) */
    double build_ms = 0.0;       /* host wall time of the whole build (upload included) */
    std::vector<void *> allocs;  /* device buffers the caller frees */
};

/* Build from a HostScene whose mesh prep is done (vpos, tri_attr,
 * face_normal, tri_cull, prune_G) on the current device, on `stream`
 * (a hipStream_t); blocks until done.  Returns CRT_OK or a CRT_E_* status. */
int build_bvh_device(const HostScene &hs, void *stream, DeviceBvh &out);

}  // namespace crt_amd
