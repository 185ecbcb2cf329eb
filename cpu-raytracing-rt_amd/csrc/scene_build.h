// scene_build.h — host-side Scene::new / make_scenes / BVH::new
// (scene.rs:92-223, bvh.rs:11-140, 224-256) producing the flattened HBM
// layout of rt_layout.h.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_layout.h"
#include "rt_math.h"

namespace rt {

struct Triangle {            // triangle.rs:5-17
    V3 a, ba, ca, ng;
    double inv_area;
    V3 na, nb, nc;
};
Triangle triangle_props(V3 a, V3 b, V3 c);                          // triangle.rs:41-47
Triangle triangle_smooth(V3 a, V3 b, V3 c, V3 na, V3 nb, V3 nc);    // triangle.rs:20-23
Triangle triangle_geometric(V3 a, V3 b, V3 c);                      // triangle.rs:25-28

// One BVH in host form: pre-order nodes + primitive permutation.
struct HostNode {
    Box3 box;
    int64_t left = -1, right = -1;
    uint64_t start = 0, end = 0;
};
struct HostBvh {
    std::vector<HostNode> nodes;
    std::vector<uint64_t> order;   // order[i] = list index of the i-th primitive in BVH order
    uint32_t depth = 0;
};
// BVH::new over primitive boxes given in list order (bvh.rs:12-17).
HostBvh build_bvh(const std::vector<Box3>& boxes);

// Flattened scene ready for upload: every array is a host vector that maps
// 1:1 onto a device allocation (see api.cpp).
struct HostBvhArrays {
    std::vector<DevNode> nodes;
    Box3 root;
    uint32_t n_prims = 0, depth = 0;
    bool fast = false;  // all box coordinates pass coord_fast (DevBvh::fast)
    bool tri_q = false;  // every triangle edge component 0 or in [2^-149, 2^129) (DevBvh::tri_q)
    std::vector<DevShape> shapes;
    std::vector<DevTri> tris;
    std::vector<DevTriCold> tri_cold;
    std::vector<double> tri_inv_area;
    std::vector<uint32_t> mat;
    std::vector<int32_t> gid;
    // compact layout of a triangle BVH (rt_layout.h DevNodeC, kTriC floats per
    // triangle): filled only when every box coordinate and vertex is an exact f32
    std::vector<DevNodeC> cnodes;
    std::vector<float> ctris;
    // pair layout over the compact nodes (rt_layout.h kPairFloats per internal slot),
    // filled when every internal child's box is the union of its children's
    std::vector<float> pnodes;
};
struct HostScene {
    std::vector<DevMaterial> mats;
    std::vector<DevShape> planes;
    std::vector<uint32_t> plane_mat;
    std::vector<int32_t> plane_gid;
    HostBvhArrays bvh[6];   // boxes, ellipsoids, triangles, light boxes, light ellipsoids, light triangles
    double build_ms = 0.0;
};
// Returns empty string on success, else an error message.
std::string build_scene(const rt_scene_desc& desc, HostScene& out);

}  // namespace rt
