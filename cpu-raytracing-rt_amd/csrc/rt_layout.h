// rt_layout.h — the scene as it lives in HBM.
//
// The reference's scene (scene.rs:56-90) is a tree of Rust structs; here it is
// flattened into read-only arrays split into HOT data (read on every test) and
// COLD data (read once per shaded hit):
//   * BVH nodes: pre-order like bvh.rs:104 (root = 0, left child = node + 1),
//     one 128-B "fat" node per node holding BOTH children's f64 boxes, so a
//     visit is one aligned 128-B line (the reference reads two 80-B Nodes
//     scattered in a Vec, bvh.rs:158-159).
//   * shapes (plane/box/ellipsoid): 80-B hot record {shape, position, rotation}
//     = the model-space transform of intersections.rs:93-99.
//   * triangles: 80-B hot record {a, ba, ca} (the 3x3 solve of
//     triangle.rs:49-67); normals / 1/area / material in cold SoA arrays.
#pragma once
#include <stdint.h>

namespace rt {

#ifndef RT_SHORT_STACK
#define RT_SHORT_STACK 12
#endif
constexpr int kMaxBvhDepthShort = RT_SHORT_STACK;   // per-lane short stack kept in LDS
// The 4-wave resumable path kernel's short stack: shorter, so the path's
// throughput and radiance fit in its LDS too (render.hip path_kernel)
#ifndef RT_SHORT_STACK_RES
#define RT_SHORT_STACK_RES 8
#endif
constexpr int kShortRes = RT_SHORT_STACK_RES;
constexpr int kMinShort = kShortRes < kMaxBvhDepthShort ? kShortRes : kMaxBvhDepthShort;  // spill sizing

struct alignas(128) DevNode {
    double lmin[3], lmax[3];   // left child's box  (bvh.rs:158)
    double rmin[3], rmax[3];   // right child's box (bvh.rs:159)
    int32_t left, right;       // child indices, -1 for a leaf
    uint32_t start, count;     // leaf primitive range [start, start+count)
    // the children's primitive ranges (count 0 = internal child): a descent
    // learns whether it enters a leaf without loading the child's line
    uint32_t lstart, lcount, rstart, rcount;
};
static_assert(sizeof(DevNode) == 128, "fat node is one 128-B line");

// Stack / child word of a BVH child (render.hip trav_step): an internal child is
// its node index (< 2^30, checked by the host); a leaf whose range fits is
// packed as 1|count(7)|start(24), so reaching it loads nothing; a leaf that does
// not fit is its node index | kLeafRef, and its range is loaded from the node.
constexpr uint32_t kPackedLeaf = 0x80000000u, kLeafRef = 0x40000000u;
#ifdef __HIPCC__
__host__ __device__
#endif
inline uint32_t child_word(uint32_t node, uint32_t start, uint32_t count) {
    if (count == 0) return node;
    if (count < 128u && start < (1u << 24)) return kPackedLeaf | (count << 24) | start;
    return node | kLeafRef;
}

// Compact triangle-BVH node (DESIGN.md §2 "compact layout"): both children's
// boxes as f32 — exact copies, the host checks that every coordinate of the
// f64 boxes round-trips through f32 — plus the children's words.  64 B instead
// of 128: a visit reads four 16-B words.  Slot order (scene_build.cpp
// build_compact): the INTERNAL nodes in pre-order first (so an internal node's
// internal left child is the next slot), then the few big leaves a child word
// cannot pack.  A child word is an internal child's slot, a packed leaf
// kPackedLeaf | count << 24 | leaf-block index (kLeafBlock, not a primitive
// index), or a big leaf's slot | kLeafRef, whose entry holds its block index in
// `start` and its primitive count in `count`.
struct alignas(64) DevNodeC {
    float lmin[3], lmax[3], rmin[3], rmax[3];
    uint32_t lw, rw;            // child words of an internal node
    uint32_t start, count;      // a leaf's own range
};
static_assert(sizeof(DevNodeC) == 64, "compact node is half a line");
// Compact triangle record: the vertices a, b, c as f32 (36 B, exact copies; the
// device rebuilds ba = b - a, ca = c - a in f64 — the same bits as the host's,
// which triangle_props computed from the same a, b, c).
constexpr uint32_t kTriC = 9;   // floats per compact triangle record
// Compact records are stored in leaf blocks (round 4, scene_build.cpp build_compact): a
// leaf's records behind a one-word header (its first primitive index), the block on a
// 128-B line; a leaf's child word / big-leaf entry carries the block index.
constexpr uint32_t kLeafBlock = 32;  // floats per 128-B line

// Pair layout (round 6, scene_build.cpp build_pairs): one 128-B line per internal
// compact slot c, two 64-B halves for c's left and right child K:
//   floats 0..5  box A, 6..11 box B, then words 12 A's word, 13 B's word, 14 K's own
//   word (its child word in c), 15 flags.
// K internal: A / B = K's children's boxes and words (what a visit of K tests); K's own
// box is their union.  K a leaf (flags kPairLeaf): A = B = K's box (the union again).  A visit of c reads
// c's line, tests both children and can visit the near child K from the same line:
// two BVH levels per dependent load.  Slot indices are the compact ones.
constexpr uint32_t kPairFloats = 32, kPairHalf = 16;
constexpr uint32_t kPairLeaf = 1u;

struct alignas(16) DevShape {  // Primitive<T> hot part (scene.rs:20-27)
    double shape[3];           // plane normal | box half sizes | ellipsoid radii
    double pos[3];
    double rot[4];             // (s, x, y, z)
    // host-precomputed constants (same IEEE ops as the device would do):
    //   ellipsoid: aux = dev_rcp(r) per axis (written by the device, api.cpp)
    //   box:       aux[0] = 1/sum/8 (intersection_probability.rs:15-23)
    double aux[3];
    // kShapeFast: identity rotation, position (and box sizes / plane normal)
    // in coord_fast range, nonzero box sizes, dir_ok radii — a ray_fast ray
    // may then take dev_quot for this shape's quotients
    // (rt_device.h shape_fast).  kPlaneAxis: plane normal = sign * e_axis.
    uint32_t flags;
    uint32_t axis;             // plane: 0..2, bit 2 = negative sign
};
// kBoxSizes: a box whose half sizes are nonzero and in coord_fast range (any
// rotation): box_model may then take dev_quot on the model-space ray.
constexpr uint32_t kShapeFast = 1u, kPlaneAxis = 2u, kBoxSizes = 4u;
static_assert(sizeof(DevShape) == 112, "shape record");

struct alignas(16) DevTri {    // Triangle hot part (triangle.rs:5-17)
    double a[3], ba[3], ca[3];
    double pad;
};
static_assert(sizeof(DevTri) == 80, "triangle record");

struct DevTriCold {            // read only on a hit
    double ng[3], na[3], nb[3], nc[3];
};

struct DevMaterial {           // Metadata (scene.rs:13-18)
    uint32_t kind, pad;
    double ior;
    double color[3], emission[3];
    // dielectric constants of raytrace.rs:36-54, host-computed with the same IEEE
    // ops: k_out = 1 / ior (entering; inside, n1 / n2 = ior / 1 = ior exactly) and
    // r0 = ((n1 - n2) / (n1 + n2))^2 of reflection_power (raytrace.rs:62-65), the
    // same bits for both sides (the quotient only changes sign)
    double k_out, r0;
};

struct DevBvh {
    const DevNode* nodes;
    double root_min[3], root_max[3];
    uint32_t n_prims;
    uint32_t depth;            // levels (root = 1)
    uint32_t fast;             // every box coordinate is 0 or in [2^-397, 2^400] (coord_fast)
    uint32_t tri_q;            // every triangle edge component is 0 or in [2^-149, 2^129)
                               // (rt_device.h tri_uvt_r: the split-division solve)
    // primitives in BVH order: exactly one of these is non-null
    const DevShape* shapes;
    const DevTri* tris;
    const DevTriCold* tri_cold;
    const double* tri_inv_area;
    const uint32_t* mat;       // material per primitive
    const int32_t* gid;        // global primitive id per primitive
    // the compact layout of a triangle BVH (DevNodeC + kTriC floats per triangle),
    // non-null only when every box coordinate and vertex is an exact f32
    const DevNodeC* cnodes;
    const float* ctris;
    const float* pnodes;       // pair layout (kPairFloats per internal compact slot) or null
};

struct DevScene {
    uint32_t n_planes;
    uint32_t n_lights;         // boxes + ellipsoids + triangles in the light BVHs
    uint64_t light_zone;       // exact UniformInt acceptance zone for gen_index(n_lights)
    const DevShape* planes;
    const uint32_t* plane_mat;
    const int32_t* plane_gid;
    DevBvh boxes, ells, tris;          // ScenePrimitives (scene.rs:56-62)
    DevBvh lboxes, lells, ltris;       // LightPrimitives (scene.rs:64-69)
    const DevMaterial* mats;
    uint32_t max_depth;                // max BVH depth over the six (stack bound)
    // with_rotated_normal (intersections.rs:32-39) of the per-primitive constant
    // normals, computed on the host with the device's ops: plane [n][side][3]
    // (side = aux bit0), box in BVH order [n][aux & 7][3] (face dim, sign bit)
    const double* plane_nrm;
    const double* box_nrm;
    // Shared light tests (render.hip boxes_slt): bit i set <=> scene box i (BVH
    // order) is the next light box of lboxes.  Nonzero only when every light is
    // a box, both box BVHs are single leaves and the light copies are the scene
    // records selected by the mask, in order: the light pdf of a diffuse bounce
    // then comes from the next segment's own box tests (same ray, same records).
    uint32_t slt_mask;
    // Last-bounce light query (render.hip segment_shade): nonzero only
    // when every light is a box (at most kLqBoxes), each with a finite positive
    // density.  Then a light query whose origin lies outside every box below (the
    // lights' world boxes grown by a margin) has no crossing at t <= 0, so every
    // term t^2 / |d.n| * density is positive or +inf and the pdf cannot be NaN; on
    // the path's last bounce, where only the pdf's NaN-ness is observable, the
    // timed kernel skips such queries.
    uint32_t lq_boxes;
    double lq_box[4][6];       // [light][min xyz, max xyz]
};
constexpr uint32_t kLqBoxes = 4;

}  // namespace rt
