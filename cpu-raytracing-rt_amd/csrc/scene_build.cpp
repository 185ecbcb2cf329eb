// scene_build.cpp — host scene model + reference BVH builder (deterministic).
//
// Restates, for the product:
//   make_scenes            scene.rs:194-223  (split per kind, lights are copies)
//   Primitive::new         scene.rs:108-123  (rotated_aabb + position, :255-268)
//   TrianglePrimitive::new scene.rs:139-165  (custom-format triangles)
//   instantiate            gltf/scene_builder.rs:42-55 (glTF triangles)
//   BVH::new/build_nodes   bvh.rs:12-17, 75-140, 224-256
// The reference sorts with sort_unstable_by(midpoint.total_cmp) (bvh.rs:102,121),
// whose order for equal midpoints is unspecified; here ties are broken by the
// primitive's list index so every build of the same input gives the same tree.
#include "scene_build.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

namespace rt {

Triangle triangle_props(V3 a, V3 b, V3 c) {
    Triangle t;
    t.a = a;
    t.ba = b - a;
    t.ca = c - a;
    V3 sized = cross(t.ba, t.ca);
    double area = sqrt(dot(sized, sized)) / 2.0;
    t.ng = normalize(sized);
    t.inv_area = 1.0 / area;
    return t;
}
Triangle triangle_smooth(V3 a, V3 b, V3 c, V3 na, V3 nb, V3 nc) {
    Triangle t = triangle_props(a, b, c);
    t.na = na; t.nb = nb; t.nc = nc;
    return t;
}
Triangle triangle_geometric(V3 a, V3 b, V3 c) {
    Triangle t = triangle_props(a, b, c);
    t.na = t.ng; t.nb = t.ng; t.nc = t.ng;
    return t;
}

namespace {

Box3 rotated_box(const Box3& b, Quat r) {  // scene.rs:255-268
    V3 mn = b.min, mx = b.max;
    Box3 o = box_empty();
    box_extend(o, rotate(r, v3(mn.x, mn.y, mn.z)));
    box_extend(o, rotate(r, v3(mn.x, mn.y, mx.z)));
    box_extend(o, rotate(r, v3(mn.x, mx.y, mn.z)));
    box_extend(o, rotate(r, v3(mn.x, mx.y, mx.z)));
    box_extend(o, rotate(r, v3(mx.x, mn.y, mn.z)));
    box_extend(o, rotate(r, v3(mx.x, mn.y, mx.z)));
    box_extend(o, rotate(r, v3(mx.x, mx.y, mn.z)));
    box_extend(o, rotate(r, v3(mx.x, mx.y, mx.z)));
    return o;
}

constexpr uint64_t kParallelBuildMin = 200000;  // primitives: below this one thread builds

inline int64_t total_key(double x) {  // f64::total_cmp as an integer key
    int64_t b;
    std::memcpy(&b, &x, 8);
    b ^= (int64_t)(((uint64_t)(b >> 63)) >> 1);
    return b;
}
inline double score(const Box3& b) {  // bvh.rs:115-118
    V3 s = b.max - b.min;
    return s.x * s.y + s.x * s.z + s.y * s.z;
}

// build_nodes (bvh.rs:75-113) in O(n log n) with the identical result.
//
// The reference re-sorts every node's primitives by midpoint on each axis
// (bvh.rs:102,121, here with ties by list index: a total order).  A total order
// restricted to a subset is the subset's sorted order, so each axis is sorted
// ONCE (S[a]) and a split stably partitions the other two axes' lists: every
// node then sees exactly the sequences the reference sorts, the SAH sweeps run
// the same float operations in the same order (same strict-< first minimum),
// nodes are numbered in the same pre-order, and leaves keep the reference's
// primitive order — the parent's split-axis order for n <= 4 (the root: list
// order), the axis-2 order (the last sort) for a SameNode leaf.
struct Builder {
    const std::vector<Box3>& boxes;
    std::vector<int64_t> key[3];   // midpoint sort key per axis and primitive
    // positions lo..hi of a node hold its primitives sorted on each axis (S) and
    // their boxes in the same order (SB, so sweeps stream instead of gathering)
    std::vector<uint64_t> S[3];
    std::vector<Box3> SB[3];
    std::vector<uint64_t>& order;  // output: leaf primitives, leaf ranges as in the reference
    // scratch indexed by position (disjoint per node, so subtrees build concurrently)
    std::vector<double> bwd_score;
    std::vector<uint8_t> left_flag;  // indexed by primitive id (disjoint per node)
    std::vector<uint64_t> tmp_i;
    std::vector<Box3> tmp_b;

    struct Out {  // nodes of one (sub)tree in local pre-order
        std::vector<HostNode> nodes;
        uint32_t depth = 0;
    };
    struct Job { uint64_t lo, hi; uint32_t level; int parent_axis; Out out; };
    std::vector<Job> jobs;
    uint32_t par_level = 0;     // 0: build everything in the calling thread
    uint64_t par_min = 0;       // a subtree smaller than this is never split off

    void presort() {
        const uint64_t n = boxes.size();
        std::vector<std::thread> th;
        for (int a = 0; a < 3; ++a) {
            th.emplace_back([this, a, n] {  // midpoint_comparator (bvh.rs:137-140), ties by index
                S[a].resize(n);
                for (uint64_t i = 0; i < n; ++i) S[a][i] = i;
                const std::vector<int64_t>& k = key[a];
                std::sort(S[a].begin(), S[a].end(),
                          [&k](uint64_t x, uint64_t y) { return k[x] != k[y] ? k[x] < k[y] : x < y; });
                SB[a].resize(n);
                for (uint64_t i = 0; i < n; ++i) SB[a][i] = boxes[S[a][i]];
            });
        }
        for (auto& t : th) t.join();
        left_flag.assign(n, 0);
        tmp_i.resize(n);
        tmp_b.resize(n);
        bwd_score.resize(n);
    }
    // leaf: order[lo..hi) from axis list `a` (-1: list order = ascending index)
    uint64_t leaf(Out& o, uint64_t lo, uint64_t hi, int a, const Box3& box) {
        HostNode node;
        node.box = box;
        node.start = lo; node.end = hi;
        if (a >= 0) {
            for (uint64_t i = lo; i < hi; ++i) order[i] = S[a][i];
        } else {
            for (uint64_t i = lo; i < hi; ++i) order[i] = S[0][i];
            std::sort(order.begin() + lo, order.begin() + hi);
        }
        o.nodes.push_back(node);
        return o.nodes.size() - 1;
    }
    // split_ok: in the calling thread's top tree (jobs build their subtree whole)
    uint64_t build(Out& o, uint64_t lo, uint64_t hi, uint32_t level, int parent_axis, bool split_ok) {
        const uint64_t n = hi - lo;
        if (split_ok && par_level && level == par_level && n >= par_min) {  // split off: built later, concurrently
            jobs.push_back(Job{lo, hi, level, parent_axis, {}});
            o.nodes.push_back(HostNode{box_empty(), -2 - (int64_t)(jobs.size() - 1), -1, 0, 0});
            return o.nodes.size() - 1;
        }
        o.depth = std::max(o.depth, level);
        Box3 box = box_empty();  // in the reference's element order (matters only for NaN coordinates)
        if (parent_axis >= 0) for (uint64_t i = lo; i < hi; ++i) box_extend(box, SB[parent_axis][i]);
        else for (uint64_t i = lo; i < hi; ++i) box_extend(box, boxes[i]);  // root: list order
        if (n <= 4) return leaf(o, lo, hi, parent_axis, box);
        uint64_t best_first = n;
        double best = score(box) * (double)n;
        int best_axis = -1;
        double* bs = bwd_score.data() + lo;
        for (int axis = 0; axis < 3; ++axis) {  // subdivision_score (bvh.rs:120-135)
            // AABBSplitsBuilder::make_splits (bvh.rs:238-255): the suffix boxes are only
            // ever scored, so keep their scores and fold the prefix sweep into the
            // comparison — the same score() of the same boxes, in the same order.
            const Box3* sb = SB[axis].data() + lo;
            Box3 acc = box_empty();
            for (uint64_t k = 0; k + 1 < n; ++k) { box_extend(acc, sb[n - 1 - k]); bs[k] = score(acc); }
            acc = box_empty();
            for (uint64_t i = 0; i + 1 < n; ++i) {
                box_extend(acc, sb[i]);
                uint64_t lc = i + 1, rc = n - lc;
                double sc = score(acc) * (double)lc + bs[(n - 1) - i - 1] * (double)rc;
                if (sc < best) { best_first = lc; best = sc; best_axis = axis; }
            }
        }
        if (best_axis < 0) return leaf(o, lo, hi, 2, box);  // SameNode (bvh.rs:93-96): last sort was axis 2
        // split: the first best_first of the best axis go left; stable-partition the others
        const uint64_t mid = lo + best_first;
        for (uint64_t i = lo; i < mid; ++i) left_flag[S[best_axis][i]] = 1;
        for (int a = 0; a < 3; ++a) {
            if (a == best_axis) continue;
            uint64_t* s = S[a].data();
            Box3* sb = SB[a].data();
            uint64_t l = lo, r = lo;
            for (uint64_t i = lo; i < hi; ++i) {
                const uint64_t p = s[i];
                if (left_flag[p]) { s[l] = p; sb[l] = sb[i]; ++l; }
                else { tmp_i[r] = p; tmp_b[r] = sb[i]; ++r; }
            }
            std::copy(tmp_i.begin() + lo, tmp_i.begin() + r, s + l);
            std::copy(tmp_b.begin() + lo, tmp_b.begin() + r, sb + l);
        }
        for (uint64_t i = lo; i < mid; ++i) left_flag[S[best_axis][i]] = 0;
        uint64_t me = o.nodes.size();
        o.nodes.push_back(HostNode{box, -1, -1, 0, 0});  // placeholder (bvh.rs:104-105)
        uint64_t l = build(o, lo, mid, level + 1, best_axis, split_ok);
        uint64_t r = build(o, mid, hi, level + 1, best_axis, split_ok);
        o.nodes[me].left = (int64_t)l;
        o.nodes[me].right = (int64_t)r;
        return me;
    }
    // top tree + finished jobs -> one array in the reference's pre-order
    int64_t emit(const Out& top, uint64_t i, std::vector<HostNode>& dst, uint32_t& depth) {
        const HostNode& n = top.nodes[i];
        if (n.left <= -2) {  // a job's subtree: copy, shifting its links
            const Out& jo = jobs[(size_t)(-2 - n.left)].out;
            const int64_t off = (int64_t)dst.size();
            for (HostNode c : jo.nodes) {
                if (c.left >= 0) { c.left += off; c.right += off; }
                dst.push_back(c);
            }
            depth = std::max(depth, jo.depth);
            return off;
        }
        const int64_t me = (int64_t)dst.size();
        dst.push_back(n);
        if (n.left >= 0) {
            const int64_t l = emit(top, (uint64_t)n.left, dst, depth);
            const int64_t r = emit(top, (uint64_t)n.right, dst, depth);
            dst[me].left = l;
            dst[me].right = r;
        }
        return me;
    }
};

void flatten(const HostBvh& h, HostBvhArrays& out) {
    out.nodes.resize(h.nodes.size());
    for (size_t i = 0; i < h.nodes.size(); ++i) {
        const HostNode& n = h.nodes[i];
        DevNode d;
        std::memset(&d, 0, sizeof(d));
        d.left = (int32_t)n.left;
        d.right = (int32_t)n.right;
        if (n.left >= 0) {
            const HostNode& l = h.nodes[n.left];
            const HostNode& r = h.nodes[n.right];
            store3(d.lmin, l.box.min); store3(d.lmax, l.box.max);
            store3(d.rmin, r.box.min); store3(d.rmax, r.box.max);
            d.lstart = (uint32_t)l.start; d.lcount = (uint32_t)(l.end - l.start);
            d.rstart = (uint32_t)r.start; d.rcount = (uint32_t)(r.end - r.start);
        }
        d.start = (uint32_t)n.start;
        d.count = (uint32_t)(n.end - n.start);
        out.nodes[i] = d;
    }
    out.root = h.nodes.empty() ? box_empty() : h.nodes[0].box;
    out.depth = h.depth;
    bool fast = !h.nodes.empty();
    for (const HostNode& n : h.nodes) {
        const double c[6] = {n.box.min.x, n.box.min.y, n.box.min.z, n.box.max.x, n.box.max.y, n.box.max.z};
        for (double v : c) fast = fast && coord_fast(v);
        // aabb_hit_fast's per-axis min/max folding needs min <= max
        fast = fast && n.box.min.x <= n.box.max.x && n.box.min.y <= n.box.max.y && n.box.min.z <= n.box.max.z;
    }
    out.fast = fast;
}

// rt_device.h dir_ok on the host: |v| in [2^-360, 2^360]
static bool dir_ok_host(double v) {
    uint64_t b;
    std::memcpy(&b, &v, sizeof b);
    return ((uint32_t)(b >> 52) & 0x7ffu) - 663u < 721u;
}
// DevShape::flags (rt_layout.h): which shapes a ray_fast ray may test with the
// unguarded exact division, and planes whose normal is a signed axis
static uint32_t shape_flags(const rt_shape& s, uint32_t& axis) {
    axis = 0;
    const double* q = s.rotation;  // (s, x, y, z)
    bool fast = q[0] == 1.0 && q[1] == 0.0 && q[2] == 0.0 && q[3] == 0.0;
    for (int k = 0; k < 3; ++k) fast = fast && coord_fast(s.position[k]);
    uint32_t f = 0;
    if (s.type == RT_SHAPE_BOX) {
        bool sizes = true;
        for (int k = 0; k < 3; ++k) sizes = sizes && coord_fast(s.shape[k]) && s.shape[k] != 0.0;
        fast = fast && sizes;
        if (sizes) f |= kBoxSizes;
    }
    if (s.type == RT_SHAPE_ELLIPSOID)  // radii in dev_quot's divisor range (rt_device.h dir_ok)
        for (int k = 0; k < 3; ++k) fast = fast && dir_ok_host(s.shape[k]);
    if (s.type == RT_SHAPE_PLANE) {
        int zeros = 0, k1 = -1;
        for (int k = 0; k < 3; ++k) {
            if (s.shape[k] == 0.0) zeros++;
            else if (s.shape[k] == 1.0 || s.shape[k] == -1.0) k1 = k;
        }
        if (zeros == 2 && k1 >= 0) {
            f |= kPlaneAxis;
            axis = (uint32_t)k1 | (s.shape[k1] < 0.0 ? 4u : 0u);
        }
    }
    return f | (fast ? kShapeFast : 0u);
}

struct ShapeItem { DevShape s; uint32_t mat; int32_t gid; Box3 box; };
struct TriItem { Triangle t; V3 b, c; uint32_t mat; int32_t gid; Box3 box; };  // b, c: the vertices t was built from

void build_shape_bvh(const std::vector<ShapeItem>& items, HostBvhArrays& out) {
    std::vector<Box3> boxes(items.size());
    for (size_t i = 0; i < items.size(); ++i) boxes[i] = items[i].box;
    HostBvh h = build_bvh(boxes);
    flatten(h, out);
    out.n_prims = (uint32_t)items.size();
    for (uint64_t i : h.order) {
        out.shapes.push_back(items[i].s);
        out.mat.push_back(items[i].mat);
        out.gid.push_back(items[i].gid);
    }
}
bool f32_exact(double v) { return (double)(float)v == v || v != v; }
bool f32_exact3(V3 v) { return f32_exact(v.x) && f32_exact(v.y) && f32_exact(v.z) && v.x == v.x && v.y == v.y && v.z == v.z; }

// Pair layout of the compact triangle BVH (rt_layout.h kPairFloats, DESIGN.md §4 "two
// levels per line"): record c (one 128-B line per internal slot c) holds, for each child
// K of c, K's children's boxes and words when K is internal — the boxes a visit of K
// tests — or K's own box when it is a leaf.  A visit of c then takes K's box as the union
// of K's children's boxes (exact: a node's box is the union of its primitives' boxes,
// bvh.rs:56-62, so the f32 min/max of the two children's boxes is the same box) and can
// go on to visit the near child K from the same line (a leaf K's box is stored as both
// boxes, so the union is its box too).  Built only when that union
// reproduces every internal child's box; otherwise left empty (the compact form stays).
void build_pairs(HostBvhArrays& out, size_t n_int) {
    const std::vector<DevNodeC>& cn = out.cnodes;
    std::vector<float> pr(n_int * kPairFloats, 0.0f);
    for (size_t c = 0; c < n_int; ++c) {
        for (int side = 0; side < 2; ++side) {
            float* h = &pr[c * kPairFloats + side * kPairHalf];
            const uint32_t w = side ? cn[c].rw : cn[c].lw;
            const float* mn = side ? cn[c].rmin : cn[c].lmin;
            const float* mx = side ? cn[c].rmax : cn[c].lmax;
            uint32_t words[4] = {0u, 0u, w, 0u};
            if (w & (kPackedLeaf | kLeafRef)) {  // a leaf child: its own box, as A and as B
                // (so the device's union of A and B is the box without a select)
                for (int k = 0; k < 2; ++k) {
                    std::memcpy(h + 6 * k, mn, 3 * sizeof(float));
                    std::memcpy(h + 6 * k + 3, mx, 3 * sizeof(float));
                }
                words[3] = kPairLeaf;
            } else {  // an internal child K = slot w: the boxes its visit tests, its words
                const DevNodeC& k = cn[w];
                std::memcpy(h, k.lmin, 3 * sizeof(float)); std::memcpy(h + 3, k.lmax, 3 * sizeof(float));
                std::memcpy(h + 6, k.rmin, 3 * sizeof(float)); std::memcpy(h + 9, k.rmax, 3 * sizeof(float));
                for (int a = 0; a < 3; ++a)
                    if (std::fmin(k.lmin[a], k.rmin[a]) != mn[a] || std::fmax(k.lmax[a], k.rmax[a]) != mx[a])
                        return;  // not the union: no pair layout for this BVH
                words[0] = k.lw;
                words[1] = k.rw;
            }
            std::memcpy(h + 12, words, sizeof(words));
        }
    }
    out.pnodes = std::move(pr);
}

// The compact layout (rt_layout.h DevNodeC + kTriC floats): built only when it
// holds the same numbers — every child-box coordinate and every vertex a, b, c
// is an exact f32 (glTF positions are f32: C3-C5; a custom TRIANGLE rotated by a
// quaternion usually is not).  The device widens them back to f64 and rebuilds
// ba = b - a, ca = c - a: the bits triangle_props computed from the same a, b, c.
void build_compact(const HostBvh& h, const std::vector<TriItem>& items, HostBvhArrays& out) {
    for (const HostNode& n : h.nodes)
        if (!f32_exact3(n.box.min) || !f32_exact3(n.box.max)) return;
    for (const TriItem& it : items)
        if (!f32_exact3(it.t.a) || !f32_exact3(it.b) || !f32_exact3(it.c)) return;
    // Triangle records in LEAF BLOCKS (round 4): each leaf's records, a, b, c as f32
    // (kTriC floats), contiguous behind a one-word header holding the leaf's first
    // primitive index, the block starting on a 128-B line (kLeafBlock floats).  A leaf of
    // up to three triangles is one line (112 B), four are two; unaligned 36-B records
    // spread a leaf over 1.3-2.1 lines (profiles/r03/fetch_calib.log: a random 36-B
    // record costs 4.4x its bytes in 128-B lines).  The leaf's child word carries the
    // block index instead of the first primitive.
    std::vector<uint64_t> block(h.nodes.size(), 0);
    uint64_t n_floats = 0;
    for (size_t i = 0; i < h.nodes.size(); ++i) {
        const HostNode& n = h.nodes[i];
        if (n.left >= 0) continue;
        block[i] = n_floats / kLeafBlock;
        const uint64_t len = 1 + (uint64_t)kTriC * (n.end - n.start);
        n_floats += (len + kLeafBlock - 1) / kLeafBlock * kLeafBlock;
    }
    // Record slots (round 4): the INTERNAL nodes only, in pre-order (the reference's
    // numbering, bvh.rs:104, with the leaves left out), then the leaves a child word
    // cannot pack (kLeafRef: >= 128 primitives or a block index past 2^24).  A packed
    // leaf is entered from its parent's word and never read as a node, so its 64-B
    // entry was dead weight between the internal nodes: without it the array halves
    // (C5: the internal nodes of a 10M-triangle tree come near the 256-MiB Infinity
    // Cache) and an internal node's internal left child is the next slot, the other
    // half of its 128-B line as often as the node sits at an even slot.  Only the
    // addresses change: every lane's visits and tests are the same.
    auto packs = [&](size_t idx) {
        const HostNode& n = h.nodes[idx];
        return n.end - n.start < 128u && block[idx] < (1u << 24);
    };
    const uint32_t kNone = ~0u;
    std::vector<uint32_t> slot(h.nodes.size(), kNone);
    size_t n_slots = 0;
    for (size_t i = 0; i < h.nodes.size(); ++i)  // h.nodes is in pre-order
        if (h.nodes[i].left >= 0) slot[i] = (uint32_t)n_slots++;
    if (n_slots == 0 || slot[0] != 0) return;  // a leaf root: nothing to traverse
    const size_t n_int = n_slots;
    for (size_t i = 0; i < h.nodes.size(); ++i)
        if (h.nodes[i].left < 0 && !packs(i)) slot[i] = (uint32_t)n_slots++;
    if (n_slots >= kLeafRef || n_floats / kLeafBlock >= (1ull << 32)) return;
    std::vector<DevNodeC> cn(n_slots);
    std::memset(cn.data(), 0, n_slots * sizeof(DevNodeC));
    auto put3 = [](float* d, V3 v) { d[0] = (float)v.x; d[1] = (float)v.y; d[2] = (float)v.z; };
    auto word = [&](int64_t idx) {
        const HostNode& c = h.nodes[idx];
        const uint32_t cnt = (uint32_t)(c.end - c.start);
        if (c.left >= 0) return slot[idx];                                        // internal
        if (packs(idx)) return kPackedLeaf | (cnt << 24) | (uint32_t)block[idx];  // packed leaf block
        return slot[idx] | kLeafRef;                                              // big leaf entry
    };
    for (size_t i = 0; i < h.nodes.size(); ++i) {
        if (slot[i] == kNone) continue;
        const HostNode& n = h.nodes[i];
        DevNodeC c;
        std::memset(&c, 0, sizeof(c));
        if (n.left >= 0) {
            const HostNode& l = h.nodes[n.left];
            const HostNode& r = h.nodes[n.right];
            put3(c.lmin, l.box.min); put3(c.lmax, l.box.max);
            put3(c.rmin, r.box.min); put3(c.rmax, r.box.max);
            c.lw = word(n.left);
            c.rw = word(n.right);
        } else {
            c.start = (uint32_t)block[i];  // a big leaf: its block
        }
        c.count = (uint32_t)(n.end - n.start);
        cn[slot[i]] = c;
    }
    std::vector<float> ct(n_floats, 0.0f);
    for (size_t i = 0; i < h.nodes.size(); ++i) {
        const HostNode& n = h.nodes[i];
        if (n.left >= 0) continue;
        float* b = &ct[block[i] * kLeafBlock];
        const uint32_t first = (uint32_t)n.start;
        std::memcpy(b, &first, sizeof(first));
        for (uint64_t k = n.start; k < n.end; ++k) {
            const TriItem& it = items[h.order[k]];
            float* r = b + 1 + (k - n.start) * kTriC;
            put3(r, it.t.a); put3(r + 3, it.b); put3(r + 6, it.c);
        }
    }
    out.cnodes = std::move(cn);
    out.ctris = std::move(ct);
    build_pairs(out, n_int);
}

void build_tri_bvh(const std::vector<TriItem>& items, HostBvhArrays& out, bool compact = false) {
    std::vector<Box3> boxes(items.size());
    for (size_t i = 0; i < items.size(); ++i) boxes[i] = items[i].box;
    HostBvh h = build_bvh(boxes);
    flatten(h, out);
    if (compact && !h.nodes.empty()) build_compact(h, items, out);
    out.n_prims = (uint32_t)items.size();
    out.tris.reserve(items.size());
    // DevBvh::tri_q: the edges' range of the split-division triangle solve
    auto edge_ok = [](double v) { const double a = std::fabs(v); return a == 0.0 || (a >= 0x1p-149 && a < 0x1p129); };
    out.tri_q = true;
    for (const TriItem& it : items)
        for (double v : {it.t.ba.x, it.t.ba.y, it.t.ba.z, it.t.ca.x, it.t.ca.y, it.t.ca.z})
            out.tri_q = out.tri_q && edge_ok(v);
    for (uint64_t i : h.order) {
        const Triangle& t = items[i].t;
        DevTri d;
        store3(d.a, t.a); store3(d.ba, t.ba); store3(d.ca, t.ca); d.pad = 0.0;
        DevTriCold c;
        store3(c.ng, t.ng); store3(c.na, t.na); store3(c.nb, t.nb); store3(c.nc, t.nc);
        out.tris.push_back(d);
        out.tri_cold.push_back(c);
        out.tri_inv_area.push_back(t.inv_area);
        out.mat.push_back(items[i].mat);
        out.gid.push_back(items[i].gid);
    }
}

bool is_light(const rt_material& m) {  // scene.rs:225-227
    return m.emission[0] != 0.0 || m.emission[1] != 0.0 || m.emission[2] != 0.0;
}

}  // namespace

HostBvh build_bvh(const std::vector<Box3>& boxes) {
    HostBvh h;
    uint64_t n = boxes.size();
    h.order.resize(n);
    for (uint64_t i = 0; i < n; ++i) h.order[i] = i;
    if (n == 0) return h;  // BVH over nothing is never traversed (bvh.rs:29,39)
    Builder b{boxes, {}, {}, {}, h.order, {}, {}, {}, {}, {}, 0, 0};
    for (int axis = 0; axis < 3; ++axis) {
        b.key[axis].resize(n);
        for (uint64_t i = 0; i < n; ++i)
            b.key[axis][i] = total_key((comp(boxes[i].min, axis) + comp(boxes[i].max, axis)) / 2.0);
    }
    b.presort();
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    if (n >= kParallelBuildMin && hw > 1) {  // subtrees below level 6 built concurrently
        b.par_level = 6;
        b.par_min = 4096;
    }
    Builder::Out top;
    top.nodes.reserve(b.par_level ? 256 : 2 * (n / 2 + 1));
    b.build(top, 0, n, 1, -1, true);
    if (b.jobs.empty()) {
        h.nodes = std::move(top.nodes);
        h.depth = top.depth;
        return h;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    const unsigned nt = (unsigned)std::min<size_t>(std::min(hw, 16u), b.jobs.size());
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&b, &next] {
            for (size_t k; (k = next.fetch_add(1)) < b.jobs.size();) {
                Builder::Job& jb = b.jobs[k];
                b.build(jb.out, jb.lo, jb.hi, jb.level, jb.parent_axis, false);
            }
        });
    for (auto& t : th) t.join();
    h.nodes.reserve(2 * (n / 2 + 1));
    h.depth = top.depth;
    b.emit(top, 0, h.nodes, h.depth);
    return h;
}

std::string build_scene(const rt_scene_desc& d, HostScene& out) {
    auto t0 = std::chrono::steady_clock::now();
    if (d.n_materials == 0 && (d.n_shapes > 0 || d.n_triangles > 0)) return "scene has primitives but no materials";
    if (d.n_shapes > 0 && !d.shapes) return "shapes is NULL";
    if (d.n_triangles > 0 && (!d.tri_vertices || !d.tri_material)) return "triangle arrays are NULL";
    if (d.n_triangles > 0 && d.tri_mode == RT_TRI_GLTF && !d.tri_normals) return "glTF triangles need normals";
    if ((uint64_t)d.n_shapes + d.n_triangles > 0x7fffffffull) return "too many primitives for int32 ids";
    out.mats.resize(d.n_materials);
    for (uint32_t i = 0; i < d.n_materials; ++i) {
        const rt_material& m = d.materials[i];
        if (m.kind > RT_MAT_DIELECTRIC) return "bad material kind";
        DevMaterial dm;
        dm.kind = m.kind; dm.pad = 0; dm.ior = m.ior;
        const double q = (1.0 - m.ior) / (1.0 + m.ior);
        dm.k_out = 1.0 / m.ior;
        dm.r0 = q * q;
        for (int k = 0; k < 3; ++k) { dm.color[k] = m.color[k]; dm.emission[k] = m.emission[k]; }
        out.mats[i] = dm;
    }
    std::vector<ShapeItem> boxes, ells;
    for (uint32_t i = 0; i < d.n_shapes; ++i) {
        const rt_shape& s = d.shapes[i];
        if (s.material >= d.n_materials) return "shape material out of range";
        ShapeItem it;
        std::memset(&it.s, 0, sizeof(it.s));
        std::memcpy(it.s.shape, s.shape, sizeof(it.s.shape));
        std::memcpy(it.s.pos, s.position, sizeof(it.s.pos));
        std::memcpy(it.s.rot, s.rotation, sizeof(it.s.rot));
        if (s.type == RT_SHAPE_ELLIPSOID)
            // placeholder: the device overwrites it with dev_rcp(r) (api.cpp launch_ell_rcp)
            for (int k = 0; k < 3; ++k) it.s.aux[k] = 1.0 / s.shape[k];
        if (s.type == RT_SHAPE_BOX) {
            const double* z = s.shape;
            it.s.aux[0] = 1.0 / ((z[1] * z[2] + z[0] * z[2]) + z[0] * z[1]) / 8.0;
        }
        it.s.flags = shape_flags(s, it.s.axis);
        it.mat = s.material;
        it.gid = (int32_t)i;
        if (s.type == RT_SHAPE_PLANE) {  // Primitive::new_without_aabb (scene.rs:126-136)
            out.planes.push_back(it.s);
            out.plane_mat.push_back(it.mat);
            out.plane_gid.push_back(it.gid);
            continue;
        }
        if (s.type != RT_SHAPE_BOX && s.type != RT_SHAPE_ELLIPSOID) return "bad shape type";
        V3 sz = load3(s.shape);
        Box3 local = box_empty();  // Box::new / Ellipsoid::new (box.rs:12-17, ellipsoid.rs:12-17)
        box_extend(local, sz);
        box_extend(local, -sz);
        Box3 w = rotated_box(local, load_quat(s.rotation));  // Primitive::new (scene.rs:109-122)
        V3 p = load3(s.position);
        w.min = w.min + p;
        w.max = w.max + p;
        it.box = w;
        (s.type == RT_SHAPE_BOX ? boxes : ells).push_back(it);
    }
    std::vector<TriItem> tris(d.n_triangles);
    for (uint64_t j = 0; j < d.n_triangles; ++j) {
        const double* v = d.tri_vertices + 9 * j;
        TriItem& it = tris[j];
        it.mat = d.tri_material[j];
        if (it.mat >= d.n_materials) return "triangle material out of range";
        it.gid = (int32_t)(d.n_shapes + j);
        if (d.tri_mode == RT_TRI_GLTF) {  // new_with_smooth_normal + instantiate (gltf/scene_builder.rs:42-55)
            const double* nn = d.tri_normals + 9 * j;
            it.t = triangle_smooth(load3(v), load3(v + 3), load3(v + 6), load3(nn), load3(nn + 3), load3(nn + 6));
            it.b = load3(v + 3);
            it.c = load3(v + 6);
            Box3 b = box_empty();
            box_extend(b, it.t.a);
            box_extend(b, it.t.a + it.t.ba);
            box_extend(b, it.t.a + it.t.ca);
            it.box = b;
        } else {  // new_with_geometry_normals (scene_parser.rs:71-73) + TrianglePrimitive::new (scene.rs:139-165)
            Triangle m = triangle_geometric(load3(v), load3(v + 3), load3(v + 6));
            V3 pos = d.tri_position ? load3(d.tri_position + 3 * j) : v3(0, 0, 0);
            Quat rot = d.tri_rotation ? load_quat(d.tri_rotation + 4 * j) : Quat{1.0, v3(0, 0, 0)};
            V3 a = rotate(rot, m.a) + pos;
            V3 b = rotate(rot, m.ba + m.a) + pos;
            V3 c = rotate(rot, m.ca + m.a) + pos;
            it.t = triangle_smooth(a, b, c, rotate(rot, m.na), rotate(rot, m.nb), rotate(rot, m.nc));
            it.b = b;
            it.c = c;
            Box3 bb = box_empty();
            box_extend(bb, a); box_extend(bb, b); box_extend(bb, c);
            it.box = bb;
        }
    }
    // lights are copies of the emissive primitives (scene.rs:209-213, :229-241)
    std::vector<ShapeItem> lboxes, lells;
    std::vector<TriItem> ltris;
    for (auto& it : boxes) if (is_light(d.materials[it.mat])) lboxes.push_back(it);
    for (auto& it : ells) if (is_light(d.materials[it.mat])) lells.push_back(it);
    for (auto& it : tris) if (is_light(d.materials[it.mat])) ltris.push_back(it);
    build_shape_bvh(boxes, out.bvh[0]);
    build_shape_bvh(ells, out.bvh[1]);
    build_tri_bvh(tris, out.bvh[2], true);  // the scene's triangle BVH: compact layout when exact
    build_shape_bvh(lboxes, out.bvh[3]);
    build_shape_bvh(lells, out.bvh[4]);
    build_tri_bvh(ltris, out.bvh[5]);
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return "";
}

}  // namespace rt
