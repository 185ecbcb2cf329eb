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
#include <chrono>
#include <cstring>

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

struct Builder {
    const std::vector<Box3>& boxes;
    std::vector<int64_t> key[3];       // midpoint sort key per axis and primitive
    std::vector<uint64_t>& idx;
    std::vector<HostNode>& nodes;
    std::vector<Box3> fwd, bwd;
    uint32_t depth = 0;

    void sort_axis(uint64_t lo, uint64_t hi, int axis) {  // midpoint_comparator (bvh.rs:137-140)
        const std::vector<int64_t>& k = key[axis];
        std::sort(idx.begin() + lo, idx.begin() + hi, [&k](uint64_t a, uint64_t b) {
            return k[a] != k[b] ? k[a] < k[b] : a < b;
        });
    }
    uint64_t build(uint64_t lo, uint64_t hi, uint32_t level) {  // build_nodes (bvh.rs:75-113)
        depth = std::max(depth, level);
        uint64_t n = hi - lo;
        Box3 box = box_empty();
        for (uint64_t i = lo; i < hi; ++i) box_extend(box, boxes[idx[i]]);
        HostNode node;
        node.box = box;
        if (n <= 4) {
            node.start = lo; node.end = hi;
            nodes.push_back(node);
            return nodes.size() - 1;
        }
        uint64_t best_first = n;
        double best = score(box) * (double)n;
        int best_axis = -1;
        for (int axis = 0; axis < 3; ++axis) {  // subdivision_score (bvh.rs:120-135)
            sort_axis(lo, hi, axis);
            Box3 acc = box_empty();  // AABBSplitsBuilder::make_splits (bvh.rs:238-255)
            for (uint64_t i = 0; i + 1 < n; ++i) { box_extend(acc, boxes[idx[lo + i]]); fwd[i] = acc; }
            acc = box_empty();
            for (uint64_t k = 0; k + 1 < n; ++k) { box_extend(acc, boxes[idx[hi - 1 - k]]); bwd[k] = acc; }
            for (uint64_t i = 0; i + 1 < n; ++i) {
                uint64_t lc = i + 1, rc = n - lc;
                double s = score(fwd[i]) * (double)lc + score(bwd[(n - 1) - i - 1]) * (double)rc;
                if (s < best) { best_first = lc; best = s; best_axis = axis; }
            }
        }
        if (best_axis < 0) {  // SubdivisionType::SameNode (bvh.rs:93-96)
            node.start = lo; node.end = hi;
            nodes.push_back(node);
            return nodes.size() - 1;
        }
        sort_axis(lo, hi, best_axis);  // bvh.rs:102
        uint64_t me = nodes.size();
        nodes.push_back(node);  // placeholder (bvh.rs:104-105)
        uint64_t l = build(lo, lo + best_first, level + 1);
        uint64_t r = build(lo + best_first, hi, level + 1);
        nodes[me].left = (int64_t)l;
        nodes[me].right = (int64_t)r;
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
    }
    out.fast = fast;
}

struct ShapeItem { DevShape s; uint32_t mat; int32_t gid; Box3 box; };
struct TriItem { Triangle t; uint32_t mat; int32_t gid; Box3 box; };

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
void build_tri_bvh(const std::vector<TriItem>& items, HostBvhArrays& out) {
    std::vector<Box3> boxes(items.size());
    for (size_t i = 0; i < items.size(); ++i) boxes[i] = items[i].box;
    HostBvh h = build_bvh(boxes);
    flatten(h, out);
    out.n_prims = (uint32_t)items.size();
    out.tris.reserve(items.size());
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
    Builder b{boxes, {}, h.order, h.nodes, {}, {}, 0};
    for (int axis = 0; axis < 3; ++axis) {
        b.key[axis].resize(n);
        for (uint64_t i = 0; i < n; ++i)
            b.key[axis][i] = total_key((comp(boxes[i].min, axis) + comp(boxes[i].max, axis)) / 2.0);
    }
    b.fwd.resize(n > 1 ? n - 1 : 1);
    b.bwd.resize(n > 1 ? n - 1 : 1);
    h.nodes.reserve(2 * (n / 2 + 1));
    b.build(0, n, 1);
    h.depth = b.depth;
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
            for (int k = 0; k < 3; ++k) it.s.aux[k] = 1.0 / s.shape[k];
        if (s.type == RT_SHAPE_BOX) {
            const double* z = s.shape;
            it.s.aux[0] = 1.0 / ((z[1] * z[2] + z[0] * z[2]) + z[0] * z[1]) / 8.0;
        }
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
    build_tri_bvh(tris, out.bvh[2]);
    build_shape_bvh(lboxes, out.bvh[3]);
    build_shape_bvh(lells, out.bvh[4]);
    build_tri_bvh(ltris, out.bvh[5]);
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return "";
}

}  // namespace rt
