// gltf.cpp — glTF subset input surface.
//
// Restates gltf/parser.rs (serde model: which fields are required, their
// defaults) and gltf/scene_builder.rs:9-398 (node TRS propagation, vertex /
// normal / index readers, cofactor normal matrix, material mapping, camera):
//   * ray_depth is hard-coded to 8 and bg to 0 (scene_builder.rs:16-17);
//   * only mode 4 (TRIANGLES) primitives, NORMAL required (:210-212);
//   * metallicFactor defaults to 1.0 => Metallic unless it is 0 (parser.rs:63-64,207);
//     alpha < 1 => Dielectric(1.5) (:231);
//   * exactly one perspective camera on exactly one node; its TRS columns
//     (not normalised) give right/up/-forward (:57-78);
//   * external .bin buffers resolved relative to the .gltf (main.rs:54-59, 77-83).
// Matrix arithmetic follows cgmath 0.18 (Matrix4 * Matrix4 / Vector4 as
// column combinations, quaternion -> matrix) so vertices match the
// reference bit for bit.  Every reference panic becomes an error code.
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "api_internal.h"
#include "json.h"
#include "rt_math.h"

using namespace rt;

namespace {

struct Err {
    int code = RT_OK;
    std::string msg;
    bool set(int c, const std::string& m) {
        if (code == RT_OK) { code = c; msg = m; }
        return false;
    }
};

// ---- serde-like field access ---------------------------------------------
bool get_uint(const Json& o, const char* k, bool required, uint64_t def, uint64_t& out, Err& e) {
    const Json* v = o.get(k);
    if (!v || (v->kind == Json::Null && !required)) {
        if (required) return e.set(RT_ERR_PARSE, std::string("missing field `") + k + "`");
        out = def;
        return true;
    }
    if (v->kind != Json::Number || !v->is_int || v->negative)
        return e.set(RT_ERR_PARSE, std::string("field `") + k + "`: expected usize");
    out = v->uint_val;
    return true;
}
bool get_opt_uint(const Json& o, const char* k, bool& has, uint64_t& out, Err& e) {
    const Json* v = o.get(k);
    has = v && v->kind != Json::Null;
    if (!has) return true;
    return get_uint(o, k, true, 0, out, e);
}
bool get_f64(const Json& v, double& out, Err& e, const char* what) {
    if (v.kind != Json::Number) return e.set(RT_ERR_PARSE, std::string(what) + ": expected number");
    out = v.num;
    return true;
}
bool get_opt_f64_vec(const Json& o, const char* k, bool& has, std::vector<double>& out, Err& e) {
    const Json* v = o.get(k);
    has = v && v->kind != Json::Null;
    if (!has) return true;
    if (v->kind != Json::Array) return e.set(RT_ERR_PARSE, std::string("field `") + k + "`: expected array");
    out.clear();
    for (const Json& x : v->arr) {
        double d;
        if (!get_f64(x, d, e, k)) return false;
        out.push_back(d);
    }
    return true;
}
bool get_uint_vec(const Json& o, const char* k, bool required, std::vector<uint64_t>& out, Err& e) {
    const Json* v = o.get(k);
    out.clear();
    if (!v) return required ? e.set(RT_ERR_PARSE, std::string("missing field `") + k + "`") : true;
    if (v->kind != Json::Array) return e.set(RT_ERR_PARSE, std::string("field `") + k + "`: expected array");
    for (const Json& x : v->arr) {
        if (x.kind != Json::Number || !x.is_int || x.negative)
            return e.set(RT_ERR_PARSE, std::string("field `") + k + "`: expected usize");
        out.push_back(x.uint_val);
    }
    return true;
}
const Json* get_array(const Json& root, const char* k, Err& e, bool& ok) {  // #[serde(default)] Vec<T>
    const Json* v = root.get(k);
    ok = true;
    if (!v) return nullptr;
    if (v->kind != Json::Array) { ok = e.set(RT_ERR_PARSE, std::string("field `") + k + "`: expected array"); return nullptr; }
    return v;
}

// ---- cgmath Matrix4 (column-major m[c][r]) ---------------------------------
struct M4 { double m[4][4]; };
M4 identity4() {
    M4 a;
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) a.m[c][r] = c == r ? 1.0 : 0.0;
    return a;
}
M4 mul4(const M4& L, const M4& R) {  // from_cols(a*rhs[c][0] + b*rhs[c][1] + c*rhs[c][2] + d*rhs[c][3])
    M4 o;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o.m[c][r] = ((L.m[0][r] * R.m[c][0] + L.m[1][r] * R.m[c][1]) + L.m[2][r] * R.m[c][2]) + L.m[3][r] * R.m[c][3];
    return o;
}
void mul4v(const M4& M, const double v[4], double out[4]) {  // m[0]*v0 + m[1]*v1 + m[2]*v2 + m[3]*v3
    for (int r = 0; r < 4; ++r)
        out[r] = ((M.m[0][r] * v[0] + M.m[1][r] * v[1]) + M.m[2][r] * v[2]) + M.m[3][r] * v[3];
}
M4 from_quat(double s, double x, double y, double z) {  // impl From<Quaternion> for Matrix4
    const double x2 = x + x, y2 = y + y, z2 = z + z;
    const double xx2 = x2 * x, xy2 = x2 * y, xz2 = x2 * z;
    const double yy2 = y2 * y, yz2 = y2 * z, zz2 = z2 * z;
    const double sy2 = y2 * s, sz2 = z2 * s, sx2 = x2 * s;
    M4 a = identity4();
    a.m[0][0] = 1.0 - yy2 - zz2; a.m[0][1] = xy2 + sz2; a.m[0][2] = xz2 - sy2;
    a.m[1][0] = xy2 - sz2; a.m[1][1] = 1.0 - xx2 - zz2; a.m[1][2] = yz2 + sx2;
    a.m[2][0] = xz2 + sy2; a.m[2][1] = yz2 - sx2; a.m[2][2] = 1.0 - xx2 - yy2;
    return a;
}
// cof() of scene_builder.rs:367-388 on the upper-left 3x3 (mat4_to_mat3, :363-365)
void cof3(const M4& M, double out[3][3]) {
    static const int other[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    for (int col = 0; col < 3; ++col)
        for (int row = 0; row < 3; ++row) {
            int lc = other[col][0], rc = other[col][1], tr = other[row][0], br = other[row][1];
            // Mat2::new(m[lc][tr], m[lc][br], m[rc][tr], m[rc][br]).determinant()
            double det = M.m[lc][tr] * M.m[rc][br] - M.m[rc][tr] * M.m[lc][br];
            out[col][row] = ((col + row) & 1) ? -det : det;
        }
}

struct Node {
    M4 trs;
    std::vector<uint64_t> children;
    bool has_mesh = false, has_camera = false;
    uint64_t mesh = 0;
};

bool extract_trs(const Json& n, M4& out, Err& e) {  // scene_builder.rs:108-123
    bool has;
    std::vector<double> v;
    if (!get_opt_f64_vec(n, "matrix", has, v, e)) return false;
    if (has) {
        if (v.size() != 16) return e.set(RT_ERR_PARSE, "node matrix must have 16 elements");
        for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) out.m[c][r] = v[4 * c + r];
        return true;
    }
    std::vector<double> t, q, s;
    bool ht, hq, hs;
    if (!get_opt_f64_vec(n, "translation", ht, t, e) || !get_opt_f64_vec(n, "rotation", hq, q, e) ||
        !get_opt_f64_vec(n, "scale", hs, s, e))
        return false;
    if ((ht && t.size() != 3) || (hs && s.size() != 3) || (hq && q.size() != 4))
        return e.set(RT_ERR_PARSE, "bad TRS vector length");
    M4 T = identity4();
    if (ht) { T.m[3][0] = t[0]; T.m[3][1] = t[1]; T.m[3][2] = t[2]; }
    M4 R = hq ? from_quat(q[3], q[0], q[1], q[2]) : from_quat(1.0, 0.0, 0.0, 0.0);
    M4 S = identity4();
    if (hs) { S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2]; }
    out = mul4(mul4(T, R), S);
    return true;
}

bool propagate(std::vector<Node>& nodes, uint64_t index, const M4& parent, int depth, Err& e) {  // :163-169
    if (index >= nodes.size()) return e.set(RT_ERR_PARSE, "node index out of range");
    if (depth > 1000) return e.set(RT_ERR_PARSE, "node hierarchy too deep (cycle?)");
    nodes[index].trs = mul4(parent, nodes[index].trs);
    const M4 me = nodes[index].trs;
    for (uint64_t c : nodes[index].children)
        if (!propagate(nodes, c, me, depth + 1, e)) return false;
    return true;
}

struct Accessor {
    bool has_view = false;
    uint64_t view = 0, byte_offset = 0, component_type = 0, count = 0;
    std::string type;
};
struct View { uint64_t buffer = 0, byte_length = 0, byte_offset = 0; bool has_stride = false; uint64_t stride = 0; };

struct Ctx {
    const Json* root;
    std::vector<Accessor> acc;
    std::vector<View> views;
    std::vector<std::string> buffer_uri;
    std::map<std::string, std::string> buffers;  // uri -> bytes
    std::vector<Node> nodes;
    rt_parsed_scene* ps;
    Err e;
};

bool bytes_of(Ctx& c, const Accessor& a, const std::string*& bytes, uint64_t& offset, uint64_t& stride,
              uint64_t elem) {
    if (a.view >= c.views.size()) return c.e.set(RT_ERR_PARSE, "bufferView index out of range");
    const View& v = c.views[a.view];
    if (v.buffer >= c.buffer_uri.size()) return c.e.set(RT_ERR_PARSE, "buffer index out of range");
    bytes = &c.buffers[c.buffer_uri[v.buffer]];
    offset = v.byte_offset + a.byte_offset;
    stride = v.has_stride ? v.stride : elem;
    return true;
}
float f32_at(const std::string& b, uint64_t pos) {
    float f;
    std::memcpy(&f, b.data() + pos, 4);  // little-endian host (x86-64)
    return f;
}

// read_vertices (scene_builder.rs:269-297)
bool read_vertices(Ctx& c, uint64_t ai, const M4& trs, std::vector<V3>& out) {
    if (ai >= c.acc.size()) return c.e.set(RT_ERR_PARSE, "accessor index out of range");
    const Accessor& a = c.acc[ai];
    out.clear();
    if (!a.has_view) return true;
    if (a.component_type != 5126 || a.type != "VEC3") return c.e.set(RT_ERR_UNSUPPORTED, "POSITION must be FLOAT VEC3");
    const std::string* b; uint64_t off, stride;
    if (!bytes_of(c, a, b, off, stride, 12)) return false;
    for (uint64_t k = 0; k < a.count; ++k, off += stride) {
        if (off + 12 > b->size()) return c.e.set(RT_ERR_PARSE, "vertex read past end of buffer");
        double v[4] = {(double)f32_at(*b, off), (double)f32_at(*b, off + 4), (double)f32_at(*b, off + 8), 1.0};
        double p[4];
        mul4v(trs, v, p);
        if (!(p[3] == 1.0)) return c.e.set(RT_ERR_UNSUPPORTED, "non-affine node transform (pos.w != 1)");
        out.push_back(v3(p[0], p[1], p[2]));
    }
    return true;
}
// read_normals (scene_builder.rs:299-327)
bool read_normals(Ctx& c, uint64_t ai, const M4& trs, std::vector<V3>& out) {
    if (ai >= c.acc.size()) return c.e.set(RT_ERR_PARSE, "accessor index out of range");
    const Accessor& a = c.acc[ai];
    out.clear();
    if (!a.has_view) return true;
    if (a.component_type != 5126 || a.type != "VEC3") return c.e.set(RT_ERR_UNSUPPORTED, "NORMAL must be FLOAT VEC3");
    const std::string* b; uint64_t off, stride;
    if (!bytes_of(c, a, b, off, stride, 12)) return false;
    double rs[3][3];
    cof3(trs, rs);
    for (uint64_t k = 0; k < a.count; ++k, off += stride) {
        if (off + 12 > b->size()) return c.e.set(RT_ERR_PARSE, "normal read past end of buffer");
        double x = (double)f32_at(*b, off), y = (double)f32_at(*b, off + 4), z = (double)f32_at(*b, off + 8);
        V3 n = v3((rs[0][0] * x + rs[1][0] * y) + rs[2][0] * z, (rs[0][1] * x + rs[1][1] * y) + rs[2][1] * z,
                  (rs[0][2] * x + rs[1][2] * y) + rs[2][2] * z);
        out.push_back(normalize(n));
    }
    return true;
}
// read_indices (scene_builder.rs:237-267)
bool read_indices(Ctx& c, uint64_t ai, std::vector<uint32_t>& out) {
    if (ai >= c.acc.size()) return c.e.set(RT_ERR_PARSE, "accessor index out of range");
    const Accessor& a = c.acc[ai];
    out.clear();
    if (!a.has_view) return true;
    if (a.component_type != 5123 && a.component_type != 5125)
        return c.e.set(RT_ERR_UNSUPPORTED, "indices must be UNSIGNED_SHORT or UNSIGNED_INT");
    if (a.type != "SCALAR") return c.e.set(RT_ERR_UNSUPPORTED, "indices must have SCALAR type");
    const uint64_t es = a.component_type == 5123 ? 2 : 4;
    const std::string* b; uint64_t off, stride;
    if (!bytes_of(c, a, b, off, stride, es)) return false;
    out.reserve(a.count);
    for (uint64_t k = 0; k < a.count; ++k, off += stride) {
        if (off + es > b->size()) return c.e.set(RT_ERR_PARSE, "index read past end of buffer");
        if (es == 2) { uint16_t v; std::memcpy(&v, b->data() + off, 2); out.push_back(v); }
        else { uint32_t v; std::memcpy(&v, b->data() + off, 4); out.push_back(v); }
    }
    return true;
}

// make_metadata (scene_builder.rs:227-235) with the serde defaults of parser.rs
bool make_material(Ctx& c, const Json* m, rt_material& out) {
    double color[4] = {1.0, 1.0, 1.0, 1.0}, em[3] = {0.0, 0.0, 0.0}, metallic = 1.0, strength = 1.0;
    if (m) {
        if (m->kind != Json::Object) return c.e.set(RT_ERR_PARSE, "material must be an object");
        if (const Json* pbr = m->get("pbrMetallicRoughness")) {
            bool has;
            std::vector<double> v;
            if (!get_opt_f64_vec(*pbr, "baseColorFactor", has, v, c.e)) return false;
            if (has) {
                if (v.size() != 4) return c.e.set(RT_ERR_PARSE, "baseColorFactor must have 4 elements");
                for (int k = 0; k < 4; ++k) color[k] = v[k];
            }
            if (const Json* mf = pbr->get("metallicFactor")) if (!get_f64(*mf, metallic, c.e, "metallicFactor")) return false;
        }
        bool has;
        std::vector<double> v;
        if (!get_opt_f64_vec(*m, "emissiveFactor", has, v, c.e)) return false;
        if (has) {
            if (v.size() != 3) return c.e.set(RT_ERR_PARSE, "emissiveFactor must have 3 elements");
            for (int k = 0; k < 3; ++k) em[k] = v[k];
        }
        if (const Json* ext = m->get("extensions"))
            if (const Json* es = ext->get("KHR_materials_emissive_strength")) {
                const Json* s = es->get("emissiveStrength");
                if (!s) return c.e.set(RT_ERR_PARSE, "missing field `emissiveStrength`");
                if (!get_f64(*s, strength, c.e, "emissiveStrength")) return false;
            }
    }
    std::memset(&out, 0, sizeof(out));
    if (color[3] < 1.0) { out.kind = RT_MAT_DIELECTRIC; out.ior = 1.5; }
    else if (metallic > 0.0) out.kind = RT_MAT_METALLIC;
    else out.kind = RT_MAT_DIFFUSE;
    for (int k = 0; k < 3; ++k) { out.color[k] = color[k]; out.emission[k] = em[k] * strength; }
    return true;
}

// convert_primitive (scene_builder.rs:209-225) + make_triangles[_by_indices] (:329-356)
bool convert_primitive(Ctx& c, const Json& p, const M4& trs) {
    uint64_t mode;
    if (!get_uint(p, "mode", false, 4, mode, c.e)) return false;
    if (mode != 4) return c.e.set(RT_ERR_UNSUPPORTED, "supported only triangles for primitive.mode");
    const Json* attr = p.get("attributes");
    if (!attr) return c.e.set(RT_ERR_PARSE, "missing field `attributes`");
    uint64_t pos_i, nrm_i;
    bool has_n;
    if (!get_uint(*attr, "POSITION", true, 0, pos_i, c.e) || !get_opt_uint(*attr, "NORMAL", has_n, nrm_i, c.e)) return false;
    std::vector<V3> verts, norms;
    if (!read_vertices(c, pos_i, trs, verts)) return false;
    if (!has_n) return c.e.set(RT_ERR_UNSUPPORTED, "empty normals");
    if (!read_normals(c, nrm_i, trs, norms)) return false;
    bool has_idx, has_mat;
    uint64_t idx_i, mat_i;
    if (!get_opt_uint(p, "indices", has_idx, idx_i, c.e) || !get_opt_uint(p, "material", has_mat, mat_i, c.e)) return false;
    if (verts.size() != norms.size()) return c.e.set(RT_ERR_PARSE, "vertex/normal count mismatch");
    std::vector<uint32_t> idx;
    if (has_idx) {
        if (!read_indices(c, idx_i, idx)) return false;
        if (idx.size() % 3) return c.e.set(RT_ERR_PARSE, "index count not a multiple of 3");
    } else if (verts.size() % 3) return c.e.set(RT_ERR_PARSE, "vertex count not a multiple of 3");
    const Json* mats = c.root->get("materials");
    const Json* mj = nullptr;
    if (has_mat) {
        if (!mats || mats->kind != Json::Array || mat_i >= mats->arr.size()) return c.e.set(RT_ERR_PARSE, "material index out of range");
        mj = &mats->arr[mat_i];
    }
    rt_material m;
    if (!make_material(c, mj, m)) return false;
    const uint32_t mid = (uint32_t)c.ps->mats.size();
    c.ps->mats.push_back(m);
    const uint64_t n = has_idx ? idx.size() : verts.size();
    for (uint64_t k = 0; k < n; k += 3) {
        uint64_t ia = has_idx ? idx[k] : k, ib = has_idx ? idx[k + 1] : k + 1, ic = has_idx ? idx[k + 2] : k + 2;
        if (ia >= verts.size() || ib >= verts.size() || ic >= verts.size()) return c.e.set(RT_ERR_PARSE, "index out of range");
        const V3 vv[3] = {verts[ia], verts[ib], verts[ic]}, nn[3] = {norms[ia], norms[ib], norms[ic]};
        for (int q = 0; q < 3; ++q) {
            c.ps->tri_v.insert(c.ps->tri_v.end(), {vv[q].x, vv[q].y, vv[q].z});
            c.ps->tri_n.insert(c.ps->tri_n.end(), {nn[q].x, nn[q].y, nn[q].z});
        }
        c.ps->tri_mat.push_back(mid);
    }
    return true;
}

bool convert_node(Ctx& c, uint64_t ni, int depth) {  // :190-207
    if (ni >= c.nodes.size()) return c.e.set(RT_ERR_PARSE, "node index out of range");
    if (depth > 1000) return c.e.set(RT_ERR_PARSE, "node hierarchy too deep (cycle?)");
    const Node& node = c.nodes[ni];
    if (node.has_mesh) {
        const Json* meshes = c.root->get("meshes");
        if (!meshes || meshes->kind != Json::Array || node.mesh >= meshes->arr.size())
            return c.e.set(RT_ERR_PARSE, "mesh index out of range");
        const Json* prims = meshes->arr[node.mesh].get("primitives");
        if (!prims || prims->kind != Json::Array) return c.e.set(RT_ERR_PARSE, "missing field `primitives`");
        for (const Json& p : prims->arr)
            if (!convert_primitive(c, p, node.trs)) return false;
    }
    const std::vector<uint64_t> ch = node.children;
    for (uint64_t k : ch)
        if (!convert_node(c, k, depth + 1)) return false;
    return true;
}

bool load(Ctx& c, const std::string& path, uint32_t W, uint32_t H, uint32_t spp) {
    const Json& root = *c.root;
    if (root.kind != Json::Object) return c.e.set(RT_ERR_PARSE, "can't parse glTF: not an object");
    bool ok;
    // required-field checks of serde structs the builder does not otherwise read
    if (const Json* imgs = get_array(root, "images", c.e, ok)) {
        for (const Json& im : imgs->arr) {
            const Json* mt = im.get("mimeType");
            if (!mt || mt->kind != Json::String) return c.e.set(RT_ERR_PARSE, "image: missing field `mimeType`");
        }
    } else if (!ok) return false;
    if (const Json* tex = get_array(root, "textures", c.e, ok)) {
        for (const Json& t : tex->arr) { uint64_t s; if (!get_uint(t, "source", true, 0, s, c.e)) return false; }
    } else if (!ok) return false;
    // serde deserialises every material and mesh up front, referenced or not (parser.rs:80-111)
    if (const Json* ms = get_array(root, "materials", c.e, ok)) {
        for (const Json& m : ms->arr) { rt_material tmp; if (!make_material(c, &m, tmp)) return false; }
    } else if (!ok) return false;
    if (const Json* ms = get_array(root, "meshes", c.e, ok)) {
        for (const Json& m : ms->arr) {
            const Json* prims = m.get("primitives");
            if (!prims || prims->kind != Json::Array) return c.e.set(RT_ERR_PARSE, "missing field `primitives`");
            for (const Json& p : prims->arr) {
                const Json* attr = p.get("attributes");
                uint64_t pos;
                if (!attr) return c.e.set(RT_ERR_PARSE, "missing field `attributes`");
                if (!get_uint(*attr, "POSITION", true, 0, pos, c.e)) return false;
                bool has;
                uint64_t v;
                if (!get_opt_uint(*attr, "NORMAL", has, v, c.e) || !get_opt_uint(p, "indices", has, v, c.e) ||
                    !get_opt_uint(p, "material", has, v, c.e) || !get_opt_uint(p, "mode", has, v, c.e))
                    return false;
            }
        }
    } else if (!ok) return false;
    // buffers / views / accessors
    const std::string prefix = path.substr(0, path.rfind('/') == std::string::npos ? 0 : path.rfind('/') + 1);
    if (const Json* bufs = get_array(root, "buffers", c.e, ok)) {
        for (const Json& b : bufs->arr) {
            uint64_t len;
            if (!get_uint(b, "byteLength", true, 0, len, c.e)) return false;
            const Json* uri = b.get("uri");
            if (!uri || uri->kind != Json::String) return c.e.set(RT_ERR_UNSUPPORTED, "expected uri for buffer");
            c.buffer_uri.push_back(uri->str);
            if (!c.buffers.count(uri->str)) {  // load_buffers (:80-87)
                std::ifstream f(prefix + uri->str, std::ios::binary);
                if (!f) return c.e.set(RT_ERR_IO, "Couldn't find or load '" + uri->str + "' file.");
                std::ostringstream ss;
                ss << f.rdbuf();
                c.buffers[uri->str] = ss.str();
            }
        }
    } else if (!ok) return false;
    if (const Json* vs = get_array(root, "bufferViews", c.e, ok)) {
        for (const Json& v : vs->arr) {
            View w;
            if (!get_uint(v, "buffer", true, 0, w.buffer, c.e) || !get_uint(v, "byteLength", true, 0, w.byte_length, c.e) ||
                !get_uint(v, "byteOffset", false, 0, w.byte_offset, c.e) ||
                !get_opt_uint(v, "byteStride", w.has_stride, w.stride, c.e))
                return false;
            c.views.push_back(w);
        }
    } else if (!ok) return false;
    if (const Json* as = get_array(root, "accessors", c.e, ok)) {
        for (const Json& a : as->arr) {
            Accessor x;
            if (!get_opt_uint(a, "bufferView", x.has_view, x.view, c.e) ||
                !get_uint(a, "byteOffset", false, 0, x.byte_offset, c.e) ||
                !get_uint(a, "componentType", true, 0, x.component_type, c.e) || !get_uint(a, "count", true, 0, x.count, c.e))
                return false;
            const Json* t = a.get("type");
            if (!t || t->kind != Json::String) return c.e.set(RT_ERR_PARSE, "accessor: missing field `type`");
            x.type = t->str;
            c.acc.push_back(x);
        }
    } else if (!ok) return false;
    // nodes + TRS propagation over every scene (convert_nodes, :145-161)
    if (const Json* ns = get_array(root, "nodes", c.e, ok)) {
        for (const Json& n : ns->arr) {
            Node node;
            if (n.kind != Json::Object) return c.e.set(RT_ERR_PARSE, "node must be an object");
            if (!extract_trs(n, node.trs, c.e) || !get_uint_vec(n, "children", false, node.children, c.e) ||
                !get_opt_uint(n, "mesh", node.has_mesh, node.mesh, c.e))
                return false;
            uint64_t cam;
            if (!get_opt_uint(n, "camera", node.has_camera, cam, c.e)) return false;
            c.nodes.push_back(node);
        }
    } else if (!ok) return false;
    std::vector<std::vector<uint64_t>> scenes;
    if (const Json* ss = get_array(root, "scenes", c.e, ok)) {
        for (const Json& s : ss->arr) {
            std::vector<uint64_t> v;
            if (!get_uint_vec(s, "nodes", true, v, c.e)) return false;
            scenes.push_back(v);
        }
    } else if (!ok) return false;
    for (const auto& s : scenes)
        for (uint64_t r : s)
            if (!propagate(c.nodes, r, identity4(), 0, c.e)) return false;
    uint64_t scene;
    if (!get_uint(root, "scene", false, 0, scene, c.e)) return false;
    if (scene >= scenes.size()) return c.e.set(RT_ERR_PARSE, "scene index out of range");
    for (uint64_t r : scenes[scene])  // convert_model (:179-188)
        if (!convert_node(c, r, 0)) return false;
    // extract_camera_params (:57-78)
    const Json* cams = root.get("cameras");
    const Json* cam0 = (cams && cams->kind == Json::Array && cams->arr.size() == 1) ? &cams->arr[0] : nullptr;
    const Json* ty = cam0 ? cam0->get("type") : nullptr;
    const Json* persp = cam0 ? cam0->get("perspective") : nullptr;
    if (!cam0 || !ty || ty->kind != Json::String || ty->str != "perspective" || !persp || persp->kind != Json::Object)
        return c.e.set(RT_ERR_UNSUPPORTED, "Supported only single perspective camera");
    const Json* yf = persp->get("yfov");
    double yfov;
    if (!yf) return c.e.set(RT_ERR_PARSE, "missing field `yfov`");
    if (!get_f64(*yf, yfov, c.e, "yfov")) return false;
    const Node* camnode = nullptr;
    for (const Node& n : c.nodes)
        if (n.has_camera) {
            if (camnode) return c.e.set(RT_ERR_UNSUPPORTED, "You must specify only one a node with the camera");
            camnode = &n;
        }
    if (!camnode) return c.e.set(RT_ERR_UNSUPPORTED, "You must specify a node with the camera");
    rt_render_params& p = c.ps->params;
    std::memset(&p, 0, sizeof(p));
    p.width = W; p.height = H; p.spp = spp;
    p.ray_depth = 8;  // scene_builder.rs:16
    const M4& t = camnode->trs;
    for (int k = 0; k < 3; ++k) {
        p.cam_position[k] = t.m[3][k];
        p.cam_right[k] = t.m[0][k];
        p.cam_up[k] = t.m[1][k];
        p.cam_forward[k] = -t.m[2][k];
    }
    p.fov_axis = RT_FOV_Y;
    p.fov = yfov;
    p.seed = 0x5EED;
    return true;
}

}  // namespace

extern "C" int rt_load_gltf(const char* path, uint32_t W, uint32_t H, uint32_t spp, rt_parsed_scene** out) {
    if (!path || !out) return set_error(RT_ERR_INVALID, "path/out is NULL");
    *out = nullptr;
    if (W == 0 || H == 0 || spp == 0) return set_error(RT_ERR_INVALID, "width/height/spp must be > 0");
    std::ifstream f(path, std::ios::binary);
    if (!f) return set_error(RT_ERR_IO, std::string("Couldn't find or load gltf file: ") + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    Json root;
    std::string err = json_parse(ss.str(), root);
    if (!err.empty()) return set_error(RT_ERR_PARSE, "can't parse glTF: " + err);
    rt_parsed_scene* ps = new rt_parsed_scene();
    ps->tri_mode = RT_TRI_GLTF;
    Ctx c;
    c.root = &root;
    c.ps = ps;
    if (!load(c, path, W, H, spp)) {
        delete ps;
        return set_error(c.e.code, c.e.msg);
    }
    *out = ps;
    return RT_OK;
}
