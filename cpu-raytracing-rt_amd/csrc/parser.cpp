// parser.cpp — the custom text scene format (input surface).
//
// Restates scene_parser.rs:5-85 (keywords, one primitive per NEW_PRIMITIVE,
// unknown lines ignored) and the defaults of Scene::new / CameraParams::new /
// Metadata::new (scene.rs:92-106, 167-191).  Where the reference panics
// (unwrap on a missing token, a property before NEW_PRIMITIVE, a primitive
// without a shape, DIELECTRIC without IOR, no DIMENSIONS) this returns
// RT_ERR_PARSE with the line number.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "api_internal.h"
#include "rt_math.h"

using namespace rt;

namespace {

struct Props {  // parsed_scene::PrimitiveProperties (parsed_scene.rs:18-26)
    std::optional<int> material;  // RT_MAT_METALLIC | RT_MAT_DIELECTRIC
    std::optional<double> ior;
    std::optional<V3> position, color, emission;
    std::optional<Quat> rotation;
};
struct Prim {  // parsed_scene::Primitive
    int type = -1;  // 0 plane 1 box 2 ellipsoid 3 triangle
    double v[9] = {0};
    Props props;
};

// Rust's f64 FromStr accepts decimal/scientific, inf/infinity/nan (any case),
// an optional sign; it rejects hex floats and surrounding junk.
bool parse_f64(const std::string& tok, double& out) {
    if (tok.empty()) return false;
    std::string t = tok;
    size_t i = (t[0] == '+' || t[0] == '-') ? 1 : 0;
    std::string body = t.substr(i);
    std::string low;
    for (char c : body) low.push_back((char)std::tolower((unsigned char)c));
    if (low == "inf" || low == "infinity" || low == "nan") {
        double v = low == "nan" ? NAN : INFINITY;
        out = (t[0] == '-') ? -v : v;
        return true;
    }
    bool digit = false;
    for (char c : body) {
        if (std::isdigit((unsigned char)c)) digit = true;
        else if (!(c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-')) return false;
    }
    if (!digit) return false;
    errno = 0;
    char* end = nullptr;
    out = std::strtod(t.c_str(), &end);
    return end && *end == '\0';
}
bool parse_uint(const std::string& tok, uint64_t maxv, uint64_t& out) {
    std::string t = tok;
    if (!t.empty() && t[0] == '+') t = t.substr(1);
    if (t.empty()) return false;
    uint64_t v = 0;
    for (char c : t) {
        if (!std::isdigit((unsigned char)c)) return false;
        uint64_t d = (uint64_t)(c - '0');
        if (v > (maxv - d) / 10) return false;
        v = v * 10 + d;
    }
    out = v;
    return true;
}

struct Reader {
    std::vector<std::string> toks;
    size_t pos = 1;
    bool ok = true;
    double f() {
        double v = 0;
        if (pos >= toks.size() || !parse_f64(toks[pos], v)) ok = false;
        ++pos;
        return v;
    }
    V3 vec() { double x = f(), y = f(), z = f(); return v3(x, y, z); }
};

}  // namespace

extern "C" int rt_parse_custom_scene(const char* text, rt_parsed_scene** out) {
    if (!text || !out) return set_error(RT_ERR_INVALID, "text/out is NULL");
    *out = nullptr;
    std::vector<Prim> prims;
    std::optional<V3> cam_pos, cam_right, cam_up, cam_fwd, bg;
    std::optional<double> fov_x;
    std::optional<uint64_t> ray_depth, samples, dim_w, dim_h;
    std::istringstream in(text);
    std::string line;
    size_t lineno = 0;
    auto fail = [&](const char* what) {
        return set_error(RT_ERR_PARSE, "line " + std::to_string(lineno) + ": " + what);
    };
    while (std::getline(in, line)) {  // scene_parser.rs:8-40
        ++lineno;
        Reader r;
        {
            std::string tok;
            for (char c : line) {  // split_ascii_whitespace
                if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f') {
                    if (!tok.empty()) { r.toks.push_back(tok); tok.clear(); }
                } else tok.push_back(c);
            }
            if (!tok.empty()) r.toks.push_back(tok);
        }
        if (r.toks.empty()) continue;
        const std::string& k = r.toks[0];
        const bool prim_kw = k == "BOX" || k == "PLANE" || k == "ELLIPSOID" || k == "TRIANGLE" || k == "POSITION" ||
                             k == "ROTATION" || k == "COLOR" || k == "EMISSION" || k == "METALLIC" ||
                             k == "DIELECTRIC" || k == "IOR";
        if (k == "NEW_PRIMITIVE") { prims.emplace_back(); continue; }
        if (prim_kw && prims.empty()) return fail("primitive property before NEW_PRIMITIVE");
        Prim* p = prims.empty() ? nullptr : &prims.back();
        if (k == "BOX" || k == "PLANE" || k == "ELLIPSOID") {
            V3 v = r.vec();
            if (!r.ok) return fail("expected 3 numbers");
            p->type = k == "PLANE" ? 0 : (k == "BOX" ? 1 : 2);
            store3(p->v, v);
        } else if (k == "TRIANGLE") {
            V3 a = r.vec(), b = r.vec(), c = r.vec();
            if (!r.ok) return fail("expected 9 numbers");
            p->type = 3;
            store3(p->v, a); store3(p->v + 3, b); store3(p->v + 6, c);
        } else if (k == "POSITION") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); p->props.position = v; }
        else if (k == "ROTATION") {  // next_quat: x y z then w (scene_parser.rs:51-57)
            V3 xyz = r.vec();
            double w = r.f();
            if (!r.ok) return fail("expected 4 numbers");
            p->props.rotation = Quat{w, xyz};
        } else if (k == "COLOR") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); p->props.color = v; }
        else if (k == "EMISSION") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); p->props.emission = v; }
        else if (k == "METALLIC") p->props.material = RT_MAT_METALLIC;
        else if (k == "DIELECTRIC") p->props.material = RT_MAT_DIELECTRIC;
        else if (k == "IOR") { double v = r.f(); if (!r.ok) return fail("expected a number"); p->props.ior = v; }
        else if (k == "CAMERA_POSITION") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); cam_pos = v; }
        else if (k == "CAMERA_RIGHT") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); cam_right = v; }
        else if (k == "CAMERA_UP") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); cam_up = v; }
        else if (k == "CAMERA_FORWARD") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); cam_fwd = v; }
        else if (k == "CAMERA_FOV_X") { double v = r.f(); if (!r.ok) return fail("expected a number"); fov_x = v; }
        else if (k == "DIMENSIONS") {
            uint64_t w = 0, h = 0;
            if (r.toks.size() < 3 || !parse_uint(r.toks[1], UINT64_MAX, w) || !parse_uint(r.toks[2], UINT64_MAX, h))
                return fail("expected 2 unsigned integers");
            dim_w = w; dim_h = h;
        } else if (k == "RAY_DEPTH") {
            uint64_t v = 0;
            if (r.toks.size() < 2 || !parse_uint(r.toks[1], 255, v)) return fail("expected a u8");
            ray_depth = v;
        } else if (k == "BG_COLOR") { V3 v = r.vec(); if (!r.ok) return fail("expected 3 numbers"); bg = v; }
        else if (k == "SAMPLES") {
            uint64_t v = 0;
            if (r.toks.size() < 2 || !parse_uint(r.toks[1], UINT64_MAX, v)) return fail("expected an unsigned integer");
            samples = v;
        }
        // any other keyword: ignored (scene_parser.rs:37-38)
    }
    if (!dim_w) return set_error(RT_ERR_PARSE, "DIMENSIONS missing (scene.rs:188 unwraps it)");
    if (*dim_w == 0 || *dim_h == 0 || *dim_w > 0xffffffffull || *dim_h > 0xffffffffull)
        return set_error(RT_ERR_PARSE, "DIMENSIONS out of range");
    if (samples && (*samples == 0 || *samples > 0xffffffffull)) return set_error(RT_ERR_PARSE, "SAMPLES out of range");

    rt_parsed_scene* ps = new rt_parsed_scene();
    ps->tri_mode = RT_TRI_CUSTOM;
    for (size_t i = 0; i < prims.size(); ++i) {  // make_scenes (scene.rs:200-207) + Metadata::new (:92-106)
        const Prim& p = prims[i];
        if (p.type < 0) { delete ps; return set_error(RT_ERR_PARSE, "primitive " + std::to_string(i) + " has no shape"); }
        rt_material m{};
        if (p.props.material && *p.props.material == RT_MAT_DIELECTRIC) {
            if (!p.props.ior) { delete ps; return set_error(RT_ERR_PARSE, "DIELECTRIC primitive without IOR"); }
            m.kind = RT_MAT_DIELECTRIC;
            m.ior = *p.props.ior;
        } else if (p.props.material) m.kind = RT_MAT_METALLIC;
        else m.kind = RT_MAT_DIFFUSE;
        store3(m.color, p.props.color.value_or(v3(0, 0, 0)));
        store3(m.emission, p.props.emission.value_or(v3(0, 0, 0)));
        uint32_t mid = (uint32_t)ps->mats.size();
        ps->mats.push_back(m);
        V3 pos = p.props.position.value_or(v3(0, 0, 0));
        Quat rot = p.props.rotation.value_or(Quat{1.0, v3(0, 0, 0)});
        if (p.type == 3) {
            ps->tri_v.insert(ps->tri_v.end(), p.v, p.v + 9);
            ps->tri_pos.insert(ps->tri_pos.end(), {pos.x, pos.y, pos.z});
            ps->tri_rot.insert(ps->tri_rot.end(), {rot.s, rot.v.x, rot.v.y, rot.v.z});
            ps->tri_mat.push_back(mid);
        } else {
            rt_shape s{};
            s.type = p.type == 0 ? RT_SHAPE_PLANE : (p.type == 1 ? RT_SHAPE_BOX : RT_SHAPE_ELLIPSOID);
            s.material = mid;
            std::memcpy(s.shape, p.v, sizeof(s.shape));
            store3(s.position, pos);
            s.rotation[0] = rot.s; s.rotation[1] = rot.v.x; s.rotation[2] = rot.v.y; s.rotation[3] = rot.v.z;
            ps->shapes.push_back(s);
        }
    }
    rt_render_params& rp = ps->params;  // Scene::new (scene.rs:180-191), CameraParams::new (:167-177)
    std::memset(&rp, 0, sizeof(rp));
    rp.width = (uint32_t)*dim_w;
    rp.height = (uint32_t)*dim_h;
    rp.spp = (uint32_t)samples.value_or(64);
    rp.ray_depth = (uint32_t)ray_depth.value_or(16);
    store3(rp.bg_color, bg.value_or(v3(0, 0, 0)));
    store3(rp.cam_position, cam_pos.value_or(v3(0, 0, 0)));
    store3(rp.cam_right, normalize(cam_right.value_or(v3(1, 0, 0))));
    store3(rp.cam_up, normalize(cam_up.value_or(v3(0, 1, 0))));
    store3(rp.cam_forward, normalize(cam_fwd.value_or(v3(0, 0, 1))));
    rp.fov_axis = RT_FOV_X;
    rp.fov = fov_x.value_or(kPi / 2.0);
    rp.seed = 0x5EED;
    *out = ps;
    return RT_OK;
}

extern "C" int rt_parsed_scene_get(const rt_parsed_scene* ps, rt_scene_desc* d, rt_render_params* p) {
    if (!ps) return set_error(RT_ERR_INVALID, "parsed scene is NULL");
    if (d) {
        std::memset(d, 0, sizeof(*d));
        d->n_materials = (uint32_t)ps->mats.size();
        d->materials = ps->mats.data();
        d->n_shapes = (uint32_t)ps->shapes.size();
        d->shapes = ps->shapes.data();
        d->n_triangles = ps->tri_mat.size();
        d->tri_mode = ps->tri_mode;
        d->tri_vertices = ps->tri_v.empty() ? nullptr : ps->tri_v.data();
        d->tri_normals = ps->tri_n.empty() ? nullptr : ps->tri_n.data();
        d->tri_position = ps->tri_pos.empty() ? nullptr : ps->tri_pos.data();
        d->tri_rotation = ps->tri_rot.empty() ? nullptr : ps->tri_rot.data();
        d->tri_material = ps->tri_mat.empty() ? nullptr : ps->tri_mat.data();
    }
    if (p) *p = ps->params;
    return RT_OK;
}

extern "C" void rt_parsed_scene_free(rt_parsed_scene* ps) { delete ps; }
