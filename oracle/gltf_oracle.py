"""Oracle for the glTF input surface — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's glTF loader, written independently of
the product's C++ reader (cpu-raytracing-rt_amd/csrc/gltf.cpp) so the two can
be compared bit for bit:
  * serde model and defaults — src/gltf/parser.rs:4-220 (metallicFactor
    default 1.0 :63-64/:204-208, emissiveStrength default 1.0 :210-214,
    mode default 4 :193-195, scene default 0 :152-153);
  * build_scene — src/gltf/scene_builder.rs:9-398 (TRS :108-143, propagation
    over every scene :155-169, default-scene traversal :179-207, readers
    :237-327, cof :367-388, make_metadata :227-235, camera :57-78).
cgmath 0.18 arithmetic (f64, no FMA) is restated with Python floats, which are
IEEE binary64 with round-to-nearest: Matrix4*Matrix4 and Matrix4*Vector4 as
left-to-right column combinations, Quaternion->Matrix4, Vector3::normalize as
v * (1/|v|).

Parity pin: the reference ships no glTF asset or golden, and it cannot run here
(Rust toolchain absent), so this oracle is anchored on the reference source and
its one unit test (scene_builder.rs:400-427: cof(M)·n ∥ (M^T)^-1·n, checked in
tests/test_gltf.py). Treat the glTF row as "parity pinned to a restatement".
Only tests/ may import this module.
"""
import json
import math
import os
import struct

MAT_DIFFUSE, MAT_METALLIC, MAT_DIELECTRIC = 0, 1, 2


class GltfError(Exception):
    """Where the reference panics (assert!/expect/index out of range)."""


# ---- cgmath restatement (Matrix4 stored as 4 columns of 4) -----------------
def identity():
    return [[1.0 if c == r else 0.0 for r in range(4)] for c in range(4)]


def matmul(a, b):
    out = []
    for c in range(4):
        col = []
        for r in range(4):
            col.append(((a[0][r] * b[c][0] + a[1][r] * b[c][1]) + a[2][r] * b[c][2]) + a[3][r] * b[c][3])
        out.append(col)
    return out


def matvec(m, v):
    return [((m[0][r] * v[0] + m[1][r] * v[1]) + m[2][r] * v[2]) + m[3][r] * v[3] for r in range(4)]


def quat_to_mat(s, x, y, z):
    x2, y2, z2 = x + x, y + y, z + z
    xx2, xy2, xz2 = x2 * x, x2 * y, x2 * z
    yy2, yz2, zz2 = y2 * y, y2 * z, z2 * z
    sy2, sz2, sx2 = y2 * s, z2 * s, x2 * s
    return [[1.0 - yy2 - zz2, xy2 + sz2, xz2 - sy2, 0.0],
            [xy2 - sz2, 1.0 - xx2 - zz2, yz2 + sx2, 0.0],
            [xz2 + sy2, yz2 - sx2, 1.0 - xx2 - yy2, 0.0],
            [0.0, 0.0, 0.0, 1.0]]


def cof(m):
    """scene_builder.rs:367-388 on mat4_to_mat3(m); result[col][row]."""
    other = {0: (1, 2), 1: (0, 2), 2: (0, 1)}
    out = [[0.0] * 3 for _ in range(3)]
    for col in range(3):
        for row in range(3):
            lc, rc = other[col]
            tr, br = other[row]
            det = m[lc][tr] * m[rc][br] - m[rc][tr] * m[lc][br]
            out[col][row] = -det if (col + row) & 1 else det
    return out


def normalize(v):
    inv = 1.0 / math.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return [v[0] * inv, v[1] * inv, v[2] * inv]


# ---- serde-ish field access -------------------------------------------------
def _req(obj, key):
    if not isinstance(obj, dict) or key not in obj or obj[key] is None:
        raise GltfError(f"missing field `{key}`")
    return obj[key]


def _usize(v, key):
    if isinstance(v, bool) or not isinstance(v, int) or v < 0:
        raise GltfError(f"field `{key}`: expected usize")
    return v


def _opt_usize(obj, key):
    v = obj.get(key)
    return None if v is None else _usize(v, key)


def _floats(v, key):
    if not isinstance(v, list) or any(isinstance(x, bool) or not isinstance(x, (int, float)) for x in v):
        raise GltfError(f"field `{key}`: expected array of numbers")
    return [float(x) for x in v]


def extract_trs(node):
    if node.get("matrix") is not None:
        mt = _floats(node["matrix"], "matrix")
        if len(mt) != 16:
            raise GltfError("matrix len")
        return [mt[4 * c:4 * c + 4] for c in range(4)]
    t = _floats(node["translation"], "translation") if node.get("translation") is not None else [0.0, 0.0, 0.0]
    q = _floats(node["rotation"], "rotation") if node.get("rotation") is not None else [0.0, 0.0, 0.0, 1.0]
    s = _floats(node["scale"], "scale") if node.get("scale") is not None else [1.0, 1.0, 1.0]
    if len(t) != 3 or len(s) != 3 or len(q) != 4:
        raise GltfError("TRS len")
    T = identity()
    T[3][0], T[3][1], T[3][2] = t
    R = quat_to_mat(q[3], q[0], q[1], q[2])
    S = identity()
    S[0][0], S[1][1], S[2][2] = s
    return matmul(matmul(T, R), S)


def make_metadata(mat):
    """scene_builder.rs:227-235 -> (kind, ior, color[3], emission[3])."""
    mat = mat or {}
    pbr = mat.get("pbrMetallicRoughness") or {}
    color = _floats(pbr["baseColorFactor"], "baseColorFactor") if pbr.get("baseColorFactor") is not None \
        else [1.0, 1.0, 1.0, 1.0]
    if len(color) != 4:
        raise GltfError("baseColorFactor len")
    metallic = float(pbr.get("metallicFactor", 1.0))
    em = _floats(mat["emissiveFactor"], "emissiveFactor") if mat.get("emissiveFactor") is not None else [0.0] * 3
    if len(em) != 3:
        raise GltfError("emissiveFactor len")
    ext = (mat.get("extensions") or {}).get("KHR_materials_emissive_strength")
    strength = 1.0 if ext is None else float(_req(ext, "emissiveStrength"))
    if color[3] < 1.0:
        kind, ior = MAT_DIELECTRIC, 1.5
    elif metallic > 0.0:
        kind, ior = MAT_METALLIC, 0.0
    else:
        kind, ior = MAT_DIFFUSE, 0.0
    return kind, ior, color[:3], [e * strength for e in em]


class _Ctx:
    def __init__(self, model, base_dir):
        self.m = model
        self.buffers = {}
        for b in model.get("buffers", []):
            _usize(_req(b, "byteLength"), "byteLength")
            uri = b.get("uri")
            if uri is None:
                raise GltfError("expected uri for buffer")
            try:
                with open(os.path.join(base_dir, uri), "rb") as f:
                    self.buffers[uri] = f.read()
            except OSError as e:
                raise GltfError(f"Couldn't find or load '{uri}' file.") from e

    def view_of(self, acc, elem):
        view = self.m["bufferViews"][acc["bufferView"]]
        buf = self.m["buffers"][_usize(_req(view, "buffer"), "buffer")]
        data = self.buffers[buf["uri"]]
        off = view.get("byteOffset", 0) + acc.get("byteOffset", 0)
        stride = view.get("byteStride")
        return data, off, elem if stride is None else stride

    def read_vec3(self, ai):
        acc = self.m["accessors"][ai]
        if acc.get("bufferView") is None:
            return []
        if acc["componentType"] != 5126 or acc["type"] != "VEC3":
            raise GltfError("vertices must be FLOAT VEC3")
        data, off, stride = self.view_of(acc, 12)
        out = []
        for _ in range(acc["count"]):
            if off + 12 > len(data):
                raise GltfError("read past end of buffer")
            out.append([float(x) for x in struct.unpack_from("<3f", data, off)])
            off += stride
        return out

    def read_indices(self, ai):
        acc = self.m["accessors"][ai]
        if acc.get("bufferView") is None:
            return []
        ct = acc["componentType"]
        if ct not in (5123, 5125) or acc["type"] != "SCALAR":
            raise GltfError("bad index accessor")
        es = 2 if ct == 5123 else 4
        data, off, stride = self.view_of(acc, es)
        out = []
        for _ in range(acc["count"]):
            if off + es > len(data):
                raise GltfError("read past end of buffer")
            out.append(struct.unpack_from("<H" if es == 2 else "<I", data, off)[0])
            off += stride
        return out


def load(path, width, height, spp):
    """gltf::parse + build_scene. Returns a dict: tri_vertices / tri_normals as
    lists of 9 floats per triangle (a, b, c / na, nb, nc — the raw world-space
    corners), tri_material (index into materials), materials (one per mesh
    primitive in traversal order), camera (position, right, up, forward, yfov)
    and ray_depth / bg."""
    with open(path, "r") as f:
        try:
            model = json.load(f)
        except json.JSONDecodeError as e:
            raise GltfError(f"can't parse glTF: {e}") from e
    if not isinstance(model, dict):
        raise GltfError("can't parse glTF")
    for m in model.get("materials", []):
        make_metadata(m)
    for mesh in model.get("meshes", []):
        for p in _req(mesh, "primitives"):
            attr = _req(p, "attributes")
            _usize(_req(attr, "POSITION"), "POSITION")
            for k, o in (("NORMAL", attr), ("indices", p), ("material", p), ("mode", p)):
                _opt_usize(o, k)
    ctx = _Ctx(model, os.path.dirname(path))
    nodes = []
    for n in model.get("nodes", []):
        nodes.append({"trs": extract_trs(n), "children": [_usize(c, "children") for c in n.get("children", [])],
                      "mesh": _opt_usize(n, "mesh"), "camera": _opt_usize(n, "camera")})
    scenes = [[_usize(x, "nodes") for x in _req(s, "nodes")] for s in model.get("scenes", [])]

    def propagate(i, parent, depth=0):
        if depth > 1000:
            raise GltfError("cycle")
        nodes[i]["trs"] = matmul(parent, nodes[i]["trs"])
        for ch in nodes[i]["children"]:
            propagate(ch, nodes[i]["trs"], depth + 1)

    for s in scenes:
        for r in s:
            propagate(r, identity())
    scene = _usize(model.get("scene", 0), "scene")
    if scene >= len(scenes):
        raise GltfError("scene index out of range")

    out = {"tri_vertices": [], "tri_normals": [], "tri_material": [], "materials": []}

    def convert_primitive(p, trs):
        if p.get("mode", 4) != 4:
            raise GltfError("supported only triangles for primitive.mode")
        attr = p["attributes"]
        verts = []
        for v in ctx.read_vec3(attr["POSITION"]):
            w = matvec(trs, v + [1.0])
            if w[3] != 1.0:
                raise GltfError("pos.w != 1")
            verts.append(w[:3])
        if attr.get("NORMAL") is None:
            raise GltfError("empty normals")
        rs = cof(trs)
        norms = [normalize([(rs[0][r] * n[0] + rs[1][r] * n[1]) + rs[2][r] * n[2] for r in range(3)])
                 for n in ctx.read_vec3(attr["NORMAL"])]
        if len(verts) != len(norms):
            raise GltfError("vertex/normal count mismatch")
        if p.get("indices") is not None:
            idx = ctx.read_indices(p["indices"])
        else:
            idx = list(range(len(verts)))
        if len(idx) % 3:
            raise GltfError("count not a multiple of 3")
        mi = p.get("material")
        md = make_metadata(None if mi is None else model["materials"][mi])
        out["materials"].append(md)
        for k in range(0, len(idx), 3):
            a, b, c = idx[k:k + 3]
            out["tri_vertices"].append(verts[a] + verts[b] + verts[c])
            out["tri_normals"].append(norms[a] + norms[b] + norms[c])
            out["tri_material"].append(len(out["materials"]) - 1)

    def convert_node(i, depth=0):
        if depth > 1000:
            raise GltfError("cycle")
        n = nodes[i]
        if n["mesh"] is not None:
            for p in _req(model["meshes"][n["mesh"]], "primitives"):
                convert_primitive(p, n["trs"])
        for ch in n["children"]:
            convert_node(ch, depth + 1)

    for r in scenes[scene]:
        convert_node(r)

    cams = model.get("cameras", [])
    if not (len(cams) == 1 and cams[0].get("type") == "perspective" and cams[0].get("perspective") is not None):
        raise GltfError("Supported only single perspective camera")
    yfov = float(_req(cams[0]["perspective"], "yfov"))
    cam_nodes = [n for n in nodes if n["camera"] is not None]
    if len(cam_nodes) != 1:
        raise GltfError("You must specify exactly one node with the camera")
    t = cam_nodes[0]["trs"]
    out["camera"] = {"position": t[3][:3], "right": t[0][:3], "up": t[1][:3],
                     "forward": [-t[2][0], -t[2][1], -t[2][2]], "yfov": yfov}
    out["ray_depth"], out["bg"] = 8, [0.0, 0.0, 0.0]
    out["width"], out["height"], out["spp"] = width, height, spp
    return out
