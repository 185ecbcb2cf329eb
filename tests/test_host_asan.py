"""The host half of the C ABI under AddressSanitizer + UBSan (CPU only).

tests/host_asan/harness.cpp links the product's host sources (parser.cpp, json.cpp,
gltf.cpp, scene_build.cpp, post.cpp) with g++ -fsanitize=address,undefined and runs
parse -> build_scene -> BVH structure checks on every input.  The inputs are the
seeded random scenes (tests/fuzz_scenes.py), the committed scenes, the glTF room
(tests/gltf_scenes.py), and mutations of all of them: truncations, deleted and
duplicated tokens, hostile numbers (nan, inf, 1e400, huge counts), wrong arity,
and glTF documents with out-of-range indices, offsets and counts, bad types, cycles
and truncated JSON.  A malformed input must give an error line — no sanitizer
report, crash or hang — and every valid one must build.
"""
import copy
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import REPO
from fuzz_scenes import random_scene
from gltf_scenes import write_room

SRC = os.path.join(REPO, "cpu-raytracing-rt_amd", "csrc")
HOST_SRCS = ["parser.cpp", "json.cpp", "gltf.cpp", "post.cpp", "scene_build.cpp"]
BAD_NUMBERS = ["nan", "inf", "-inf", "1e400", "-1e400", "-0", "1e-320", "0", "abc", "", "4294967296", "-1",
               "99999999999999999999", "0x10", "1e", "--1", "1,5"]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "harness")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", *[os.path.join(SRC, s) for s in HOST_SRCS],
           os.path.join(REPO, "tests", "host_asan", "harness.cpp"), "-lpthread", "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def run(harness, out_dir, files, timeout=300):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([harness, str(out_dir), *map(str, files)], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "ERROR: LeakSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    lines = r.stdout.splitlines()
    assert lines[-1] == "done"
    # pair-layout lines the harness checked (check_pairs), over every input
    pl = [ln.split() for ln in lines if ln.startswith("pairs ")]
    run.pairs = (int(pl[-1][1]), int(pl[-1][2])) if pl else (0, 0)
    res = {}
    for ln in lines:
        parts = ln.split(" ", 2)
        if len(parts) >= 2 and parts[0] in {str(f) for f in files}:
            res[parts[0]] = parts[1]
    assert len(res) == len(files), "an input printed no result line"
    assert "INVALID" not in res.values()
    return res


def _mutate_text(text, rng):
    toks = text.split(" ")
    lines = text.split("\n")
    k = rng.integers(0, 7)
    if k == 0:
        return text[: int(rng.integers(0, len(text) + 1))]
    if k == 1:
        i = int(rng.integers(0, len(toks)))
        return " ".join(toks[:i] + toks[i + 1:])
    if k == 2:
        i = int(rng.integers(0, len(lines)))
        return "\n".join(lines[: i + 1] + [lines[i]] * int(rng.integers(1, 4)) + lines[i + 1:])
    if k == 3:
        i = int(rng.integers(0, len(toks)))
        toks[i] = str(rng.choice(BAD_NUMBERS))
        return " ".join(toks)
    if k == 4:
        i = int(rng.integers(0, len(lines)))
        kw = str(rng.choice(["NEW_PRIMITIVE", "PLANE", "BOX 1 2", "ELLIPSOID", "TRIANGLE 1 2 3", "ROTATION 1",
                             "DIMENSIONS 0 0", "DIMENSIONS 70000 70000", "SAMPLES 0", "RAY_DEPTH 0",
                             "CAMERA_FOV_X 0", "IOR", "EMISSION 1 1", "UNKNOWN_KEYWORD 1"]))
        return "\n".join(lines[:i] + [kw] + lines[i:])
    if k == 5:
        i = int(rng.integers(0, len(text) + 1))
        junk = bytes(rng.integers(1, 256, int(rng.integers(1, 40)), dtype=np.uint8)).decode("latin-1")
        return text[:i] + junk + text[i:]
    return text + "\n" + "9" * int(rng.integers(300, 5000))


SPECIAL_TEXTS = [
    "", "\n", "NEW_PRIMITIVE", "BOX 1 1 1", "DIMENSIONS", "DIMENSIONS 0 0\nNEW_PRIMITIVE\nBOX 1 1 1",
    "SAMPLES 0\nNEW_PRIMITIVE\nPLANE 0 1 0", "NEW_PRIMITIVE\nTRIANGLE 0 0 0 0 0 0 0 0 0",
    "NEW_PRIMITIVE\nTRIANGLE 0 0 0 1 0 0 2 0 0\nEMISSION 1 1 1",
    "NEW_PRIMITIVE\nBOX 0 0 0\nEMISSION 1 1 1", "NEW_PRIMITIVE\nELLIPSOID 0 0 0\nEMISSION 1 1 1",
    "NEW_PRIMITIVE\nELLIPSOID 1e308 1e308 1e308\nPOSITION 1e308 -1e308 0",
    "NEW_PRIMITIVE\nBOX nan 1 1", "NEW_PRIMITIVE\nPLANE 0 0 0\nROTATION 0 0 0 0",
    "NEW_PRIMITIVE\nPLANE 0 1 0\nNEW_PRIMITIVE\nNEW_PRIMITIVE\nBOX 1 1 1",
    "NEW_PRIMITIVE\nBOX 1 1 1\nBOX 2 2 2\nPLANE 0 1 0",
    "\n".join(["NEW_PRIMITIVE\nTRIANGLE 0 0 0 1 0 0 0 1 0"] * 300),  # 300 identical triangles: one big leaf
]


def test_host_parser_and_builder_fuzz(harness, tmp_path, scene_text):
    rng = np.random.default_rng(2024)
    bases = [random_scene(s) for s in range(40)] + [scene_text(n) for n in
                                                    ("cornell.txt", "kitchen_sink.txt", "box_lights.txt")]
    files, valid = [], []
    for i, t in enumerate(bases):
        p = tmp_path / f"v{i}.txt"
        p.write_text(t)
        files.append(p)
        valid.append(str(p))
    for i in range(600):
        p = tmp_path / f"m{i}.txt"
        t = _mutate_text(bases[int(rng.integers(0, len(bases)))], rng)
        if rng.random() < 0.3:
            t = _mutate_text(t, rng)
        p.write_bytes(t.encode("latin-1", "replace"))
        files.append(p)
    for i, t in enumerate(SPECIAL_TEXTS):
        p = tmp_path / f"s{i}.txt"
        p.write_text(t)
        files.append(p)
    res = run(harness, tmp_path, files)
    for v in valid:
        assert res[v] == "ok", (v, res[v])
    kinds = {k: list(res.values()).count(k) for k in set(res.values())}
    assert kinds.get("parse-error", 0) > 50 and kinds.get("ok", 0) > 100, kinds
    assert run.pairs[0] > 0, "no scene built a pair layout (grid-exact triangles should)"


def _gltf_mutations():
    """(name, mutate(gltf dict)) pairs: every one must end in an error or a valid build."""
    big = 2 ** 31

    def acc(i, **kw):
        return lambda g: g["accessors"][i].update(kw)

    def view(i, **kw):
        return lambda g: g["bufferViews"][i].update(kw)

    def node(i, **kw):
        return lambda g: g["nodes"][i].update(kw)

    def prim(m, p, **kw):
        return lambda g: g["meshes"][m]["primitives"][p].update(kw)

    def setk(path, v):
        def f(g):
            d = g
            for k in path[:-1]:
                d = d[k]
            d[path[-1]] = v
        return f

    def delk(path):
        def f(g):
            d = g
            for k in path[:-1]:
                d = d[k]
            del d[path[-1]]
        return f

    return [
        ("acc_count_huge", acc(0, count=big)), ("acc_count_neg", acc(0, count=-1)),
        ("acc_offset_past", acc(1, byteOffset=10 ** 6)), ("acc_offset_neg", acc(1, byteOffset=-4)),
        ("acc_ctype_bad", acc(2, componentType=5124)), ("acc_ctype_float_idx", acc(2, componentType=5126)),
        ("acc_type_vec2", acc(0, type="VEC2")), ("acc_type_str", acc(0, type=3)),
        ("acc_view_missing", acc(0, bufferView=99)), ("acc_view_neg", acc(0, bufferView=-1)),
        ("acc_no_view", lambda g: g["accessors"][0].pop("bufferView")),
        ("view_len_past", view(0, byteLength=10 ** 7)), ("view_off_past", view(0, byteOffset=10 ** 7)),
        ("view_stride_small", view(0, byteStride=4)), ("view_stride_zero", view(0, byteStride=0)),
        ("view_stride_huge", view(0, byteStride=big)), ("view_buffer_missing", view(0, buffer=5)),
        ("buffer_len_short", setk(["buffers", 0, "byteLength"], 10)),
        ("buffer_len_huge", setk(["buffers", 0, "byteLength"], 10 ** 12)),
        ("buffer_uri_missing", setk(["buffers", 0, "uri"], "nope.bin")),
        ("buffer_uri_data", setk(["buffers", 0, "uri"], "data:application/octet-stream;base64,AAAA")),
        ("no_buffers", delk(["buffers"])),
        ("prim_indices_missing", prim(0, 0, indices=999)), ("prim_pos_missing", prim(0, 0, attributes={})),
        ("prim_normal_wrong_acc", prim(0, 0, attributes={"POSITION": 0, "NORMAL": 2})),
        ("prim_material_missing", prim(0, 0, material=77)), ("prim_mode_points", prim(0, 0, mode=0)),
        ("prim_indices_vec3", prim(1, 0, indices=0)),
        ("idx_count_not3", acc(2, count=35)),
        ("node_mesh_missing", node(1, mesh=42)), ("node_child_missing", node(0, children=[1, 99])),
        ("node_cycle", node(5, children=[4, 5])), ("node_cycle2", node(4, children=[5])),
        ("node_matrix_short", node(4, matrix=[1.0] * 15)), ("node_rot_short", node(5, rotation=[0, 0, 1])),
        ("node_scale_str", node(2, scale="big")), ("node_nan_translation", node(2, translation=[float("nan"), 0, 0])),
        ("camera_missing", node(6, camera=3)), ("no_cameras", delk(["cameras"])),
        ("camera_ortho", setk(["cameras", 0], {"type": "orthographic", "orthographic": {"xmag": 1, "ymag": 1}})),
        ("yfov_zero", setk(["cameras", 0, "perspective", "yfov"], 0.0)),
        ("scene_missing", setk(["scene"], 7)), ("scenes_empty", setk(["scenes"], [])),
        ("scene_node_missing", setk(["scenes", 0, "nodes"], [12])), ("no_nodes", delk(["nodes"])),
        ("meshes_not_list", setk(["meshes"], {"a": 1})), ("materials_null", setk(["materials"], None)),
        ("color_short", setk(["materials", 0, "pbrMetallicRoughness", "baseColorFactor"], [1.0])),
        ("emissive_str", setk(["materials", 3, "emissiveFactor"], "bright")),
    ]


def test_host_gltf_fuzz(harness, tmp_path):
    files, valid = [], []
    path, base = write_room(str(tmp_path), "room")
    files.append(path)
    valid.append(path)
    bin_name = base["buffers"][0]["uri"]
    for name, mut in _gltf_mutations():
        g = copy.deepcopy(base)
        mut(g)
        p = tmp_path / f"{name}.gltf"
        for b in g.get("buffers", []) or []:
            if isinstance(b, dict) and b.get("uri") == bin_name:
                b["uri"] = bin_name  # the room's .bin sits beside every variant
        p.write_text(json.dumps(g))
        files.append(str(p))
    text = open(path).read()
    rng = np.random.default_rng(7)
    for i in range(80):  # truncated and byte-flipped JSON
        t = text[: int(rng.integers(0, len(text)))] if i % 2 == 0 else text
        if i % 2:
            b = bytearray(t.encode())
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(0, len(b)))] = int(rng.choice(list(b'{}[],:"0123456789-.e ')))
            t = b.decode("latin-1")
        p = tmp_path / f"j{i}.gltf"
        p.write_bytes(t.encode("latin-1"))
        files.append(str(p))
    res = run(harness, tmp_path, files)
    assert res[path] == "ok"
    assert list(res.values()).count("parse-error") > 40
