"""glTF input surface: the product's C++ reader
(`rt_load_gltf`, csrc/gltf.cpp) against the independent Python restatement in
oracle/gltf_oracle.py, bit for bit, plus the reference's own cof unit test
(src/gltf/scene_builder.rs:400-427) and its panics as error codes.

CPU only: the reader is host code.  Parity note: the reference ships no glTF
asset, so the fixtures are synthetic (tests/gltf_scenes.py); see the oracle
header.
"""
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
import gltf_scenes

sys.path.insert(0, os.path.join(REPO, "oracle"))
import gltf_oracle as go  # noqa: E402


def bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


def assert_same(rt, path, W=64, H=48, spp=4):
    desc, params = rt.load_gltf(path, W, H, spp)
    ref = go.load(path, W, H, spp)
    assert desc.tri_mode == rt.RT_TRI_GLTF
    assert len(desc.shapes) == 0
    n = len(ref["tri_material"])
    assert len(desc.tri_material) == n
    if n:
        assert np.array_equal(bits(desc.tri_vertices), bits(ref["tri_vertices"]))
        assert np.array_equal(bits(desc.tri_normals), bits(ref["tri_normals"]))
        assert np.array_equal(desc.tri_material, np.array(ref["tri_material"], np.uint32))
    assert len(desc.materials) == len(ref["materials"])
    for m, (kind, ior, color, em) in zip(desc.materials, ref["materials"]):
        assert int(m["kind"]) == kind
        assert float(m["ior"]) == ior
        assert np.array_equal(bits(m["color"]), bits(color))
        assert np.array_equal(bits(m["emission"]), bits(em))
    cam = ref["camera"]
    assert (params.width, params.height, params.spp) == (W, H, spp)
    assert params.ray_depth == 8 and tuple(params.bg_color) == (0.0, 0.0, 0.0)
    assert params.fov_axis == rt.RT_FOV_Y and params.fov == cam["yfov"]
    for k in ("position", "right", "up", "forward"):
        assert np.array_equal(bits(getattr(params, "cam_" + k)), bits(cam[k])), k
    return desc, params, ref


def test_reference_cof_unit_test():
    """scene_builder.rs:400-427: cof(M)·n and (M^T)^-1·n have the same direction."""
    def rx(d):
        c, s = math.cos(math.radians(d)), math.sin(math.radians(d))
        return np.array([[1, 0, 0], [0, c, s], [0, -s, c]]).T  # cgmath from_angle_x (columns)

    def ry(d):
        c, s = math.cos(math.radians(d)), math.sin(math.radians(d))
        return np.array([[c, 0, -s], [0, 1, 0], [s, 0, c]]).T

    def rz(d):
        c, s = math.cos(math.radians(d)), math.sin(math.radians(d))
        return np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]]).T

    mt = rx(10) @ ry(20) @ rz(30) @ np.diag([2.0, 3.0, 4.0])   # row-major here
    m4 = [[mt[0][c], mt[1][c], mt[2][c], 0.0] for c in range(3)] + [[0.0, 0.0, 0.0, 1.0]]
    cof = go.cof(m4)
    inv_t = np.linalg.inv(mt.T)
    for n in ([1.0, 2.0, 3.0], [-1.0, 2.0, 3.0], [-1.0, -2.0, 1.0]):
        n = np.array(n) / np.linalg.norm(n)
        a = np.array([sum(cof[c][r] * n[c] for c in range(3)) for r in range(3)])
        b = inv_t @ n
        assert np.allclose(a / np.linalg.norm(a), b / np.linalg.norm(b), atol=4 * np.finfo(float).eps)


def test_room_bit_exact(rt, tmp_path):
    path, _ = gltf_scenes.write_room(str(tmp_path))
    desc, params, ref = assert_same(rt, path)
    # 12 room + 2*256 sphere + 2 light + 2*12 cube triangles; one material per primitive
    assert len(desc.tri_material) == 12 + 2 * 256 + 2 + 24
    kinds = [int(m["kind"]) for m in desc.materials]
    assert kinds == [rt.RT_MAT_DIFFUSE, rt.RT_MAT_METALLIC, rt.RT_MAT_DIELECTRIC, rt.RT_MAT_DIFFUSE,
                     rt.RT_MAT_DIFFUSE, rt.RT_MAT_METALLIC]  # last: no material => default (metallic 1.0)
    assert desc.materials[2]["ior"] == 1.5
    assert list(desc.materials[3]["emission"]) == [6.0, 0.9 * 6.0, 0.7 * 6.0]
    assert list(desc.materials[3]["color"]) == [1.0, 1.0, 1.0]
    # normals are unit length after cof + normalize
    nn = desc.tri_normals.reshape(-1, 3)
    assert np.allclose(np.linalg.norm(nn, axis=1), 1.0, atol=1e-15)


def test_scene_and_yfov_selection(rt, tmp_path):
    path = gltf_scenes.write_variant(str(tmp_path), lambda g: g.update(scene=1))
    desc, _, _ = assert_same(rt, path)
    assert len(desc.tri_material) == 24 + 12   # cube mesh (2 primitives) at node 8 + room


def test_propagation_runs_over_every_scene(rt, tmp_path):
    """A node listed by a second scene is propagated twice (scene_builder.rs:155-161)."""
    base, _ = gltf_scenes.write_room(str(tmp_path / "a"))
    d0, _ = rt.load_gltf(base, 8, 8, 1)
    path = gltf_scenes.write_variant(str(tmp_path / "b"), lambda g: g["scenes"][1]["nodes"].append(5))
    d1, _, _ = assert_same(rt, path, 8, 8, 1)
    cube = slice(12 + 512 + 2, None)
    assert not np.array_equal(d0.tri_vertices[cube], d1.tri_vertices[cube])
    assert np.array_equal(d0.tri_vertices[:12], d1.tri_vertices[:12])


def test_sponza_like_generator_small(rt, tmp_path):
    gen = os.path.join(REPO, "scenes", "gen_sponza_like.py")
    subprocess.run([sys.executable, gen, str(tmp_path), "--scale", "0.02", "--name", "mini"], check=True,
                   capture_output=True)
    desc, _, _ = assert_same(rt, str(tmp_path / "mini.gltf"), 32, 18, 1)
    kinds = [int(m["kind"]) for m in desc.materials]
    assert rt.RT_MAT_METALLIC in kinds and rt.RT_MAT_DIELECTRIC in kinds
    assert any(m["emission"].max() > 0 for m in desc.materials)


def test_hairball_generator_small(rt, tmp_path):
    gen = os.path.join(REPO, "scenes", "gen_hairball.py")
    subprocess.run([sys.executable, gen, str(tmp_path), "--tris", "3000", "--name", "hb"], check=True,
                   capture_output=True)
    desc, params, _ = assert_same(rt, str(tmp_path / "hb.gltf"), 32, 24, 1)
    assert len(desc.tri_material) == 3002
    assert sum(1 for m in desc.materials if m["emission"].max() > 0) == 1
    assert desc.tri_vertices.reshape(-1, 3)[:-6].__abs__().max() < 1.0  # inside the unit ball


def _del(path):
    def f(g):
        obj = g
        for k in path[:-1]:
            obj = obj[k]
        del obj[path[-1]]
    return f


ERRORS = {
    "mode_lines": lambda g: g["meshes"][0]["primitives"][0].update(mode=1),
    "no_normal": _del(["meshes", 2, "primitives", 0, "attributes", "NORMAL"]),
    "no_position": _del(["meshes", 2, "primitives", 0, "attributes", "POSITION"]),
    "two_cameras": lambda g: g["cameras"].append(g["cameras"][0]),
    "ortho_camera": lambda g: g["cameras"][0].update(type="orthographic"),
    "no_camera_node": _del(["nodes", 6, "camera"]),
    "two_camera_nodes": lambda g: g["nodes"][8].update(camera=0),
    "missing_bin": lambda g: g["buffers"][0].update(uri="nope.bin"),
    "buffer_without_uri": _del(["buffers", 0, "uri"]),
    "bad_matrix": lambda g: g["nodes"][4].update(matrix=[1.0] * 15),
    "bad_translation": lambda g: g["nodes"][2].update(translation=[1.0, 2.0]),
    "scene_out_of_range": lambda g: g.update(scene=7),
    "unused_material_bad_ext": lambda g: g["materials"].append(
        {"extensions": {"KHR_materials_emissive_strength": {}}}),
    "negative_index": lambda g: g["meshes"][0]["primitives"][0].update(material=-1),
    "float_index": lambda g: g["meshes"][0]["primitives"][0].update(indices=1.5),
    "bad_base_color": lambda g: g["materials"][0]["pbrMetallicRoughness"].update(baseColorFactor=[1, 1, 1]),
    "index_accessor_float": lambda g: g["accessors"][2].update(componentType=5126),
    "position_u16": lambda g: g["accessors"][0].update(componentType=5123),
}


@pytest.mark.parametrize("case", sorted(ERRORS))
def test_reference_panics_become_errors(rt, tmp_path, case):
    path = gltf_scenes.write_variant(str(tmp_path), ERRORS[case])
    with pytest.raises(go.GltfError):
        go.load(path, 8, 8, 1)
    with pytest.raises(rt.RtError) as e:
        rt.load_gltf(path, 8, 8, 1)
    assert e.value.code in (rt.RT_ERR_PARSE, rt.RT_ERR_UNSUPPORTED, rt.RT_ERR_IO)


def test_unparseable_and_missing(rt, tmp_path):
    p = tmp_path / "bad.gltf"
    p.write_text('{"asset": {"version": "2.0"}, "nodes": [}')
    with pytest.raises(rt.RtError) as e:
        rt.load_gltf(str(p), 8, 8, 1)
    assert e.value.code == rt.RT_ERR_PARSE
    with pytest.raises(rt.RtError) as e:
        rt.load_gltf(str(tmp_path / "absent.gltf"), 8, 8, 1)
    assert e.value.code == rt.RT_ERR_IO
    path, _ = gltf_scenes.write_room(str(tmp_path))
    with pytest.raises(rt.RtError) as e:
        rt.load_gltf(path, 0, 8, 1)
    assert e.value.code == rt.RT_ERR_INVALID
