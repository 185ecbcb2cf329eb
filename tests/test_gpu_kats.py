"""The reference's known-answer tests and the committed golden fixtures, run
through the device path (C ABI -> HIP kernels)."""
import json
import os

import numpy as np
import pytest

from conftest import REPO
from test_oracle import KATS, cg_normalize, triangle_aaa_scene

pytestmark = pytest.mark.gpu
GOLD = os.path.join(REPO, "tests", "golden")


def _one_shape_scene(rt, kind, size, emission=(0.0, 0.0, 0.0)):
    mats = np.zeros(1, rt.MATERIAL_DTYPE)
    mats[0]["emission"] = emission
    shapes = np.zeros(1, rt.SHAPE_DTYPE)
    shapes[0]["type"] = kind
    shapes[0]["shape"] = size
    shapes[0]["rotation"] = (1.0, 0.0, 0.0, 0.0)
    return rt.SceneDesc(materials=mats, shapes=shapes)


def test_kat_box_on_device(rt):
    """primitives/box.rs:129-171 through intersect (intersections.rs:42-62)."""
    s = rt.Scene(_one_shape_scene(rt, rt.RT_SHAPE_BOX, (1.0, 2.0, 1.0)))
    rays = np.array([k["origin"] + cg_normalize(k["dir"]) for k in KATS["box"]])
    hits = s.intersect(rays)
    for k, h in zip(KATS["box"], hits):
        if k["expected"] is None:
            assert h["prim"] == rt.RT_HIT_MISS
        else:
            e = k["expected"]
            assert h["prim"] == 0 and h["t"] == e["t"] and list(h["geometry_normal"]) == e["normal"]
            assert bool(h["inside"]) == e["inside"]


def test_kat_aabb_gate_on_device(rt, orc):
    """aabb.rs:118-151 rays against a light box of the same extent: the BVH root
    AABB gate (bvh.rs:39-44) admits exactly the KAT 'Some' rays."""
    desc = _one_shape_scene(rt, rt.RT_SHAPE_BOX, (1.0, 2.0, 1.0), emission=(1.0, 1.0, 1.0))
    rays = np.array([k["origin"] + cg_normalize(k["dir"]) for k in KATS["aabb"]])
    imp, cnt = rt.Scene(desc).intersect_lights(rays)
    oimp, ocnt = orc.OracleScene(desc).intersect_lights(rays)
    assert np.array_equal(cnt, ocnt) and np.array_equal(imp, oimp)
    assert [c > 0 for c in cnt] == [k["expected_t"] is not None for k in KATS["aabb"]]


def test_kat_triangles_on_device(rt):
    desc, ray = triangle_aaa_scene(rt)
    imp, cnt = rt.Scene(desc).intersect_lights(ray)
    assert cnt[0] >= 1  # primitives/triangle.rs:98-128
    k = KATS["triangle_bbb"]
    mats = np.zeros(1, rt.MATERIAL_DTYPE)
    d2 = rt.SceneDesc(materials=mats, shapes=np.zeros(0, rt.SHAPE_DTYPE),
                      tri_vertices=np.array([k["a"] + k["b"] + k["c"]]), tri_material=np.zeros(1, np.uint32))
    h = rt.Scene(d2).intersect(np.array([k["origin"] + k["dir"]]))
    assert h["prim"][0] == rt.RT_HIT_MISS  # primitives/triangle.rs:130-144


@pytest.mark.parametrize("name", ["cornell_24x16_4spp", "kitchen_sink", "kitchen_sink_deep"])
def test_golden_fixtures_on_device(rt, name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import CASES
    g = np.load(os.path.join(GOLD, name + ".npz"))
    scene, over = CASES[name]
    with open(os.path.join(REPO, "scenes", scene)) as f:
        desc, params = rt.parse_scene(f.read())
    params = params.replace(**over)
    img, hits, st = rt.Scene(desc).generate_image(params, hit_ids=True, stats=True)
    assert np.array_equal(hits, g["hit_ids"])
    assert np.array_equal(img, g["image"])
    keys = ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests", "shaded_hits", "light_queries",
            "light_hits")
    assert [st[k] for k in keys] == [int(v) for v in g["stats"]]
