"""GPU parity on glTF scenes (smooth-normal triangles, tri_mode 1 — the C3
"Sponza-class" code path): the HIP renderer through the C ABI against the
oracle, with the same bar as test_gpu_parity.py (hit ids and iterative-form
radiance bit-exact; recursive form within REL_TOL; counters equal)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
import gltf_scenes
from test_gpu_parity import _compare, form, intersect_device, segment_form  # noqa: F401 (autouse: every form)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def room(rt, orc, tmp_path_factory):
    path, _ = gltf_scenes.write_room(str(tmp_path_factory.mktemp("room")))
    desc, params = rt.load_gltf(path, 40, 30, 4)
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.fixture(scope="module")
def atrium(rt, orc, tmp_path_factory):
    """gen_sponza_like at ~1/10 of its triangle count: deep BVH, every material."""
    d = tmp_path_factory.mktemp("atrium")
    subprocess.run([sys.executable, os.path.join(REPO, "scenes", "gen_sponza_like.py"), str(d), "--scale", "0.1",
                    "--name", "atrium"], check=True, capture_output=True)
    desc, params = rt.load_gltf(str(d / "atrium.gltf"), 48, 27, 2)
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.fixture(scope="module")
def hairball(rt, orc, tmp_path_factory):
    """gen_hairball at 30k triangles: thin random triangles, deep BVH, one quad light."""
    d = tmp_path_factory.mktemp("hairball")
    subprocess.run([sys.executable, os.path.join(REPO, "scenes", "gen_hairball.py"), str(d), "--tris", "30000",
                    "--name", "hb"], check=True, capture_output=True)
    desc, params = rt.load_gltf(str(d / "hb.gltf"), 40, 30, 3)
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


def test_hairball(hairball, segment_form):
    desc, params, g, o = hairball
    img, _, st = _compare(g, o, params)
    assert st["tri_tests"] > 0 and st["shaded_hits"] > 0
    # glTF positions are f32: the compact triangle layout exists and the resumable forms read it
    assert g.info()["layout_flags"] & 1
    assert g.info()["layout_flags"] & 4  # and its pair layout (every inner box is its children's union)
    want = {"resume": 2, "resume_eager": 2, "resume_c64": 1}.get(segment_form, 0)
    assert g.tuning()["compact"] == want


def test_room(room):
    desc, params, g, o = room
    img, _, st = _compare(g, o, params)
    assert st["light_hits"] > 0 and img.max() > 0


def test_room_deep_fov(room):
    desc, params, g, o = room
    _compare(g, o, params.replace(width=17, height=23, spp=3, ray_depth=20, fov=1.4, seed=11))


@pytest.mark.parametrize("waves", [3, 4])
def test_atrium(atrium, waves):
    desc, params, g, o = atrium
    img, _, st = _compare(g, o, params, waves=waves)
    assert st["tri_tests"] > 0 and img.max() > 0
    assert st["lane_steps"] <= st["wave_steps"]


def test_atrium_intersect_random(atrium):
    desc, params, g, o = atrium
    rng = np.random.default_rng(5)
    n = 50000
    orig = np.stack([rng.uniform(-11, 11, n), rng.uniform(0.1, 11, n), rng.uniform(-5.5, 5.5, n)], axis=1)
    d = rng.standard_normal((n, 3))
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh["prim"], oh["prim"])
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    assert (gh["prim"] >= 0).mean() > 0.75   # open-roofed atrium: upward rays may escape


@pytest.mark.parametrize("method,compact", [(0, -1), (1, -1), (1, 1), (1, 0)])
def test_atrium_intersect_device(atrium, rt, method, compact):
    """Deep triangle BVH through both device batch kernels (the persistent one on the
    compact layout's pair lines by default, on its 64-B nodes, and forced to the f64
    layout): the oracle's hits."""
    desc, params, g, o = atrium
    g.set_tuning(compact=compact)
    rng = np.random.default_rng(14)
    n = 30000
    pos = np.stack([rng.uniform(-10, 10, n), rng.uniform(0.5, 11, n), rng.uniform(-5, 5, n)], axis=1)
    rays = np.concatenate([pos, rng.standard_normal((n, 3))], axis=1)
    gh, oh = intersect_device(rt, g, rays, method), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))


def test_atrium_light_pdf_random(atrium):
    desc, params, g, o = atrium
    rng = np.random.default_rng(6)
    n = 20000
    pos = np.stack([rng.uniform(-10, 10, n), rng.uniform(0.5, 11, n), rng.uniform(-5, 5, n)], axis=1)
    d = rng.standard_normal((n, 3))
    d[:, 1] = np.abs(d[:, 1])
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pd = np.concatenate([pos, d], axis=1)
    gp, op = g.light_pdf(pd), o.light_pdf(pd)
    assert np.array_equal(gp, op)
    assert (gp > 0).sum() > 100
