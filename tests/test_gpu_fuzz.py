"""GPU parity on seeded random scenes (tests/fuzz_scenes.py): every primitive kind,
material and light kind in random mixes, grid-exact and arbitrary coordinates, meshes
with shared vertices and exact duplicate triangles (ties), boxes resting on planes,
flat boxes, degenerate triangles and non-normalised rotations.

Per seed: the rendered frame in every path-kernel form (hit ids, radiance and work
counters bit-exact vs the oracle, test_gpu_parity._compare), and batch intersection /
light-pdf queries on random rays and on rays aimed exactly at mesh vertices and edge
midpoints, where neighbouring triangles tie.
"""
import numpy as np
import pytest

from fuzz_scenes import random_scene
from test_gpu_parity import FORM, _compare, intersect_device

pytestmark = pytest.mark.gpu

N_SEEDS = 160
FORMS = {
    "fused": {},
    "resume": dict(resume=1),
    "resume_eager": dict(resume=1, suspend_lanes=64, leaf_lanes=1),
    "resume_f64": dict(resume=1, compact=0),
    "general": dict(kinds=3),
}


def _scenes(rt, orc, seed, **kw):
    desc, params = rt.parse_scene(random_scene(seed, **kw))
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.mark.parametrize("seed", range(N_SEEDS))
def test_fuzz_render(rt, orc, seed):
    desc, params, g, o = _scenes(rt, orc, seed, spp=4, depth=None if seed % 4 else 12)
    for name, f in FORMS.items():
        FORM.clear()
        FORM.update(f)
        try:
            _compare(g, o, params)
        finally:
            FORM.clear()


# the compact layout's pair lines (two BVH levels per line, rt_layout.h kPairFloats) on
# triangle-only grid scenes: ties (duplicates, shared edges and vertices, coplanar tiles),
# flat leaf boxes and degenerate triangles through the 4-wave resumable kernel, which
# reads the pair lines by default; the 64-B compact nodes and the eager form beside it.
# The lazy form (no suspension, leaves tested only once every live lane waits at one)
# deals up to 256 records per leaf step: render.hip leaf_coop's multi-round case.
PAIR_FORMS = {
    "pair": dict(resume=1, waves=4),
    "pair_eager": dict(resume=1, waves=4, suspend_lanes=64, leaf_lanes=1),
    "pair_lazy": dict(resume=1, waves=4, suspend_lanes=1, leaf_lanes=64),
    "compact64": dict(resume=1, waves=4, compact=1),
}


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_pair_layout(rt, orc, seed):
    desc, params, g, o = _scenes(rt, orc, 5000 + seed, spp=4, depth=None if seed % 3 else 10, tri_only=True)
    assert g.info()["layout_flags"] & 0x5 == 0x5  # the compact layout and its pair lines
    for name, f in PAIR_FORMS.items():
        FORM.clear()
        FORM.update(f)
        try:
            _compare(g, o, params)
            assert g.tuning()["compact"] == (1 if name == "compact64" else 2)
        finally:
            FORM.clear()


def _aimed_rays(desc, rng, n):
    """Rays through mesh vertices and edge midpoints, from grid origins along grid
    directions (axis-parallel ones included): exact on a 1/16 grid, so each ray meets
    the point exactly and the triangles sharing it tie."""
    tv = np.asarray(desc.tri_vertices, np.float64).reshape(-1, 3, 3)
    if len(tv) == 0:
        return np.zeros((0, 6))
    pts = np.concatenate([tv.reshape(-1, 3), (tv + np.roll(tv, 1, axis=1)).reshape(-1, 3) / 2])
    p = pts[rng.integers(0, len(pts), n)]
    d = rng.choice([-1.0, -0.5, 0.0, 0.5, 1.0], (n, 3))
    d[np.all(d == 0, axis=1)] = [0.0, -1.0, 0.0]
    return np.concatenate([p - 2.0 * d, d], axis=1)


@pytest.mark.parametrize("seed", range(0, N_SEEDS, 2))
def test_fuzz_queries(rt, orc, seed):
    desc, params, g, o = _scenes(rt, orc, seed)
    rng = np.random.default_rng(1000 + seed)
    n = 6000
    rays = np.concatenate([rng.uniform(-1.5, 1.5, (n, 3)), rng.standard_normal((n, 3))], axis=1)
    rays = np.concatenate([rays, _aimed_rays(desc, rng, n)])
    oh = o.intersect(rays)
    assert np.array_equal(g.intersect(rays).view(np.uint8), oh.view(np.uint8))
    for method in (0, 1):
        assert np.array_equal(intersect_device(rt, g, rays, method).view(np.uint8), oh.view(np.uint8)), method
    d = rays[:, 3:] / np.linalg.norm(rays[:, 3:], axis=1, keepdims=True)
    pd = np.concatenate([rays[:, :3], d], axis=1)
    assert np.array_equal(g.light_pdf(pd), o.light_pdf(pd), equal_nan=True)
