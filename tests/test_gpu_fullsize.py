"""GPU parity at BASELINE.json's full sizes: the C2 and C3 frames (1920x1080,
256 spp) rendered whole on the device, then a band of rows checked bit for bit
against the oracle's iterative form with the device's sample chunking.

The RNG is keyed by (pixel, sample), so any row of the full frame can be
re-rendered on its own by the oracle (`rows=`) and must match exactly: the
same image at the size the bench measures.  Frame-level properties are checked
too: every pixel finite and non-negative, one path per (pixel, sample), and
(C3) the identical frame and counters from the other segment form.
"""
import os
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

sys.path.insert(0, REPO)


def _workload(rt, name):
    import bench
    scene_file, W, H, spp, depth = bench.WORKLOADS[name]
    desc, params = bench.load_workload(rt, scene_file, W, H, spp)
    if depth:
        params = params.replace(ray_depth=depth)
    return desc, params


def _threads():
    return min(16, os.cpu_count() or 1)


@pytest.mark.parametrize("name,rows", [("C2", [0, 540, 1079]), ("C3", [1, 600])])
def test_full_frame_rows_match_oracle(rt, orc, name, rows):
    desc, params = _workload(rt, name)
    scene = rt.Scene(desc)
    img, _, st = scene.generate_image(params, stats=True)
    # the timed product kernel (no stats) renders the same bits
    assert np.array_equal(scene.generate_image(params)[0], img)
    assert img.shape == (params.height, params.width, 3)
    assert np.isfinite(img).all() and (img >= 0).all()
    assert st["paths"] == params.width * params.height * params.spp
    _, chunk_spp = rt.sample_chunks(params)
    osc = orc.OracleScene(desc)
    for r in rows:
        o_img, _, o_st = osc.render(params, mode=1, threads=_threads(), rows=(r, r + 1), chunk_spp=chunk_spp)
        assert np.array_equal(img[r], o_img[r]), f"{name} row {r}: max |d| {np.abs(img[r] - o_img[r]).max()}"
        assert o_st["paths"] == params.width * params.spp
    if name == "C3":
        # the other segment form renders the identical frame (C3 picks the resumable one)
        # C3 runs the resumable kernel on the compact triangle layout's pair lines; its 64-B
        # nodes, the f64 layout in the same kernel and the fused form render the identical
        # frame and counters
        assert scene.tuning()["resume"] == 1 and scene.tuning()["compact"] == 2  # pair layout
        # the compact layouts' cooperative leaf step runs with its own thresholds (render.h
        # kSuspendCoopCached / kLeafCoopCached); the f64 layout's serial leaf loop (and the
        # fused form, which does not use them) reports 32 / 32
        lanes = lambda: (scene.tuning()["suspend_lanes"], scene.tuning()["leaf_lanes"])
        assert lanes() == (24, 16)
        for tune in (dict(compact=1), dict(compact=0), dict(resume=0)):
            scene.set_tuning(**tune)
            assert lanes() == ((24, 16) if tune == dict(compact=1) else (32, 32)), tune  # api.cpp path_compact
            img2, _, st2 = scene.generate_image(params, stats=True)
            assert np.array_equal(img, img2), tune
            assert st2["segments"] == st["segments"] and st2["tri_tests"] == st["tri_tests"], tune
