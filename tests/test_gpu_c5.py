"""GPU parity at BASELINE.json configs[4] (C5): the 10M-triangle hairball
(scenes/gen_hairball.py) at 1920x1080, 64 spp, depth 8 (gltf/scene_builder.rs:16)
— the deep, HBM-streamed BVH (the triangle BVH and its records, ~0.7 GB in the
compact layout, are past the 256-MiB Infinity Cache).

Bar: the host picks the streamed-BVH form (suspend 48, leaf batch 12 with the
cooperative leaf step, compact layout: api.cpp bvh_streamed), the product instance's full frame is bit-identical
to the stats instance's, and two full rows match the oracle's iterative form bit
for bit with the device's sample chunking (bvh.rs:151-186 traversal in the
reference's visit order; main.rs:94-111 restated, oracle rows=)."""
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
sys.path.insert(0, REPO)


def test_c5_full_frame(rt, orc):
    import bench
    scene_file, W, H, spp, _ = bench.WORKLOADS["C5"]
    desc, params = bench.load_workload(rt, scene_file, W, H, spp)
    assert (params.width, params.height, params.spp, params.ray_depth) == (1920, 1080, 64, 8)
    assert len(desc.tri_material) >= 10_000_000
    scene = rt.Scene(desc)
    info = scene.info()
    assert info["layout_flags"] & 1  # f32 glTF positions: the compact triangle layout exists
    assert info["layout_flags"] & 4  # ... with its pair layout, which the resumable kernel reads
    t = scene.tuning()
    assert (t["waves"], t["resume"], t["kinds"], t["compact"]) == (4, 1, 2, 2)
    assert (t["suspend_lanes"], t["leaf_lanes"]) == (48, 12)  # streamed-BVH thresholds (render.h kLeafCoop*)
    chunks, chunk_spp = scene.sample_chunks(params)

    img, _, st = scene.generate_image(params, stats=True)     # stats instance
    prod, _, _ = scene.generate_image(params)                 # the timed (product) instance
    assert np.array_equal(prod, img), f"product vs stats instance: max |d| {np.abs(prod - img).max()}"
    assert np.isfinite(img).all() and (img >= 0).all() and img.max() > 0
    assert st["paths"] == W * H * spp and st["tri_tests"] > st["segments"]
    # the compact layout's 64-B nodes (one BVH level per line) give the same frame and work
    scene.set_tuning(compact=1)
    img1, _, st1 = scene.generate_image(params, stats=True)
    assert np.array_equal(img1, img)
    for k in ("paths", "segments", "aabb_tests", "tri_tests", "shaded_hits", "light_queries", "light_hits"):
        assert st1[k] == st[k], k
    scene.set_tuning()

    threads, _ = bench.cpu_share()
    osc = orc.OracleScene(desc)  # the restated reference builder, once
    for row in (300, 540):
        o_img, _, o_st = osc.render(params, mode=1, threads=threads, rows=(row, row + 1), chunk_spp=chunk_spp)
        assert np.array_equal(img[row], o_img[row]), f"row {row}: max |d| {np.abs(img[row] - o_img[row]).max()}"
        assert o_st["paths"] == W * spp and o_img[row].max() > 0
