"""GPU parity at BASELINE.json configs[3] (C4): the synthetic atrium at
3840x2160, 1024 spp, depth 8 — the frame the 8-GPU scaling is quoted on — run
whole on one GPU as the 8 rank shares of the multi-GPU partition
(rt_render_tiles_async rank 0..7, 16x16 tiles round-robin), then
the root's unpack, as the 8-GPU bench does after its single gather.

Bar: the 8-share frame is bit-identical to the one-launch rt_render frame (the
RNG is keyed by the global pixel and sample, the chunking by the frame alone),
two full rows match the oracle's iterative form bit for bit with the device's
sample chunking (main.rs:94-111 restated, oracle rows=), and the fused device
epilogue gives the host's PPM bytes exactly."""
import os
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, REPO)


def test_c4_frame_as_eight_rank_shares(rt, orc):
    import bench
    scene_file, W, H, spp, _ = bench.WORKLOADS["C4"]
    desc, params = bench.load_workload(rt, scene_file, W, H, spp)
    assert (params.width, params.height, params.spp, params.ray_depth) == (3840, 2160, 1024, 8)
    scene = rt.Scene(desc)
    chunks, chunk_spp = scene.sample_chunks(params)
    assert (chunks, chunk_spp) == (16, 64)  # the 4-GiB partial-sum budget (render.h sample_chunks)

    world = 8
    per = scene.tiles_per_rank(params, world)
    gathered = torch.empty((world, per, 256, 3), dtype=torch.float64, device="cuda")
    for r in range(world):
        scene.render_tiles_async(params, r, world, gathered[r].data_ptr())
    img = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    rt.unpack_tiles_async(params, world, gathered.data_ptr(), img.data_ptr())
    byts = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    rt.unpack_tiles_bytes_async(params, world, gathered.data_ptr(), byts.data_ptr())
    torch.cuda.synchronize()
    shares = img.cpu().numpy()
    del gathered, img

    ref, _, st = scene.generate_image(params, stats=True)
    assert np.array_equal(shares, ref), f"max |d| {np.abs(shares - ref).max()}"
    assert np.isfinite(ref).all() and (ref >= 0).all() and ref.max() > 0
    assert st["paths"] == W * H * spp

    host = orc.ppm_bytes(orc.tonemap_gamma(ref.reshape(-1, 3))).reshape(H, W, 3)
    assert np.array_equal(byts.cpu().numpy(), host)

    threads, _ = bench.cpu_share()
    osc = orc.OracleScene(desc)
    for row in (3, 1400):
        o_img, _, o_st = osc.render(params, mode=1, threads=threads, rows=(row, row + 1), chunk_spp=chunk_spp)
        assert np.array_equal(ref[row], o_img[row]), f"row {row}: max |d| {np.abs(ref[row] - o_img[row]).max()}"
        assert o_st["paths"] == W * spp
