"""Batch closest-hit throughput on a bench scene: one-thread-per-ray vs the
persistent traversal (rt_intersect_rays_async methods 0 and 1).

usage: [TRACE_COMPACT=-1|0|1] python tools/trace_bench.py WORKLOAD [N_RAYS]

Rays: the scene's camera rays at the workload's resolution (one jittered ray per
pixel), then diffuse bounce rays from their hits (cosine directions about the
shading normal, origin offset by EPSILON along the direction as raytrace.rs:33
does): the incoherent secondary rays that dominate a path-traced frame.
Checks that both methods return identical hits, then times each.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402
import bench  # noqa: E402

HIT_BYTES = 64


def camera_tans(c, W, H):
    """Camera::new (camera.rs:23-35), as api.cpp make_kparams computes it."""
    aspect = W / H
    if c.fov_axis == 1:  # fov given along y
        ty = np.tan(c.fov / 2.0)
        return ty * aspect, ty
    tx = np.tan(c.fov / 2.0)
    return tx, tx / aspect


def main():
    wl = sys.argv[1]
    n_max = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22
    rt = load_package()
    scene_file, W, H, spp, _ = bench.WORKLOADS[wl]
    desc, params = bench.load_workload(rt, scene_file, W, H, 1)
    scene = rt.Scene(desc)
    # TRACE_COMPACT: the persistent form's triangle layout (rt_tuning.compact: -1 auto = the
    # pair lines when the scene has them, 1 the 64-B compact nodes, 0 the f64 layout)
    scene.set_tuning(compact=int(os.environ.get("TRACE_COMPACT", "-1")))
    c = params.to_c()
    rng = np.random.default_rng(7)
    # Camera::fuzzy_ray (camera.rs:48-55), normalised as raytrace.rs:9 does
    ys, xs = np.mgrid[0:H, 0:W]
    fx = xs.ravel() + rng.random(W * H)
    fy = ys.ravel() + rng.random(W * H)
    tan_x, tan_y = camera_tans(c, W, H)
    x = (2.0 * fx / W - 1.0) * tan_x
    y = -(2.0 * fy / H - 1.0) * tan_y
    right, up, fwd = (np.array(getattr(c, k)[:]) for k in ("cam_right", "cam_up", "cam_forward"))
    d = x[:, None] * right + y[:, None] * up + fwd
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(np.array(c.cam_position[:]), d.shape)
    prim = np.concatenate([o, d], axis=1)
    hits = scene.intersect(prim)
    ok = hits["prim"] >= 0
    # diffuse bounce rays from the hits
    pos = prim[ok, :3] + prim[ok, 3:] * hits["t"][ok, None]
    n = hits["shading_normal"][ok]
    v = rng.random((len(n), 3)) * 2.0 - 1.0
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    dd = v + n
    dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    sec = np.concatenate([pos + dd * 1e-9, dd], axis=1)
    sec = np.ascontiguousarray(np.tile(sec, (int(np.ceil(n_max / len(sec))), 1))[:n_max])
    out = {"workload": wl, "primary_hit_frac": float(ok.mean())}
    dev = torch.device("cuda:0")
    for name, rays in (("primary", prim), ("bounce", sec)):
        d_rays = torch.from_numpy(np.ascontiguousarray(rays)).to(dev)
        nr = len(rays)
        res = {}
        ref = None
        for method in (0, 1):
            d_hits = torch.zeros(nr * HIT_BYTES // 8, dtype=torch.float64, device=dev)
            s = torch.cuda.current_stream().cuda_stream
            scene.intersect_async(d_rays.data_ptr(), nr, d_hits.data_ptr(), method, s)
            torch.cuda.synchronize()
            h = d_hits.cpu().numpy().view(np.uint8)
            if ref is None:
                ref = h
            else:
                assert np.array_equal(ref, h), f"{name}: methods differ"
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                scene.intersect_async(d_rays.data_ptr(), nr, d_hits.data_ptr(), method, s)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[f"method{method}_ms"] = min(ts)
            res[f"method{method}_Grays_s"] = nr / min(ts) / 1e6
        res["n"] = nr
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
