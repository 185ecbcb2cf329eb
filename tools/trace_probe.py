"""Experiment: the traversal-only probe kernel (render.hip trace_tri_kernel, a
-DRT_WF_PROBE build, method 2) against the persistent batch trace (method 1) on a
glTF workload's diffuse bounce rays: same closest triangle and t, and the rate.
usage: RT_AMD_LIB=<probe build> python tools/trace_probe.py WORKLOAD [N_RAYS]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from conftest import load_package  # noqa: E402
import bench  # noqa: E402
import trace_bench as tb  # noqa: E402


def main():
    wl = sys.argv[1]
    n_max = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22
    rt = load_package()
    scene_file, W, H, _, _ = bench.WORKLOADS[wl]
    desc, params = bench.load_workload(rt, scene_file, W, H, 1)
    scene = rt.Scene(desc)
    c = params.to_c()
    rng = np.random.default_rng(7)
    ys, xs = np.mgrid[0:H, 0:W]
    fx = xs.ravel() + rng.random(W * H)
    fy = ys.ravel() + rng.random(W * H)
    tan_x, tan_y = tb.camera_tans(c, W, H)
    x = (2.0 * fx / W - 1.0) * tan_x
    y = -(2.0 * fy / H - 1.0) * tan_y
    right, up, fwd = (np.array(getattr(c, k)[:]) for k in ("cam_right", "cam_up", "cam_forward"))
    d = x[:, None] * right + y[:, None] * up + fwd
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(np.array(c.cam_position[:]), d.shape)
    prim = np.concatenate([o, d], axis=1)
    hits = scene.intersect(prim)
    ok = hits["prim"] >= 0
    pos = prim[ok, :3] + prim[ok, 3:] * hits["t"][ok, None]
    n = hits["shading_normal"][ok]
    v = rng.random((len(n), 3)) * 2.0 - 1.0
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    dd = v + n
    dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    sec = np.concatenate([pos + dd * 1e-9, dd], axis=1)
    sec = np.ascontiguousarray(np.tile(sec, (int(np.ceil(n_max / len(sec))), 1))[:n_max])
    dev = torch.device("cuda:0")
    out = {"workload": wl, "lib": os.environ.get("RT_AMD_LIB", "")}
    for name, rays in (("primary", prim), ("bounce", sec)):
        d_rays = torch.from_numpy(np.ascontiguousarray(rays)).to(dev)
        nr = len(rays)
        res, got = {}, {}
        for method in (1, 2):
            d_hits = torch.zeros(nr * tb.HIT_BYTES // 8, dtype=torch.float64, device=dev)
            s = torch.cuda.current_stream().cuda_stream
            scene.intersect_async(d_rays.data_ptr(), nr, d_hits.data_ptr(), method, s)
            torch.cuda.synchronize()
            h = d_hits.cpu().numpy().view(np.uint8).reshape(nr, tb.HIT_BYTES)
            got[method] = (h[:, 0:8].copy().view(np.float64).ravel(), h[:, 60:64].copy().view(np.int32).ravel())
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
        t1, p1 = got[1]
        t2, p2 = got[2]
        hit = p1 >= 0
        res["same_prim"] = bool(np.array_equal(p1, p2))
        res["same_t"] = bool(np.array_equal(t1[hit], t2[hit]))
        res["n"] = nr
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
