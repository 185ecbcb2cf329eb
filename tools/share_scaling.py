"""Per-rank render time of a strong-scaled frame on ONE GPU: rank r's tile share
of an N-way partition (rt_render_tiles_async), timed alone with HIP events, for
each N and EVERY rank (median of 3 timed runs after a warm one).  The slowest
share x N over the N=1 frame is the render-side strong-scaling efficiency the
N-GPU bench can reach (no gather or launch cost).
usage: python tools/share_scaling.py [WORKLOAD] [SPP] [N ...]
RT_SHARE_TUNE="chunk_spp=4,..." forces rt_tuning fields (Scene.set_tuning)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (one HIP runtime per process)

import bench  # noqa: E402
from conftest import load_package  # noqa: E402

rt = load_package()
wl = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene_file, W, H, spp, depth = bench.WORKLOADS[wl]
if len(sys.argv) > 2:
    spp = int(sys.argv[2])
ns = [int(x) for x in sys.argv[3:]] or [1, 2, 4, 8]
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
if depth:
    params = params.replace(ray_depth=depth)
scene = rt.Scene(desc)
tune = {k: int(v) for k, v in (kv.split("=", 1) for kv in os.environ.get("RT_SHARE_TUNE", "").split(",") if kv)}
if tune:
    scene.set_tuning(**tune)
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
out = {"workload": wl, "spp": spp, "chunks": scene.sample_chunks(params)[0], "tuning": scene.tuning(), "ms": {}}
t1 = None
for n in ns:
    per = scene.tiles_per_rank(params, n)
    tiles = torch.empty((per, 256, 3), dtype=torch.float64, device=dev)
    times = []
    runs = []
    for rank in range(n):
        scene.render_tiles_async(params, rank, n, tiles.data_ptr(), stream.cuda_stream)  # warm
        ms = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            scene.render_tiles_async(params, rank, n, tiles.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        runs.append(ms)
        times.append(float(sorted(ms)[1]))  # median of 3
    worst = max(times)
    if n == 1:
        t1 = worst
    out["ms"][n] = {"per_rank_median": times, "per_rank_runs": runs, "worst": worst,
                    "efficiency": (t1 / (n * worst)) if t1 else None}
    print(json.dumps({n: out["ms"][n]}), flush=True)
print(json.dumps(out))
