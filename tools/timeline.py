"""Wave timeline of one path-kernel launch (the stats instance's raw words 52..59,
render.hip path_kernel, s_memrealtime at 100 MHz): when the waves start, when each
first finds the wave-tile queue drained, when they exit.  The drain phase (last exit
minus earliest drain) is the per-launch tail a tile share pays however small it is.
    python tools/timeline.py [WORKLOAD] [SPP] [N ...]   (rank 0's share of an N-way partition)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import torch  # noqa: E402  (one HIP runtime per process)
import bench  # noqa: E402
from conftest import load_package  # noqa: E402

TICK_MS = 1e-5  # s_memrealtime: 100 MHz
rt = load_package()
wl = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene_file, W, H, spp, depth = bench.WORKLOADS[wl]
if len(sys.argv) > 2:
    spp = int(sys.argv[2])
ns = [int(x) for x in sys.argv[3:]] or [1, 8]
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
scene = rt.Scene(desc)
tune = {k: int(v) for k, v in (kv.split("=", 1) for kv in os.environ.get("RT_SHARE_TUNE", "").split(",") if kv)}
if tune:
    scene.set_tuning(**tune)
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
M = (1 << 64) - 1
for n in ns:
    tiles = torch.empty((scene.tiles_per_rank(params, n), 256, 3), dtype=torch.float64, device=dev)
    for rep in range(2):
        scene.read_stats(reset=True)
        scene.render_tiles_async(params, 0, n, tiles.data_ptr(), stream.cuda_stream, stats=True)
        torch.cuda.synchronize()
        w = [int(x) for x in scene.read_raw_stats(64)[52:60]]
        t0, te, td0, td1, dsum, dmax, busy, waves = M - w[0], w[1], M - w[2], w[3], w[4], w[5], w[6], w[7]
        span = (te - t0) * TICK_MS
        print(f"N={n} rep {rep}: waves {waves}, span {span:.3f} ms; first drain at {(td0 - t0) * TICK_MS:.3f} ms, "
              f"last drain at {(td1 - t0) * TICK_MS:.3f} ms; drain phase {(te - td0) * TICK_MS:.3f} ms "
              f"({(te - td0) / max(te - t0, 1):.3f} of the span); per wave drain-to-exit mean "
              f"{dsum / max(waves, 1) * TICK_MS:.3f} max {dmax * TICK_MS:.3f} ms; mean wave busy "
              f"{busy / max(waves, 1) * TICK_MS:.3f} ms", flush=True)
