"""Lane utilisation of the path-regeneration loop vs sample-run length.
usage: python tools/lane_util.py WORKLOAD [SPP] [chunk_spp ...]
Per chunk length (rt_tuning.chunk_spp): kernel ms of a plain render and
lane_steps / wave_steps from a stats render (fraction of SIMD lane-steps doing
path work; the rest is lanes idling at the end of their wave's run)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process)
import bench  # noqa: E402
from conftest import load_package  # noqa: E402

rt = load_package()
wl = sys.argv[1]
scene_file, W, H, spp, depth = bench.WORKLOADS[wl]
if len(sys.argv) > 2:
    spp = int(sys.argv[2])
chunks = [int(x) for x in sys.argv[3:]] or [spp, 64, 32, 16, 8]
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
scene = rt.Scene(desc)
for cs in chunks:
    scene.set_tuning(chunk_spp=cs)
    _, _, st = scene.generate_image(params, stats=True)
    ms = min(scene.generate_image(params)[2]["kernel_ms"] for _ in range(2))
    print(json.dumps({"workload": wl, "spp": spp, "chunk_spp": cs, "chunks": scene.sample_chunks(params)[0],
                      "kernel_ms": ms, "Mseg_s": st["segments"] / ms / 1e3,
                      "lane_util": st["lane_steps"] / max(1, st["wave_steps"]), "segments": st["segments"]}),
          flush=True)
