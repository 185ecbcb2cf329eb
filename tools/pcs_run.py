"""One C2 frame at reduced spp, for PC sampling under rocprofv3 (tools/pcs_summary.py).
usage: python tools/pcs_run.py [WORKLOAD] [SPP]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process)
import bench  # noqa: E402
from conftest import load_package  # noqa: E402

rt = load_package()
wl = sys.argv[1] if len(sys.argv) > 1 else "C2"
scene_file, W, H, spp, depth = bench.WORKLOADS[wl]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
if depth:
    params = params.replace(ray_depth=depth)
s = rt.Scene(desc)
img, _, st = s.generate_image(params)
print(wl, spp, st["kernel_ms"], flush=True)
