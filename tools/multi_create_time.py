"""rt_multi_create of a bench workload's scene with N replicas (one GPU: a device listed N
times, RT_MULTI_PEER): the host build once, devices[0] from the host, the replicas filled
device to device from devices[0]; prints each replica's upload_ms beside a plain
rt_scene_create (what one replica's own host upload costs).
    python tools/multi_create_time.py [WORKLOAD] [N]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import torch  # noqa: E402,F401  (one HIP runtime per process)
import bench  # noqa: E402
from conftest import load_package  # noqa: E402

rt = load_package()
wl = sys.argv[1] if len(sys.argv) > 1 else "C5"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
scene_file, W, H, spp, _ = bench.WORKLOADS[wl]
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
t = time.perf_counter()
s = rt.Scene(desc)
one = time.perf_counter() - t
i0 = s.info()
print(f"{wl}: rt_scene_create {one * 1e3:.0f} ms (build {i0['build_ms']:.0f} ms, host upload {i0['upload_ms']:.1f} ms, "
      f"{i0['device_bytes'] / 1e9:.3f} GB)", flush=True)
del s
t = time.perf_counter()
m = rt.MultiScene(desc, [0] * n, peer=True)
tot = time.perf_counter() - t
for i in range(n):
    inf = m.scene_info(i)
    print(f"  replica {i}: upload_ms {inf['upload_ms']:.1f} ({'host' if i == 0 else 'device-to-device fill'}), "
          f"{inf['device_bytes'] / 1e9:.3f} GB", flush=True)
print(f"rt_multi_create x{n}: {tot * 1e3:.0f} ms", flush=True)
