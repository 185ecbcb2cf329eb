"""Time alternate builds of librt_amd.so on a bench workload at reduced spp.
usage: python tools/variants.py WORKLOAD SPP lib1.so lib2.so[@VAR=val,VAR2=val] ...   (each in its own process)
WORKLOAD is a bench.py workload name (C1, C2, C3, ...); `@field=val,...` forces rt_tuning fields
(e.g. waves=3,resume=0,suspend_lanes=32) for that run (Scene.set_tuning)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r'''
import os, sys, json
root = sys.argv[1]
sys.path.insert(0, os.path.join(root, "tests")); sys.path.insert(0, root)
import torch  # one HIP runtime per process
from conftest import load_package
import bench
rt = load_package()
scene_file, W, H, spp, depth = bench.WORKLOADS[sys.argv[2]]
desc, params = bench.load_workload(rt, scene_file, W, H, int(sys.argv[3]))
if depth:
    params = params.replace(ray_depth=depth)
s = rt.Scene(desc)
tune = {k: int(v) for k, v in (kv.split("=", 1) for kv in os.environ.get("RT_VARIANT_ENV", "").split(",") if kv)}
s.set_tuning(**tune)
import hashlib
_, _, st = s.generate_image(params, stats=True)
ks = []
for i in range(3):
    img, _, st2 = s.generate_image(params)
    ks.append(st2["kernel_ms"])
print(json.dumps({"lib": os.environ["RT_AMD_LIB"], "tuning": s.tuning(), "workload": sys.argv[2], "spp": params.spp, "kernel_ms": ks,
                  "Mseg_s": st["segments"] / min(ks) / 1e3, "segments": st["segments"],
                  "image_sha256": hashlib.sha256(img.tobytes()).hexdigest()[:16]}))
'''
wl, spp = sys.argv[1], sys.argv[2]
rc = 0
for arg in sys.argv[3:]:
    lib, _, over = arg.partition("@")
    env = dict(os.environ, RT_AMD_LIB=os.path.abspath(lib), RT_VARIANT_ENV=over)
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.dirname(HERE), wl, spp], env=env, capture_output=True,
                       text=True, timeout=600)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
    rc = rc or r.returncode
sys.exit(rc)
