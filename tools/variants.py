"""Time alternate builds of librt_amd.so on the C2 workload at reduced spp.
usage: python tools/variants.py SPP lib1.so lib2.so ...  (each in its own process)"""
import json, os, subprocess, sys
HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r'''
import os, sys, time, json
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
from conftest import load_package
rt = load_package()
desc, params = rt.parse_scene(open(os.path.join(sys.argv[1], "scenes", "cornell.txt")).read())
s = rt.Scene(desc)
p = params.replace(width=1920, height=1080, spp=int(sys.argv[2]))
_, _, st = s.generate_image(p, stats=True)
ks = []
for i in range(3):
    _, _, st2 = s.generate_image(p)
    ks.append(st2["kernel_ms"])
print(json.dumps({"lib": os.environ["RT_AMD_LIB"], "kernel_ms": ks, "Mseg_s": st["segments"] / min(ks) / 1e3,
                  "segments": st["segments"]}))
'''
spp = sys.argv[1]
for lib in sys.argv[2:]:
    env = dict(os.environ, RT_AMD_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.dirname(HERE), spp], env=env, capture_output=True,
                       text=True, timeout=300)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
