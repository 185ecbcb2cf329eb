"""Quick perf probe: C2 workload at reduced spp (kernel time + counters)."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import load_package
rt = load_package()
import numpy as np
desc, params = rt.parse_scene(open(os.path.join(os.path.dirname(__file__), "..", "scenes", "cornell.txt")).read())
s = rt.Scene(desc)
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
p = params.replace(width=1920, height=1080, spp=spp)
img, _, st = s.generate_image(p, stats=True)
print(json.dumps(st))
for i in range(3):
    t = time.time(); img, _, st2 = s.generate_image(p); w = time.time() - t
    print(f"spp={spp} kernel_ms={st2['kernel_ms']:.1f} wall={w*1e3:.1f} Mseg/s={st['segments']/st2['kernel_ms']/1e3:.1f}")
bytes_ = 32*st['aabb_tests'] + 72*st['tri_tests'] + 80*st['shape_tests'] + 100*st['shaded_hits']
print("algo GB/s", bytes_/st2['kernel_ms']/1e6, "bytes/seg", bytes_/st['segments'])
