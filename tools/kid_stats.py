"""Child-box outcomes of the closest-hit traversal's inner-node visits (raw stats
words 11..13: none / one / both of the two child slab tests hit), per workload,
from the stats instance.  DESIGN.md §4 uses them to price a certain-miss prefilter.

    python tools/kid_stats.py C3 64 [C5 16 ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import torch  # noqa: F401,E402  (one HIP runtime per process)
from conftest import load_package  # noqa: E402
import bench  # noqa: E402

rt = load_package()
args = sys.argv[1:]
for wl, spp in zip(args[::2], args[1::2]):
    scene_file, W, H, _, depth = bench.WORKLOADS[wl]
    desc, params = bench.load_workload(rt, scene_file, W, H, int(spp))
    s = rt.Scene(desc)
    _, _, st = s.generate_image(params, stats=True)
    raw = [int(x) for x in s.read_raw_stats(14)]
    none, one, both = raw[11:14]
    visits = none + one + both
    tests = 2 * visits
    out = {"workload": wl, "spp": int(spp), "tuning": s.tuning(), "segments": st["segments"],
           "aabb_tests": st["aabb_tests"], "inner_visits": visits, "kids_none": none, "kids_one": one,
           "kids_both": both, "child_tests": tests, "child_miss_frac": (2 * none + one) / max(tests, 1),
           "visits_per_segment": visits / max(st["segments"], 1),
           "frac_visits_none": none / max(visits, 1), "frac_visits_one": one / max(visits, 1),
           "frac_visits_both": both / max(visits, 1)}
    print(json.dumps(out), flush=True)
