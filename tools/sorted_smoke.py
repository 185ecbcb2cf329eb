import os, sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
from conftest import load_package, load_oracle
rt = load_package(); orc = load_oracle()
desc, params = rt.parse_scene(open("scenes/cornell.txt").read())
s = rt.Scene(desc)
p = params.replace(width=40, height=24, spp=3)
s.set_tuning(sorted=1)
print("tuning", s.tuning(), flush=True)
t = time.time()
img, hits, st = s.generate_image(p, hit_ids=True, stats=True)
print("sorted ran", time.time() - t, st, flush=True)
_, cs = s.sample_chunks(p)
o_img, o_hits, o_st = orc.OracleScene(desc).render(p, mode=1, hit_ids=True, chunk_spp=cs)
print("hits equal", np.array_equal(hits, o_hits), "img equal", np.array_equal(img, o_img, equal_nan=True),
      "maxdiff", np.nanmax(np.abs(img - o_img)), flush=True)
for k in ("paths", "segments", "aabb_tests", "shape_tests", "shaded_hits", "light_queries", "light_hits"):
    print(k, st[k], o_st[k])
