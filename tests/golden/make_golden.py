"""Writes the self-generated golden fixtures tests/golden/<name>.npz.

The reference publishes no images and its RNG is OS-seeded (main.rs:95), so
end-to-end goldens come from this repo's own oracle (oracle/oracle.c, the C
restatement of the reference) on the committed scenes with a fixed Philox
seed.  They pin the oracle against regressions and give the GPU tests a
second, stored comparison point.  Regenerate only when the estimator changes
on purpose:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))

CASES = {
    # name: (scene, overrides)
    "cornell_24x16_4spp": ("cornell.txt", dict(width=24, height=16, spp=4)),
    "kitchen_sink": ("kitchen_sink.txt", {}),
    "kitchen_sink_deep": ("kitchen_sink.txt", dict(width=12, height=10, spp=3, ray_depth=24, seed=99)),
}


def render_case(name):
    from conftest import load_oracle, load_package
    rt, orc = load_package(), load_oracle()
    scene, over = CASES[name]
    with open(os.path.join(REPO, "scenes", scene)) as f:
        desc, params = rt.parse_scene(f.read())
    params = params.replace(**over)
    img, hits, st = orc.OracleScene(desc).render(params, mode=1, hit_ids=True)
    stats = np.array([st[k] for k in ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests",
                                      "shaded_hits", "light_queries", "light_hits")], np.uint64)
    return params, img, hits, stats


if __name__ == "__main__":
    for name in CASES:
        params, img, hits, stats = render_case(name)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), image=img, hit_ids=hits, stats=stats,
                            params=np.array([params.width, params.height, params.spp, params.ray_depth,
                                             params.seed], np.uint64))
        print(name, img.shape, hits.shape, stats)
