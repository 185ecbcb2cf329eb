#!/usr/bin/env python3
"""Experiment driver for tools/f32slab_sim.c (test infrastructure only): renders a
scene with the oracle's iterative form (mode 1) through the hooked traversal and
reports how often an f32 slab test with a proven error bound would leave a
decision of Node::intersection (bvh.rs:151-186) to the exact f64 test.

    python tools/f32slab_sim.py [--scene gltf:sponza_like|gltf:hairball_1m|cornell.txt] [-W 192 -H 108 --spp 4]
"""
import argparse
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
SO = os.path.join(REPO, "oracle", "build", "libf32sim.so")
NAMES = ["nodes", "kids", "miss_certain", "hit_certain", "undecided_hit", "visit_undecided", "order_undecided",
         "node_exact", "pops", "pop_undecided", "violations", "ineligible_rays", "viol_miss", "viol_hit", "viol_interval", "viol_pop"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="gltf:sponza_like")
    ap.add_argument("-W", type=int, default=192)
    ap.add_argument("-H", type=int, default=108)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--mode", type=int, default=0, help="bit 0 double-float origin, bit 1 pairwise hit test")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math",
                    "-I", os.path.join(REPO, "oracle"), "-shared", "-o", SO, os.path.join(HERE, "f32slab_sim.c"),
                    "-lm"], check=True)
    import ctypes as C
    import oracle as orc
    orc.LIB_PATHS["sim"] = SO
    from conftest import load_package
    rt = load_package()
    if args.scene.startswith("gltf:"):
        name = args.scene[5:]
        path = os.path.join(REPO, "scenes", "gen", name + ".gltf")
        if not os.path.exists(path):
            gen, extra = ("gen_hairball.py", ["--tris", "1000000"]) if name.startswith("hairball") else \
                ("gen_sponza_like.py", [])
            subprocess.run([sys.executable, os.path.join(REPO, "scenes", gen), os.path.join(REPO, "scenes", "gen"),
                            "--name", name, *extra], check=True, stdout=subprocess.DEVNULL)
        desc, params = rt.load_gltf(path, args.W, args.H, args.spp)
    else:
        desc, params = rt.parse_scene(open(os.path.join(REPO, "scenes", args.scene)).read())
        params = params.replace(width=args.W, height=args.H, spp=args.spp)
    osc = orc.OracleScene(desc, variant="sim")
    L = orc.lib("sim")
    L.sim_read.argtypes = [C.c_void_p]
    L.sim_read.restype = None
    L.sim_mode.argtypes = [C.c_int]
    L.sim_mode(args.mode)
    buf = np.zeros(len(NAMES), np.uint64)
    L.sim_read(buf.ctypes.data)
    _, _, st = osc.render(params, mode=1)
    L.sim_read(buf.ctypes.data)
    c = dict(zip(NAMES, (int(x) for x in buf)))
    print(f"mode {args.mode}: {args.scene} {args.W}x{args.H}x{args.spp}: segments {st['segments']}")
    for k, v in c.items():
        print(f"  {k:16s} {v}")
    n, k = max(c["nodes"], 1), max(c["kids"], 1)
    print(f"  per child test: certain miss {c['miss_certain'] / k:.4f}, certain hit {c['hit_certain'] / k:.4f}, "
          f"undecided {c['undecided_hit'] / k:.5f}")
    print(f"  per node visit: exact f64 needed {c['node_exact'] / n:.5f} (visit {c['visit_undecided'] / n:.5f}, "
          f"order {c['order_undecided'] / n:.5f})")
    print(f"  per pop: undecided {c['pop_undecided'] / max(c['pops'], 1):.5f}")
    print(f"  violations {c['violations']} (must be 0)")


if __name__ == "__main__":
    main()
