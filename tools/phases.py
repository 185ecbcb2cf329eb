"""Wave-cycle breakdown of the path kernel by code region (needs a -DRT_PHASES
build: make -C cpu-raytracing-rt_amd/csrc OUT=../ph_build EXTRA=-DRT_PHASES,
then RT_AMD_LIB=.../ph_build/librt_amd.so).
usage: python tools/phases.py WORKLOAD [SPP]
Each region's s_memtime delta is added once per wave that executes it, so the
shares are of wave-time (all waves summed), the quantity that divergence and
stalls inflate.  segment = intersect + light sample + light pdf + shading."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process)
import bench  # noqa: E402
from conftest import load_package  # noqa: E402

NAMES = ["assign", "intersect", "light_sample", "light_pdf", "segment", "commit", "tile",
         "trav_wave_iters", "trav_lane_iters", "leaf_wave_trips", "leaf_lane_tests",
         "rng_wave_refills", "rng_lane_refills",
         "w_intersect", "w_light_sample", "w_light_pdf", "w_segment", "w_commit",
         "isect_planes", "isect_boxes", "isect_ellipsoids", "isect_triangles", "isect_materialise",
         "inner_wave_iters", "inner_lane_iters", "live_lane_iters", "idle_window_lanes", "idle_drained_lanes",
         "push_lane", "push_global", "pop_global", "leaf_cycles", "inner_cycles", "pop_cycles", "step_cycles",
         "inner_uniform_waves"]
rt = load_package()
wl = sys.argv[1]
scene_file, W, H, spp, depth = bench.WORKLOADS[wl]
if len(sys.argv) > 2:
    spp = int(sys.argv[2])
desc, params = bench.load_workload(rt, scene_file, W, H, spp)
scene = rt.Scene(desc)
_, _, st = scene.generate_image(params, stats=True)
raw = scene.read_raw_stats(64)
ph = {n: int(raw[16 + i]) for i, n in enumerate(NAMES)}
tile = max(ph["tile"], 1)
shading = ph["segment"] - ph["intersect"] - ph["light_sample"] - ph["light_pdf"]
share = {k: ph[k] / tile for k in ("assign", "intersect", "light_sample", "light_pdf", "commit")}
share["shading_rest"] = shading / tile
share["loop_other"] = 1.0 - ph["assign"] / tile - ph["segment"] / tile - ph["commit"] / tile
for k in ("isect_planes", "isect_boxes", "isect_ellipsoids", "isect_triangles", "isect_materialise"):
    share[k] = ph[k] / tile
for k in ("leaf", "inner", "pop", "step"):  # inside the resumable walk's steps (part of the walks above)
    share["trav_" + k] = ph[k + "_cycles"] / tile
print(json.dumps({"workload": wl, "spp": spp, "segments": st["segments"],
                  "lane_util": st["lane_steps"] / max(1, st["wave_steps"]),
                  "traversal_loop_util": ph["trav_lane_iters"] / max(1, 64 * ph["trav_wave_iters"]),
                  "live_lane_frac": ph["live_lane_iters"] / max(1, 64 * ph["trav_wave_iters"]),
                  "inner_node_util": ph["inner_lane_iters"] / max(1, 64 * ph["inner_wave_iters"]),
                  "inner_iter_share": ph["inner_wave_iters"] / max(1, ph["trav_wave_iters"]),
                  "inner_uniform_share": ph["inner_uniform_waves"] / max(1, ph["inner_wave_iters"]),
                  "leaf_loop_util": ph["leaf_lane_tests"] / max(1, 64 * ph["leaf_wave_trips"]),
                  "rng_refill_util": ph["rng_lane_refills"] / max(1, 64 * ph["rng_wave_refills"]),
                  "rng_wave_refills_per_segment": ph["rng_wave_refills"] * 64 / max(1, st["segments"]),
                  # lanes without a path per path-loop trip: held by the commit window / queue drained
                  "idle_window_frac": ph["idle_window_lanes"] / max(1, st["wave_steps"]),
                  "idle_drained_frac": ph["idle_drained_lanes"] / max(1, st["wave_steps"]),
                  "stack_pushes_per_segment": ph["push_lane"] / max(1, st["segments"]),
                  "global_push_share": ph["push_global"] / max(1, ph["push_lane"]),
                  "global_stack_bytes": 12 * (ph["push_global"] + ph["pop_global"]),
                  "region_entry_lane_util": {k: round(ph["w_" + k] / max(1, ph[k]), 4)
                                             for k in ("intersect", "light_sample", "light_pdf", "segment")},
                  "wave_cycles": ph, "share_of_tile_time": {k: round(v, 4) for k, v in share.items()}}))
