#!/usr/bin/env python3
"""Headline benchmark: Msamples/s (rays traced x bounces) of the path-tracing
hot path on the C2 workload (BASELINE.json configs[1]: Cornell box,
1920x1080, 256 spp, depth 16) on N MI355X GPUs.

One step = one full frame: every (pixel, sample) path of the frame
(generate_image, main.rs:85-114), tile-partitioned across the ranks (16x16
tiles round-robin), then ONE RCCL gather of the packed
framebuffer tiles to rank 0 and the fused device epilogue: unpack + ACES +
gamma + PPM bytes (main.rs:104, ppm.rs:13-19) into the row-major payload.
"Sample" = one path segment = one closest-hit query (raytrace.rs:14); the
per-frame segment count is counted on the device in an untimed pass.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without a torchrun environment, --gpus N > 1 starts the N ranks itself: torchrun
as a child process (this process makes no HIP call first), whose rank 0 prints
the line; its exit code is bench.py's.  Under torchrun, --gpus must equal
WORLD_SIZE.  The line carries world_size_seen (dist.get_world_size()) and each
rank's device (PCI id; distinct under nccl, or every rank exits non-zero).

Rank 0 prints ONE JSON line.  Extras: "roofline" (the path kernel's f64 VALU
issue roofline: PMC instruction mix of its launch over the chip's issue limit,
timed by HIP events; plus its measured HBM rate and the SURVEY §8d algorithmic
byte rate) and "cpu_baseline" (the oracle, the C restatement of the reference, timed on
a bounded row window of the same frame on the host cores; rank 0, N=1 only).
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before the package: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from conftest import load_package  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
# canonical algorithmic bytes per work unit
B_AABB, B_TRI, B_SHAPE, B_SHADE = 32, 72, 80, 100

WORKLOADS = {
    # name: (scene, width, height, spp, depth override or None); "gltf:<name>" = scenes/gen/<name>.gltf
    "C2": ("cornell.txt", 1920, 1080, 256, None),
    "C1": ("cornell.txt", 256, 256, 64, None),
    "C3": ("gltf:sponza_like", 1920, 1080, 256, None),   # ray_depth 8 comes from the glTF builder
    "C4": ("gltf:sponza_like", 3840, 2160, 1024, None),  # BASELINE configs[3]: the 8-GPU scaling frame
    "C5": ("gltf:hairball", 1920, 1080, 64, None),       # BASELINE configs[4]: 10M-triangle stress scene
}
GENERATORS = {"sponza_like": "gen_sponza_like.py", "hairball": "gen_hairball.py"}
DESCRIPTIONS = {
    "cornell.txt": "Cornell box (scenes/cornell.txt, custom format, 9 primitives, 1 emissive box light)",
    "gltf:sponza_like": "synthetic Sponza-class atrium (scenes/gen_sponza_like.py -> glTF, 263k smooth-normal "
                        "triangles, full BVH, emissive ceiling quad, black background)",
    "gltf:hairball": "synthetic hairball (scenes/gen_hairball.py -> glTF, 10M thin random triangles in a unit "
                     "ball, 1 emissive quad, black background; BVH + triangles ~1.7 GB, past the Infinity Cache)",
}


def load_workload(rt, scene_file, W, H, spp):
    if scene_file.startswith("gltf:"):
        name = scene_file[5:]
        path = os.path.join(HERE, "scenes", "gen", name + ".gltf")
        if not os.path.exists(path):  # deterministic generator; the asset is not committed
            import subprocess
            subprocess.run([sys.executable, os.path.join(HERE, "scenes", GENERATORS[name]),
                            os.path.join(HERE, "scenes", "gen"), "--name", name], check=True,
                           stdout=subprocess.DEVNULL)
        return rt.load_gltf(path, W, H, spp)
    desc, params = rt.parse_scene(open(os.path.join(HERE, "scenes", scene_file)).read())
    return desc, params.replace(width=W, height=H, spp=spp)


def algo_bytes(st):
    return B_AABB * st["aabb_tests"] + B_TRI * st["tri_tests"] + B_SHAPE * st["shape_tests"] + B_SHADE * st["shaded_hits"]


PATH_KERNEL = "path_kernel<false, false,"  # the timed instance (any waves/SIMD budget)

# VALU issue roofline.  The path kernel is f64 VALU-issue bound,
# not HBM- or MFMA-bound.  Every PMC class of VALU instruction is priced in SIMD
# issue cycles per wave64 instruction, measured at full load (8 waves/SIMD, wall
# clock; tools/valu_rates.hip, profiles/r04/valu_rates_full.log): v_fma/mul/add_f64
# 4.2, f64 transcendentals 16.2, int64 (v_mad_u64_u32, v_lshl_add_u64) 4.5.  The
# classes without a single rate — int32 (v_add_u32 2.3 ... v_lshlrev / v_bfe /
# v_mul_lo 4.2), conversions, f32, and the uncounted rest (v_cmp_*, v_cndmask,
# moves, readlane: 2.3 ... 4.2) — take the mean measured cost of their opcodes
# weighted by the kernel instance's static code (tools/valu_mix.py ->
# tools/valu_prices.json: rest 4.0, int32 2.8, cvt 4.4).  frac is priced
# that way; frac_lower / frac_upper price every class without its own rate at the
# cheapest (2.3) / dearest (4.2) measured 32-bit cost.
SIMDS = 256 * 4
MAX_CLOCK_HZ = 2.4e9
VALU_CYCLES = {"f64": 4.2, "trans_f64": 16.2, "int64": 4.5}
CHEAP, DEAR = 2.3, 4.2
PRICES_FILE = os.path.join(HERE, "tools", "valu_prices.json")  # profiles/ does not travel to the box
PMC_PASSES = (
    # (counters, one pass each: <= 8 SQ, <= 4 TCC (FETCH_SIZE uses 3, WRITE_SIZE 2), <= 2 GRBM)
    ("FETCH_SIZE", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"),
    ("WRITE_SIZE",),
    ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
     "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT64", "GRBM_GUI_ACTIVE"),
    ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
     "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32"),
)


# Each PMC child may take up to PMC_CHILD_TIMEOUT_S.  Under torchrun the other ranks wait
# in init_process_group while rank 0 runs them, so the process group's rendezvous
# timeout must outlast all of them (torch's default is 10 min for nccl): DIST_TIMEOUT_S.
PMC_CHILD_TIMEOUT_S = 900
DIST_TIMEOUT_S = len(PMC_PASSES) * PMC_CHILD_TIMEOUT_S + 600


def kernel_instance(tuning):
    """The timed path-kernel instance's template arguments from the scene's resolved
    form (rt_scene_get_tuning; render.hip path_fn_r): <ST, HIT, WAVES, RES, KM, CMP>."""
    w, res, k = tuning["waves"], tuning["resume"] == 1, tuning["kinds"]
    if res and w == 4:
        km, cmp_ = (2, tuning["compact"] == 1) if k == 2 else (3, False)
    elif res:
        km, cmp_ = 3, False
    else:
        km, cmp_ = (1 if k == 1 else 3), False
    return f"path_kernel<false, false, {w}, {'true' if res else 'false'}, {km}, {'true' if cmp_ else 'false'}>"


def class_prices(kernel):
    """Static-mix mean prices of the int32 / cvt / f32 / rest classes for one kernel
    instance (tools/valu_mix.py), matched by its template arguments; (None, None) when
    the table has no row for that instance."""
    try:
        table = json.load(open(PRICES_FILE))["instances"]
    except (OSError, KeyError, ValueError):
        return None, None
    for name, row in table.items():
        if row.get("kernel") == kernel:
            d = row["classes"]
            return {k: d[k]["mean_cycles"] for k in ("int32", "cvt", "f32", "rest") if k in d}, name
    return None, None


DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT",
            "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_RUN_ID",
            "TORCHELASTIC_USE_AGENT_STORE", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


def child_env(env):
    """Environment of a PMC child: the parent's, minus the torchrun rendezvous
    variables, so the child is a standalone one-GPU process on the parent's
    device and never joins (or blocks) the parent's process group."""
    out = {k: v for k, v in env.items() if k not in DIST_ENV}
    local = env.get("LOCAL_RANK")
    if local is not None and "HIP_VISIBLE_DEVICES" not in env and "CUDA_VISIBLE_DEVICES" not in env:
        out["HIP_VISIBLE_DEVICES"] = local  # rank 0's own GPU
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_plan(gpus, env, pmc_child=False):
    """How this bench.py process runs for `--gpus N` (main.rs:94-111 is one frame over
    every pixel; here N ranks, one per GPU, share it).  Returns one of
      ("run", world)        render as rank RANK of WORLD_SIZE (1 when not under torchrun);
      ("launch", n)         no torchrun environment and N > 1: start N ranks under
                            torchrun as a CHILD process (never an exec) and relay its rc;
      ("error", message)    --gpus disagrees with the torchrun world.
    Decided from arguments and environment only: nothing here touches the GPU."""
    if pmc_child:
        return ("run", 1)
    if gpus < 1:
        return ("error", f"bench.py: --gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" not in env:
        return ("launch", gpus) if gpus > 1 else ("run", 1)
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        return ("error", f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the rank count must be the GPU "
                         f"count asked for")
    return ("run", world)


def torchrun_cmd(n, argv, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def pmc_counters(args, world):
    """Counters of the timed path kernel's launch, from child rocprofv3 --pmc
    passes of this same workload (rank 0's tile share of a world-`world`
    partition), run BEFORE this process initialises the GPU.  Returns
    ({counter: value}, dispatch_ns) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    vals, ns = {}, None
    env = child_env(os.environ)
    with tempfile.TemporaryDirectory(prefix="rt_pmc_") as td:
        for i, counters in enumerate(PMC_PASSES):
            d = os.path.join(td, f"p{i}")
            cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.abspath(__file__), "--workload", args.workload, "--steps", "1",
                   "--warmup", "0", "--no-cpu-baseline", "--no-pmc", "--as-rank0-of", str(world)]
            cmd += ["--tune", args.tune] if args.tune else []
            cmd += ["--spp", str(args.spp)] if args.spp else []
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=PMC_CHILD_TIMEOUT_S, env=env)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {' '.join(counters)} failed rc={r.returncode}: {r.stderr[-300:]}"
            rows = []
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        rows += [x for x in csv.DictReader(open(os.path.join(root, f))) if PATH_KERNEL in x["Kernel_Name"]]
            if not rows:
                return None, f"no rows for {PATH_KERNEL} in the pass {counters}"
            last = max(int(x["Dispatch_Id"]) for x in rows)  # the timed launch (the first is the counting pass)
            for x in rows:
                if int(x["Dispatch_Id"]) == last:
                    vals[x["Counter_Name"]] = vals.get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
                    ns = int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
    missing = [c for p in PMC_PASSES for c in p if c not in vals]
    if missing:
        return None, f"counters missing: {missing}"
    return vals, ns


def hbm_traffic(pmc):
    """Memory-side bytes per launch.  Correction per MI355X_MICROARCH.md "HBM":
    FETCH_SIZE is in KiB and reports half the bytes on gfx950, so fetch = 2 *
    1024 * FETCH_SIZE; WRITE_SIZE is taken as reported (KiB).  The x2 factor is
    calibrated for the traversal's own access pattern (tools/fetch_calib.hip,
    profiles/r03/fetch_calib.log): for dependent random gathers of 128-B fat
    nodes, 80-B / 36-B triangle records and 64-B compact nodes, over a 128-MiB
    (Infinity-Cache-resident) and a 4-GiB table, 2 x 1024 x FETCH_SIZE equals
    the 128-B-line bytes the L2 requested from the memory side (TCC_EA0_RDREQ
    by size) within 3%, MALL hits included (TCC_EA0_RDREQ_DRAM counts them
    too).  So `fetch` is line bytes past the L2, MALL + DRAM; it is >= the
    algorithmic bytes (1.0x for 128-B records, 2.0x for 64-B, 2.4x for 80-B,
    4.4x for 36-B)."""
    fetch = 2.0 * 1024.0 * pmc["FETCH_SIZE"]
    write = 1024.0 * pmc["WRITE_SIZE"]
    return fetch + write, {"FETCH_SIZE_KiB": pmc["FETCH_SIZE"], "WRITE_SIZE_KiB": pmc["WRITE_SIZE"],
                           "fetch_bytes": fetch, "write_bytes": write,
                           "correction": "fetch = 2 x 1024 x FETCH_SIZE = 128-B-line bytes past the L2 (MALL + "
                                         "DRAM), calibrated for the traversal's gathers in "
                                         "profiles/r03/fetch_calib.log; write = 1024 x WRITE_SIZE",
                           "kernel": PATH_KERNEL}


def valu_roofline(pmc, pmc_ns, kern_s, instance):
    """VALU issue roofline of the path kernel: busy SIMD issue cycles of the launch's
    instruction mix (every PMC class at its measured price) over the cycles the
    chip's 1024 SIMDs had during the launch."""
    n = pmc["SQ_INSTS_VALU"]
    f64 = pmc["SQ_INSTS_VALU_FMA_F64"] + pmc["SQ_INSTS_VALU_MUL_F64"] + pmc["SQ_INSTS_VALU_ADD_F64"]
    trans, i64 = pmc["SQ_INSTS_VALU_TRANS_F64"], pmc["SQ_INSTS_VALU_INT64"]
    i32, cvt = pmc["SQ_INSTS_VALU_INT32"], pmc["SQ_INSTS_VALU_CVT"]
    f32 = (pmc["SQ_INSTS_VALU_ADD_F32"] + pmc["SQ_INSTS_VALU_MUL_F32"] + pmc["SQ_INSTS_VALU_FMA_F32"] +
           pmc["SQ_INSTS_VALU_TRANS_F32"])
    rest = max(0.0, n - f64 - trans - i64 - i32 - cvt - f32)
    mix = {"int32": i32, "cvt": cvt, "f32": f32, "rest": rest}
    prices, row = class_prices(instance)
    prices = prices or {}
    priced = {k: prices.get(k, (CHEAP + DEAR) / 2) for k in mix}
    fixed = VALU_CYCLES["f64"] * f64 + VALU_CYCLES["trans_f64"] * trans + VALU_CYCLES["int64"] * i64
    busy = fixed + sum(priced[k] * mix[k] for k in mix)  # SIMD issue cycles the launch needs
    lo = fixed + CHEAP * sum(mix.values())
    hi = fixed + DEAR * sum(mix.values())
    # shader clock of the profiled launch: GRBM_GUI_ACTIVE is summed over the 8 XCDs
    clk = pmc["GRBM_GUI_ACTIVE"] / 8.0 / (pmc_ns * 1e-9) if pmc_ns else 0.0
    clk_used = clk if 1.0e9 <= clk <= MAX_CLOCK_HZ else MAX_CLOCK_HZ
    avail = SIMDS * clk_used * kern_s
    frac = busy / avail
    achieved = n / kern_s / 1e9
    lanes = pmc["SQ_THREAD_CYCLES_VALU"] / pmc["SQ_ACTIVE_INST_VALU"]
    return {
        "bound": "valu",
        "achieved": achieved,
        "peak": achieved / frac,
        "unit": "G wave64 VALU instr/s",
        "frac": frac,
        "valu_detail": {
            "instr_per_launch": n, "f64_fma_mul_add": f64, "f64_trans": trans, "int64": i64, "int32": i32,
            "cvt": cvt, "f32": f32, "rest": rest,
            "issue_cycles_per_instr": {**VALU_CYCLES, **priced},
            "kernel_instance": instance,
            "prices_source": ("profiles/r04/valu_rates_full.log (measured, 8 waves/SIMD); int32/cvt/f32/rest: "
                              f"static-mix means of {instance} (tools/valu_prices.json row {row})"
                              if prices else f"int32/cvt/f32/rest at the mid of the measured 32-bit range (no "
                                             f"static-mix row for {instance})"),
            "busy_simd_cycles": busy,
            "frac_lower": lo / avail, "frac_upper": hi / avail,
            "clock_GHz": clk_used / 1e9, "clock_measured_GHz": clk / 1e9,
            "active_lanes_per_instr": lanes, "lane_util": lanes / 64.0,
            "useful_lane_frac": frac * lanes / 64.0,
            # the arithmetic roofline beside the issue one: f64 FMA/MUL/ADD lane-ops per second
            # (instructions x the launch's mean active lanes) over the FP64 vector rate at
            # the measured price, 64 lanes per 4.2 cycles on each of the 1024 SIMDs
            "f64_arith_frac": f64 * lanes / kern_s / (64.0 / VALU_CYCLES["f64"] * SIMDS * clk_used),
            "f64_instr_share": f64 / n,
            "hw_active_frac": 4.0 * pmc["SQ_ACTIVE_INST_VALU"] / avail,
            "peak_note": "peak = the same instruction mix issued back to back on all 1024 SIMDs at the measured "
                         "clock; frac = busy SIMD cycles (every class at its measured issue cost) / available; "
                         "frac_lower / frac_upper = the classes without their own rate at 2.3 / 4.2 cycles; "
                         "useful_lane_frac = frac x active lanes / 64 (divergence); hw_active_frac = "
                         "SQ_ACTIVE_INST_VALU quad-cycles x 4 / available cycles; f64_arith_frac = f64 FMA/MUL/ADD "
                         "lane-ops/s (x mean active lanes) / (64 / 4.2 x 1024 SIMDs x clock)",
        },
    }


def cpu_share():
    """The host cores this process may use: its affinity mask, capped by the cgroup CPU
    quota when one is set (a GPU box's share of the machine; nproc shows every CPU)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpus": quota,
                     "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_band(osc, params, threads, target_s, rows=None):
    """One timed render of a centred band of rows at full spp.  rows=None grows the band
    in small slices until ~target_s of CPU work is done (the box's CPU share varies, so a
    one-shot calibration over- or under-shoots by several x); otherwise renders exactly
    `rows`.  Returns (Msamples/s, (r0, r1), paths, segments, seconds)."""
    segs = paths = 0
    dt = 0.0
    if rows is not None:
        t = time.perf_counter()
        _, _, st = osc.render(params, mode=0, threads=threads, rows=rows)
        dt = time.perf_counter() - t
        return st["segments"] / dt / 1e6, rows, st["paths"], st["segments"], dt
    mid = params.height // 2
    r0 = r1 = mid
    step = 2
    while dt < target_s and (r0 > 0 or r1 < params.height):
        lo, hi = max(0, r0 - step // 2), min(params.height, r1 + step - step // 2)
        for a, b in ((lo, r0), (r1, hi)):
            if b <= a:
                continue
            t = time.perf_counter()
            _, _, st = osc.render(params, mode=0, threads=threads, rows=(a, b))
            dt += time.perf_counter() - t
            segs += st["segments"]
            paths += st["paths"]
        r0, r1 = lo, hi
        rate = (r1 - r0) / max(dt, 1e-3)  # rows per second so far
        step = int(max(2, min(2 * (r1 - r0), rate * (target_s - dt) / 2)))
    return segs / dt / 1e6, (r0, r1), paths, segs, dt


def cpu_baseline(desc, params, target_s, runs=3):
    """Oracle (C restatement, kind "port") on a bounded window of rows at full spp, on
    every host core this process may use (rayon uses all cores, main.rs:94).  Two builds
    (SURVEY.md §8d): -O3 -march=native, compiled here on this host (`make -C oracle
    native`), and the portable -O3 build that travels with the tree.  Each is timed
    `runs` times on the same band (the first run sizes it to ~target_s / runs); the
    reported rate is the median, with the spread.  value = the faster build's median
    (the stricter baseline)."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as orc
    threads, host = cpu_share()
    out = {"unit": "Msamples/s", "cores": threads, "host": host, "kind": "port"}
    rows = None
    builds = {}
    for variant in ("native", "portable"):
        print(f"bench: cpu baseline ({variant}): building the oracle scene on {threads} threads",
              file=sys.stderr, flush=True)
        try:
            tb = time.perf_counter()
            osc = orc.OracleScene(desc, variant=variant)  # the restated reference builder: outside the timed leg
            build_s = time.perf_counter() - tb
        except Exception as e:  # noqa: BLE001  (no compiler for the native build: report it)
            builds[variant] = {"error": f"{type(e).__name__}: {e}"}
            continue
        rates, secs = [], []
        for _ in range(runs):
            rate, rows, paths, segs, dt = cpu_band(osc, params, threads, target_s / runs, rows)
            rates.append(rate)
            secs.append(dt)
        builds[variant] = {"median": float(np.median(rates)), "runs": rates, "seconds": secs,
                           "spread": (max(rates) - min(rates)) / float(np.median(rates)),
                           "oracle_build_s": build_s,
                           "flags": "-O3 -march=native" if variant == "native" else "-O3 (portable)"}
        del osc
    done = [v for v in ("native", "portable") if "median" in builds.get(v, {})]
    out["builds"] = builds
    if not done:  # no oracle build on this host: report the errors, keep the GPU line
        out["value"] = None
        out["value_build"] = None
        return out
    ok = max(done, key=lambda v: builds[v]["median"])
    out["value"] = builds[ok]["median"]
    out["value_build"] = ok
    out["sample"] = (f"rows {rows[0]}..{rows[1]} of {params.width}x{params.height} at {params.spp} spp "
                     f"({paths} paths, {segs} segments per run), recursive raytrace_impl, OpenMP dynamic over "
                     f"pixels; median of {runs} runs per build")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--spp", type=int, default=None, help="override spp (not the headline config)")
    ap.add_argument("--cpu-seconds", type=float, default=18.0, help="CPU work per oracle build (split over 3 runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc child passes (roofline=null)")
    ap.add_argument("--as-rank0-of", type=int, default=0, help=argparse.SUPPRESS)  # PMC child: rank 0's share
    ap.add_argument("--tune", default="", help="experiments: force rt_tuning fields, e.g. compact=0,waves=4 "
                                                  "(the headline runs the library's own pick)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI, the product path); gloo gathers host copies and lets several "
                         "ranks share one GPU (a rehearsal of the N>1 path on a one-GPU box)")
    args = ap.parse_args()

    plan, arg = rank_plan(args.gpus, os.environ, pmc_child=bool(args.as_rank0_of))
    if plan == "error":
        sys.exit(arg)
    if plan == "launch":
        # `python bench.py --gpus N`: N ranks under torchrun, started as a child (this
        # process has made no HIP call), whose rank 0 prints the JSON line
        import subprocess
        cmd = torchrun_cmd(arg, sys.argv[1:], free_port())
        print("bench: " + " ".join(cmd), file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)
    world = arg
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.as_rank0_of:  # a PMC child is a standalone process, whatever its environment says
        world, rank, local = 1, 0, 0
    pmc, pmc_ns = None, "not collected (--no-pmc)"
    if rank == 0 and not args.no_pmc and not args.as_rank0_of:  # before this process touches the GPU
        pmc, pmc_ns = pmc_counters(args, world)
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and world > ndev:
        sys.exit(f"bench.py: WORLD_SIZE={world} ranks but {ndev} visible GPU(s): RCCL needs one GPU per rank "
                 f"(use --dist-backend gloo to rehearse several ranks on one GPU)")
    local = local % max(1, ndev)  # > 1 rank per GPU only in a gloo rehearsal
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import datetime
        pg_timeout = datetime.timedelta(seconds=DIST_TIMEOUT_S)  # rank 0's PMC passes come first
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group("gloo", timeout=pg_timeout)
    rt = load_package()

    scene_file, W, H, spp, depth = WORKLOADS[args.workload]
    if args.spp:
        spp = args.spp
    desc, params = load_workload(rt, scene_file, W, H, spp)
    if depth:
        params = params.replace(ray_depth=depth)
    t0 = time.perf_counter()
    scene = rt.Scene(desc)
    build_s = time.perf_counter() - t0
    if args.tune:
        scene.set_tuning(**{k: int(v) for k, v in (kv.split("=", 1) for kv in args.tune.split(","))})

    # a PMC child renders rank 0's tile share of the parent's partition, alone
    part = args.as_rank0_of or world
    per = scene.tiles_per_rank(params, part)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    tiles = torch.empty((per, 256, 3), dtype=torch.float64, device=dev)
    gathered = torch.empty((world, per, 256, 3), dtype=torch.float64, device=dev) if rank == 0 else None
    # the epilogue writes the PPM payload (tonemap + gamma + bytes fused into the unpack)
    image = torch.empty((H, W, 3), dtype=torch.uint8, device=dev) if rank == 0 else None

    # untimed counting pass: this rank's work of one frame
    scene.read_stats(reset=True)
    scene.render_tiles_async(params, rank, part, tiles.data_ptr(), sptr, stats=True)
    torch.cuda.synchronize()
    lq_skipped = int(scene.read_raw_stats(11)[10])  # last-bounce light queries the timed kernel skips
    st = scene.read_stats(reset=True)
    seg = torch.tensor([st["segments"], st["paths"]], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(seg)
    frame_segments, frame_paths = int(seg[0].item()), int(seg[1].item())

    # HIP events on the stream the kernels run on, per timed step: [render, gather,
    # epilogue] boundaries (the gather and epilogue pair stay unrecorded in a PMC child)
    ev = []

    def mark():
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def step(timed):
        marks = [mark()] if timed else None
        scene.render_tiles_async(params, rank, part, tiles.data_ptr(), sptr)
        if timed:
            marks.append(mark())
            ev.append(marks)
        if part != world:  # PMC child: only the path kernel is of interest
            return
        if args.dist_backend == "nccl" or world == 1:
            src = rt.gather_tiles(tiles, gathered, rank, world)
        else:  # gloo: the same single gather on host copies
            g_host = torch.empty(gathered.shape, dtype=gathered.dtype) if rank == 0 else None
            rt.gather_tiles(tiles.cpu(), g_host, rank, world)
            if rank == 0:
                gathered.copy_(g_host)
            src = gathered
        if timed:
            marks.append(mark())
        if rank == 0:
            rt.unpack_tiles_bytes_async(params, world, src.data_ptr(), image.data_ptr(), sptr)
        if timed:
            marks.append(mark())

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t
    # the host copy of the frame's PPM payload (main.rs:74 writes it), outside the timed
    # region: SURVEY §8d's end-to-end figure = ms_per_step + this D2H (pinned host buffer)
    d2h_ms = None
    if rank == 0 and part == world:
        host_img = torch.empty(tuple(image.shape), dtype=torch.uint8, pin_memory=True)
        d2h = []
        for _ in range(3):
            a = mark()
            host_img.copy_(image, non_blocking=True)
            b_ = mark()
            b_.synchronize()
            d2h.append(a.elapsed_time(b_))
        d2h_ms = float(np.median(d2h))
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    kern_ms = float(np.mean([m[0].elapsed_time(m[1]) for m in ev]))
    # per-rank phases of the timed steps (mean ms): render kernel, the single gather
    # (as this rank's stream sees it), the epilogue (rank 0) — so an N > 1 line
    # separates rank imbalance from communication
    phases = torch.tensor([kern_ms,
                           float(np.mean([m[1].elapsed_time(m[2]) for m in ev])) if len(ev[0]) > 2 else 0.0,
                           float(np.mean([m[2].elapsed_time(m[3]) for m in ev])) if len(ev[0]) > 3 else 0.0],
                          dtype=torch.float64, device=dev)
    # which device each rank rendered on (PCI domain:bus:device): under nccl every rank
    # must own a distinct GPU, so the line proves RCCL saw N ranks on N devices
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local, "hip_device": dev.index,
          "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
          "name": props.name}
    if world > 1:
        every = [torch.zeros_like(phases) for _ in range(world)]
        dist.all_gather(every, phases)
        per_rank = torch.stack(every).cpu().numpy()
        devices = [None] * world
        dist.all_gather_object(devices, me)
        world_seen = dist.get_world_size()
    else:
        per_rank = phases.cpu().numpy()[None, :]
        devices, world_seen = [me], 1
    if args.dist_backend == "nccl" and len({d["pci"] for d in devices}) != world:  # every rank exits
        sys.exit(f"bench.py: {world} nccl ranks but devices {[d['pci'] for d in devices]} are not distinct")

    if rank == 0 and part != world:  # PMC child: nothing to report
        return
    if rank == 0:
        value = frame_segments * args.steps / elapsed / 1e6
        kern_s = kern_ms * 1e-3
        algo = algo_bytes(st)
        if pmc is None:
            roofline = {"bound": "valu", "achieved": None, "peak": None, "unit": "G wave64 VALU instr/s",
                        "frac": None, "traffic": None, "note": f"PMC passes unavailable: {pmc_ns}"}
        else:
            roofline = valu_roofline(pmc, pmc_ns, kern_s, kernel_instance(scene.tuning()))
            traffic, detail = hbm_traffic(pmc)
            roofline["traffic"] = traffic
            roofline["hbm"] = {"achieved_GBps": traffic / kern_s / 1e9, "peak_GBps": HBM_PEAK_GBS,
                               "frac": traffic / kern_s / 1e9 / HBM_PEAK_GBS, "detail": detail}
        roofline.update({
            "kernel": "rt::path_kernel<false,false,W,RES> (W = waves/SIMD budget, RES = resumable traversal; "
                      "both chosen per scene)",
            "kernel_ms": kern_ms,
            "pmc_kernel_ms": (pmc_ns * 1e-6) if isinstance(pmc_ns, int) else None,
            # the SURVEY §8d canonical bytes: what the reference's data layout would move per
            # launch.  The kernel serves them from L1/L2/scalar cache/MALL, so their rate is a
            # cache-level throughput, not an HBM one, and is not used as `frac`
            "algorithmic": {"bytes_per_launch": algo, "GBps": algo / kern_s / 1e9,
                            "model": "32*aabb_tests + 72*tri_tests + 80*shape_tests + 100*shaded_hits "
                                     "(rank 0 tiles)",
                            # counted by the stats instance, which also runs the last-bounce light
                            # queries the timed kernel proves NaN-free and skips
                            "light_queries": st["light_queries"], "light_queries_skipped": lq_skipped},
            "note": "bound = f64 VALU issue: frac = VALU busy SIMD-cycles / available (valu_detail); the "
                    "measured HBM rate is roofline.hbm (traffic = PMC HBM bytes per launch)",
        })
        out = {
            "metric": "Msamples/s (rays traced x bounces) at 1920x1080, 256 spp; fraction of f64 VALU-issue "
                      "roofline (measured issue costs per instruction class; the measured HBM fraction is "
                      "roofline.hbm)",
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "world_size_seen": world_seen,
            "rank_devices": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{args.workload}: {DESCRIPTIONS[scene_file]}, {W}x{H}, {spp} spp, "
                            f"ray_depth {params.ray_depth}",
                "triangles": int(len(desc.tri_material)), "shapes": int(len(desc.shapes)),
                "width": W, "height": H, "spp": spp, "ray_depth": params.ray_depth,
                "paths_per_step": frame_paths, "segments_per_step": frame_segments,
                "parallelism": f"tiles16x16 round-robin over {world} rank(s) + 1 "
                               f"{'RCCL' if args.dist_backend == 'nccl' else 'gloo (rehearsal)'} gather",
                "epilogue": "device unpack + ACES + gamma + PPM bytes (rt_unpack_tiles_bytes_async)",
                "seed": params.seed,
            },
            "roofline": roofline,
            "paths_per_s": frame_paths * args.steps / elapsed,
            "tuning": scene.tuning(),
            "scene_build_s": build_s,
            # HIP-event means over the timed steps, one entry per rank: the render kernel
            # (incl. the chunk reduce), the gather as each rank's stream sees it, and rank
            # 0's fused epilogue; max(render) / mean(render) is the render-side imbalance
            "phases_ms": {"render": per_rank[:, 0].tolist(), "gather": per_rank[:, 1].tolist(),
                          "epilogue": float(per_rank[0, 2]),
                          "render_imbalance": float(per_rank[:, 0].max() / per_rank[:, 0].mean()),
                          # PPM payload device -> pinned host, median of 3, after the timed steps
                          "d2h": d2h_ms},
            # kernel-only (roofline.kernel_ms), whole step on the device (ms_per_step:
            # render + gather + epilogue), and end to end with the payload's host copy
            "end_to_end_ms_per_step": elapsed / args.steps * 1e3 + (d2h_ms or 0.0),
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(desc, params, args.cpu_seconds)
            cb = out["cpu_baseline"]["value"]
            out["speedup_vs_cpu"] = value / cb if cb else None
        # the PPM payload of the last frame (outside the timed region): identical for any N
        out["image_sha256"] = hashlib.sha256(image.cpu().numpy().tobytes()).hexdigest()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
