"""Host logic of bench.py that runs without a GPU."""
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _bench():
    spec = importlib.util.spec_from_file_location("rt_bench", os.path.join(HERE, "..", "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pmc_child_leaves_the_process_group():
    """Under torchrun rank 0 starts its rocprofv3 --pmc children before it joins
    the group: a child that inherited WORLD_SIZE/RANK/MASTER_* would join the
    rendezvous as a rank of its own.  child_env strips them and pins rank 0's GPU."""
    b = _bench()
    env = {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "8", "GROUP_RANK": "0",
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29500", "TORCHELASTIC_RUN_ID": "x",
           "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/usr/bin"}
    out = b.child_env(env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR",
              "MASTER_PORT", "TORCHELASTIC_RUN_ID"):
        assert k not in out
    assert out["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and out["PATH"] == "/usr/bin"
    assert out["HIP_VISIBLE_DEVICES"] == "0"
    # an explicit device mask is the caller's: left alone
    out = b.child_env({**env, "HIP_VISIBLE_DEVICES": "3"})
    assert out["HIP_VISIBLE_DEVICES"] == "3"
    # a single-process run has nothing to strip
    assert b.child_env({"PATH": "/usr/bin"}) == {"PATH": "/usr/bin"}


def test_valu_roofline_prices_every_class():
    """frac prices each PMC class at its measured issue cost (tools/valu_prices.json for the
    classes without a single rate); the 2.3 / 4.2-cycle bounds bracket it."""
    b = _bench()
    pmc = {"SQ_INSTS_VALU": 100.0, "SQ_INSTS_VALU_FMA_F64": 20.0, "SQ_INSTS_VALU_MUL_F64": 10.0,
           "SQ_INSTS_VALU_ADD_F64": 10.0, "SQ_INSTS_VALU_TRANS_F64": 1.0, "SQ_INSTS_VALU_INT64": 4.0,
           "SQ_INSTS_VALU_INT32": 10.0, "SQ_INSTS_VALU_CVT": 5.0, "SQ_INSTS_VALU_ADD_F32": 0.0,
           "SQ_INSTS_VALU_MUL_F32": 0.0, "SQ_INSTS_VALU_FMA_F32": 0.0, "SQ_INSTS_VALU_TRANS_F32": 0.0,
           "SQ_THREAD_CYCLES_VALU": 3000.0, "SQ_ACTIVE_INST_VALU": 100.0, "GRBM_GUI_ACTIVE": 8 * 2.0e9 * 1e-6}
    r = b.valu_roofline(pmc, 1000, 1e-6, "path_kernel<false, false, 5, false, 1, false>")
    d = r["valu_detail"]
    assert d["rest"] == 100 - 40 - 1 - 4 - 10 - 5
    assert d["frac_lower"] < r["frac"] < d["frac_upper"]
    assert 3.5 < d["issue_cycles_per_instr"]["rest"] < 4.5 and 2.0 < d["issue_cycles_per_instr"]["int32"] < 4.3
    busy = 4.2 * 40 + 16.2 + 4.5 * 4 + sum(d["issue_cycles_per_instr"][k] * d[k] for k in ("int32", "cvt", "f32", "rest"))
    assert abs(d["busy_simd_cycles"] - busy) < 1e-9


def test_gpus_flag_plans_the_ranks():
    """`--gpus N` means N ranks: without torchrun, N > 1 launches them (torchrun as a child
    process); under torchrun, --gpus must equal WORLD_SIZE; a PMC child is always one
    standalone process."""
    b = _bench()
    assert b.rank_plan(1, {}) == ("run", 1)
    assert b.rank_plan(8, {"PATH": "/usr/bin"}) == ("launch", 8)
    assert b.rank_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}) == ("run", 8)
    kind, msg = b.rank_plan(8, {"WORLD_SIZE": "2"})
    assert kind == "error" and "--gpus 8" in msg and "WORLD_SIZE=2" in msg
    assert b.rank_plan(1, {"WORLD_SIZE": "4"})[0] == "error"  # the default --gpus 1 under a 4-rank torchrun
    assert b.rank_plan(0, {})[0] == "error"
    assert b.rank_plan(8, {"WORLD_SIZE": "8"}, pmc_child=True) == ("run", 1)
    assert b.rank_plan(1, {}, pmc_child=True) == ("run", 1)


def test_torchrun_child_command():
    """The launch relays every argument to the ranks and pins the rendezvous to 127.0.0.1."""
    b = _bench()
    argv = ["--gpus", "4", "--steps", "5", "--dist-backend", "gloo"]
    cmd = b.torchrun_cmd(4, argv, 29611)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29611"
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    p = b.free_port()
    assert 0 < p < 65536


def test_f64_arith_frac():
    """The arithmetic roofline: f64 FMA/MUL/ADD lane-ops/s over 64 lanes per 4.2 cycles on 1024 SIMDs."""
    b = _bench()
    pmc = {"SQ_INSTS_VALU": 100.0, "SQ_INSTS_VALU_FMA_F64": 20.0, "SQ_INSTS_VALU_MUL_F64": 10.0,
           "SQ_INSTS_VALU_ADD_F64": 10.0, "SQ_INSTS_VALU_TRANS_F64": 1.0, "SQ_INSTS_VALU_INT64": 4.0,
           "SQ_INSTS_VALU_INT32": 10.0, "SQ_INSTS_VALU_CVT": 5.0, "SQ_INSTS_VALU_ADD_F32": 0.0,
           "SQ_INSTS_VALU_MUL_F32": 0.0, "SQ_INSTS_VALU_FMA_F32": 0.0, "SQ_INSTS_VALU_TRANS_F32": 0.0,
           "SQ_THREAD_CYCLES_VALU": 3000.0, "SQ_ACTIVE_INST_VALU": 100.0, "GRBM_GUI_ACTIVE": 8 * 2.0e9 * 1e-6}
    d = b.valu_roofline(pmc, 1000, 1e-6, "path_kernel<false, false, 5, false, 1, false>")["valu_detail"]
    want = 40 * 30 / 1e-6 / (64 / 4.2 * 1024 * 2.0e9)
    assert abs(d["f64_arith_frac"] - want) < 1e-12 * want + 1e-18
    assert d["f64_instr_share"] == 0.4


def test_kernel_instance_from_tuning():
    """The VALU prices are the timed instance's own (render.hip path_fn_r's choice)."""
    b = _bench()
    c2 = dict(waves=5, resume=0, kinds=1, compact=0)
    c3 = dict(waves=4, resume=1, kinds=2, compact=1)
    f64 = dict(waves=4, resume=1, kinds=2, compact=0)
    assert b.kernel_instance(c2) == "path_kernel<false, false, 5, false, 1, false>"
    assert b.kernel_instance(c3) == "path_kernel<false, false, 4, true, 2, true>"
    assert b.kernel_instance(f64) == "path_kernel<false, false, 4, true, 2, false>"
    for t in (c2, c3, f64):
        prices, row = b.class_prices(b.kernel_instance(t))
        assert prices and row in ("C2", "C3", "tri_f64")
    assert b.class_prices("path_kernel<false, false, 3, false, 3, false>") == (None, None)


def test_dist_timeout_outlasts_the_pmc_passes():
    """Under torchrun ranks 1..N-1 wait in init_process_group while rank 0 runs its
    rocprofv3 --pmc children: the group's timeout covers every child's
    own limit, and both backends are given it."""
    b = _bench()
    assert b.DIST_TIMEOUT_S > len(b.PMC_PASSES) * b.PMC_CHILD_TIMEOUT_S
    src = open(os.path.join(HERE, "..", "bench.py")).read()
    assert 'init_process_group("nccl", device_id=dev, timeout=pg_timeout)' in src
    assert 'init_process_group("gloo", timeout=pg_timeout)' in src


def test_cpu_baseline_without_any_oracle_build(monkeypatch):
    """a host where neither oracle build works keeps the GPU line: the
    baseline's value is None and the per-build errors are reported."""
    import sys
    import types
    b = _bench()
    fake = types.ModuleType("oracle")

    class Boom:
        def __init__(self, *a, **k):
            raise RuntimeError("no compiler")

    fake.OracleScene = Boom
    monkeypatch.setitem(sys.modules, "oracle", fake)
    out = b.cpu_baseline(None, None, 1.0)
    assert out["value"] is None and out["value_build"] is None
    assert set(out["builds"]) == {"native", "portable"}
    assert all("no compiler" in v["error"] for v in out["builds"].values())
