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
