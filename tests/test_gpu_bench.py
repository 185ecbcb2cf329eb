"""bench.py's N-rank path on the GPU box: `--gpus 2` without a torchrun
environment launches two ranks (torchrun as a child process); with gloo both share the
one GPU and the line reports n_gpus 2, world_size_seen 2 and the one-rank frame digest;
with nccl on a one-GPU box it must fail instead of silently rendering on one GPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

BASE = ["--workload", "C1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
ARGS = BASE + ["--no-pmc"]


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _run(extra, timeout=240, args=ARGS):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args, *extra], capture_output=True,
                          text=True, timeout=timeout, env=env)


def test_bench_gpus2_gloo_matches_one_rank():
    one = _run([])
    assert one.returncode == 0, one.stderr[-2000:]
    two = _run(["--gpus", "2", "--dist-backend", "gloo"])
    assert two.returncode == 0, two.stderr[-2000:]
    a, b = _line(one.stdout), _line(two.stdout)
    assert a["n_gpus"] == 1 and a["world_size_seen"] == 1
    assert b["n_gpus"] == 2 and b["world_size_seen"] == 2 and len(b["rank_devices"]) == 2
    assert b["image_sha256"] == a["image_sha256"]
    assert b["config"]["segments_per_step"] == a["config"]["segments_per_step"]


@pytest.mark.skipif(torch.cuda.device_count() > 1, reason="needs a one-GPU box")
def test_bench_gpus2_nccl_refuses_one_gpu():
    r = _run(["--gpus", "2"])
    assert r.returncode != 0
    assert "visible GPU" in r.stdout + r.stderr


def test_bench_gpus2_gloo_with_pmc_passes():
    """The driver's N>1 command keeps its PMC passes: rank 0 runs its
    rocprofv3 --pmc children while rank 1 waits in init_process_group (timeout =
    bench.DIST_TIMEOUT_S); the line then carries rank 0's roofline (VALU and HBM), the
    world it saw and the one-rank digest."""
    one = _run([])
    assert one.returncode == 0, one.stderr[-2000:]
    two = _run(["--gpus", "2", "--dist-backend", "gloo"], timeout=600, args=BASE)
    assert two.returncode == 0, two.stderr[-2000:]
    a, b = _line(one.stdout), _line(two.stdout)
    assert b["world_size_seen"] == 2 and b["image_sha256"] == a["image_sha256"]
    r = b["roofline"]
    assert r["frac"] is not None and r["frac"] > 0, r
    assert r["hbm"]["frac"] > 0 and r["traffic"] > 0
