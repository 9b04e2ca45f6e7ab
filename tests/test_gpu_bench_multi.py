"""bench.py's N > 1 config-4 leg checks its own result: two ranks of `bench.py --gpus 2` on one GPU
(HGX_DEVICE=0) over the host-staged gloo transport (HGX_BENCH_C4_TRANSPORT=host; the driver's
8-GPU run uses RCCL through the same Transport interface) compare the parts' summed per-source
counts with the replica's after the timed steps, report `config4.partitioned.parity`, and exit
non-zero when they differ (HGX_BENCH_INJECT_MISMATCH=1 perturbs one summed count)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "2", "--steps", "1", "--warmup", "1", "--scale", "0.005", "--sources", "64", "--no-queries",
        "--no-config5", "--no-cpu-baseline", "--c4-scale", "0.005", "--c4-timeout", "100"]


def run_bench(extra_env):
    env = dict(os.environ, HGX_DEVICE="0", HGX_BENCH_C4_TRANSPORT="host", **extra_env)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS, env=env, capture_output=True,
                       text=True, timeout=110)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr[-3000:]


def test_two_rank_partitioned_leg_checks_itself():
    rc, line, err = run_bench({})
    assert rc == 0, err
    part = line["config4"]["partitioned"]
    assert part["n_gpus"] == 2 and part["scaling"] == "strong"
    assert part["parity"] is True, err
    assert "host-staged" in part["parallelism"]
    assert "error" not in line["config4"]


def test_two_rank_partitioned_leg_fails_on_mismatch():
    rc, line, err = run_bench({"HGX_BENCH_INJECT_MISMATCH": "1"})
    assert rc == 3, err
    assert line["config4"]["partitioned"]["parity"] is False
    assert "differ" in line["config4"]["error"]
