"""bench.py --gpus N starts N ranks by itself: the driver
may run `python bench.py --gpus N` without torch.distributed.run. The rank
count must equal --gpus, or the run fails (rc != 0) instead of timing one
rank labelled as N."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench(args, env_extra, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_world_mismatch_fails_before_any_gpu_call():
    r = _bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, 120)
    assert r.returncode != 0
    assert "--gpus 4 but the launcher started 2 rank(s)" in r.stderr


@pytest.mark.gpu
def test_bench_gpus_2_self_launch_gloo(cuda):
    """On the one-GPU box: `BQ_BENCH_BACKEND=gloo bench.py --gpus 2` (two
    ranks sharing the GPU, collectives over gloo) reports n_gpus 2, the
    whole panel's symbols, and the breadth leg's tracked total from the one
    all-reduce equal to every symbol of both shards."""
    S, T = 3000, 512
    r = _bench(["--gpus", "2", "--symbols", str(S), "--candles", str(T), "--steps", "2", "--warmup", "1",
                "--no-shard", "--no-tick", "--no-rows", "--no-cpu-baseline", "--breadth-steps", "1"],
               {"BQ_BENCH_BACKEND": "gloo"}, 240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["config"]["symbols"] == S and res["config"]["symbols_per_gpu"] == S // 2
    assert res["breadth"]["tracked_symbols"] == S
    assert res["value"] > 0
