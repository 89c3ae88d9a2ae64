"""bench.py's multi-rank orchestration on CPU: `bench.py --gpus 2` started WITHOUT a launcher
spawns two ranks itself (gloo here, RCCL on the GPU box), each processes its own shard, the
accumulator block is summed over the ranks, and rank 0's JSON line reports n_gpus = 2 and the
digest of a block equal to one oracle run over the union of the shards.  A launcher whose
WORLD_SIZE disagrees with --gpus is refused."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

from batch_util import run_oracle, synth_pack

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIRS = 2000


def run_bench(*extra, env=None):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--runner", "bench_cpu_runner:OracleRunner",
           "--steps", "2", "--warmup", "1", "--pairs", str(PAIRS), "--config", "C3", *extra]
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e, cwd=REPO)


def test_bench_gpus2_self_spawns_and_reduces(oracle):
    import bench
    from fqtool_amd import abi

    r = run_bench("--gpus", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["pairs_per_gpu"] == PAIRS
    p = bench.config_params(abi, "C3")
    pk = synth_pack(oracle, 2 * PAIRS, True, first=0)
    _, acc = run_oracle(oracle, p, pk)
    assert out["acc_sha256"] == hashlib.sha256(acc.tobytes()).hexdigest()
    assert abs(out["value"] - 2 * 2 * PAIRS * 2 / (out["ms_per_step"] * 2 / 1e3) / 1e6) <= 1e-3 * out["value"] + 0.006  # value is rounded to 2 decimals


def test_bench_refuses_world_size_mismatch():
    r = run_bench("--gpus", "2", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_gpus4_c5_rehearsal_equals_oracle_over_union(oracle):
    """Config 5's shape (C5 options, N ranks each owning a contiguous index range, one SUM of the
    accumulator block) at 4 ranks on gloo: the reduced block is one oracle run over the union."""
    import bench
    from fqtool_amd import abi

    r = run_bench("--gpus", "4", "--config", "C5", "--pairs", "1000")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 4 and out["config"]["pairs_per_gpu"] == 1000 and out["config"]["first_index"] == 0
    p = bench.config_params(abi, "C5")
    pk = synth_pack(oracle, 4000, True, first=0)
    _, acc = run_oracle(oracle, p, pk)
    assert out["acc_sha256"] == hashlib.sha256(acc.tobytes()).hexdigest()


def test_bench_shard_option_runs_one_rank_of_a_larger_job(oracle):
    """--shard 3/4 --pg: one process takes rank 3's index range and still runs the collective
    (a world-1 process group), the rehearsal the GPU suite runs for config 5's rank 7 of 8."""
    import bench
    from fqtool_amd import abi

    r = run_bench("--config", "C5", "--pairs", "1000", "--shard", "3/4", "--pg",
                  env={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(bench.free_port())})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["config"]["first_index"] == 3000
    assert "process group (gloo) closed" in r.stderr
    p = bench.config_params(abi, "C5")
    pk = synth_pack(oracle, 1000, True, first=3000)
    _, acc = run_oracle(oracle, p, pk)
    assert out["acc_sha256"] == hashlib.sha256(acc.tobytes()).hexdigest()
