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
