"""Config 5 (BASELINE.json configs[4]: 1 B pairs, C5 options, 8 GPUs, RCCL Stats reduce) as far as
one GPU goes: bench.py runs rank 7's full 125 M-pair shard (global pair indices 875 M .. 1 B) on
this GPU through a real (world-1) RCCL process group, so the accumulator all-reduce of the
product path runs on hardware, and its post-timing parity sample of that shard must agree with
the oracle (the checker).  The driver's 8-GPU SCALE run launches the same code with 8 ranks."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config5_rank7_shard_through_rccl():
    import bench

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(bench.free_port()))
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--config", "C5", "--pairs", "125000000",
           "--shard", "7/8", "--pg", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--engine-pairs", "0", "--paths-pairs", "0", "--sample-pairs", "1000000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=840, env=env, cwd=REPO)
    sys.stderr.write(r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["pairs_per_gpu"] == 125_000_000
    assert out["config"]["first_index"] == 875_000_000
    assert "process group (nccl) closed" in r.stderr
    s = out["parity_sample"]
    assert s["ok"] and s["full_run_records_equal"] and s["sample_run_acc_equal"], s
    assert out["roofline"]["frac"] > 0
