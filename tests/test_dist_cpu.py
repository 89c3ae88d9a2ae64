"""The N>1 path on CPU: two gloo ranks each process their own shard of the synthetic workload
(the oracle stands in for the engine), reduce the accumulator block with the same function
bench.py uses, and rank 0 checks the result equals one process over the union of the shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

TESTS = os.path.dirname(os.path.abspath(__file__))
N = 3000


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(TESTS))
    sys.path.insert(0, TESTS)
    from batch_util import config, run_oracle, synth_pack
    from fqtool_amd.dist import merge_adapter_counts, reduce_accumulator, shard
    from oracle_lib import load_oracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        orc = load_oracle()
        p = config("C3b", max_cycles=160)
        first, n = shard(rank, world, N)
        pk = synth_pack(orc, n, True, first=first)
        res, acc = run_oracle(orc, p, pk)
        t = torch.from_numpy(acc.view(np.int64).copy())
        reduce_accumulator(t)
        counts = merge_adapter_counts({"rank%d" % rank: 1, "shared": int(res["ad_len"].sum())})
        if rank == 0:
            np.save(out + ".acc.npy", t.numpy().view(np.uint64))
            np.save(out + ".counts.npy", np.array([counts["rank0"], counts["rank1"], counts["shared"]]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_reduce_equals_single_process(world, oracle, tmp_path):
    from batch_util import config, run_oracle, synth_pack

    out = str(tmp_path / "r")
    mp.spawn(worker, args=(world, free_port(), out), nprocs=world, join=True)
    got = np.load(out + ".acc.npy")
    p = config("C3b", max_cycles=160)
    pk = synth_pack(oracle, N * world, True, first=0)
    res, want = run_oracle(oracle, p, pk)
    assert np.array_equal(got, want)
    c = np.load(out + ".counts.npy")
    assert c[0] == 1 and c[1] == 1 and c[2] == int(res["ad_len"].sum())


def test_shard_ranges():
    from fqtool_amd.dist import shard

    assert [shard(r, 4, 10) for r in range(4)] == [(0, 10), (10, 10), (20, 10), (30, 10)]
    with pytest.raises(ValueError):
        shard(4, 4, 10)
