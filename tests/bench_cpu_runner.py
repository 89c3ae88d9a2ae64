"""CPU stand-in for bench.py's HipRunner (tests only): lets tests/test_bench_cpu.py rehearse the
rank orchestration of `bench.py --gpus N` (self-spawned ranks, gloo process group, shard ranges,
accumulator reduction, max-over-ranks timing, the one JSON line) without a GPU.  The oracle
processes each rank's shard; the product path (HipRunner) never uses this module."""
import ctypes
import os

import numpy as np
import torch

from fqtool_amd import abi
from sample_parity import oracle_parallel

STRIDE, L, SEED = 160, 150, 20261015


class OracleRunner:
    backend = "gloo"

    def __init__(self, args, local):
        import bench
        from oracle_lib import load_oracle

        self.abi, self.args = abi, args
        self.dev = torch.device("cpu")
        self.oracle = load_oracle()
        self.p = bench.config_params(abi, args.config)
        self.paired = bool(self.p.paired)
        self.ms = []

    def alloc(self, first, n):
        self.first, self.n = first, n
        names = ("seq1", "qual1", "seq2", "qual2") if self.paired else ("seq1", "qual1")
        self.planes = {k: np.zeros(abi.batch_bytes(n, STRIDE), np.uint8) for k in names}
        self.len1 = np.zeros(n, np.uint16)
        self.len2 = np.zeros(n, np.uint16) if self.paired else None
        b = abi.FqBatch()
        b.n, b.stride = n, STRIDE
        b.seq1, b.qual1, b.len1 = self.planes["seq1"].ctypes.data, self.planes["qual1"].ctypes.data, self.len1.ctypes.data
        if self.paired:
            b.seq2, b.qual2, b.len2 = (self.planes["seq2"].ctypes.data, self.planes["qual2"].ctypes.data,
                                       self.len2.ctypes.data)
        self.oracle.orc_synth_fill(ctypes.byref(b), SEED, first, L)
        self.acc = torch.zeros(abi.acc_words(self.p.insert_size_max, self.p.max_cycles), dtype=torch.int64)

    def step(self, timed):
        import time

        t0 = time.perf_counter()
        _, acc = oracle_parallel(self.oracle, self.p, self.planes, self.len1, self.len2, self.n, STRIDE, threads=2)
        self.acc.copy_(torch.from_numpy(acc.view(np.int64)))
        if timed:
            self.ms.append((time.perf_counter() - t0) * 1e3)

    def sync(self):
        pass

    def elapsed_tensor(self, x):
        return torch.tensor([x], dtype=torch.float64)

    def kernel_ms(self):
        return sum(self.ms) / len(self.ms) if self.ms else None

    def finish(self):
        pass

    def acc_host(self):
        return self.acc.numpy().view(np.uint64)

    def parity_sample(self, target):
        return None  # the oracle is the engine here: nothing to check against

    def close(self):
        pass
