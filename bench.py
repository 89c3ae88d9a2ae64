#!/usr/bin/env python3
"""Headline benchmark: Mreads/s of the per-read hot path on MI355X.

Workload (BASELINE.json configs[2]): synthetic 150 bp paired-end reads, options
`-q -a --detect_pe_adapter -g` (quality filter + overlap adapter trimming + polyG), generated
directly in HBM by the engine's counter-based generator.  A *step* is one pass of the hot
path (fq_engine_process_device: one persistent kernel launch) over the whole resident batch,
i.e. every pair's trim/filter result record and the Stats x4 / FilterResult / insert-size
accumulators; with N ranks the accumulator block is then summed over RCCL (the only exchange
the path has).  Scaling is weak: each rank owns `--pairs` pairs (its own index range).

Launch:  python bench.py [--gpus N --steps K --warmup W]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
READ_LEN = 150
STRIDE = 160
SEED = 20261015
WORKLOADS = {
    "C2": "C2: synthetic SE 150bp, -q (BASELINE.json configs[1])",
    "C3": "C3: synthetic PE 2x150bp, -q -a --detect_pe_adapter -g (BASELINE.json configs[2])",
    "C4": "C4: synthetic PE 2x150bp, -q -a -g --enable_cut_right -m (BASELINE.json configs[3])",
    "C5": "C5: synthetic PE 2x150bp, -q -a -g -x --enable_cut_right (BASELINE.json configs[4], per GPU)",
}
WORKLOAD = WORKLOADS["C3"]


def pmc_traffic(cfg, pairs):
    """HBM bytes per launch of the fast kernel for this workload, from the latest committed PMC
    profile (tools/profile_round.sh: rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same bench
    command, corrected per MI355X_MICROARCH.md); None when no profile matches the batch size."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{cfg}.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    if int(d.get("pairs", -1)) != pairs:
        return None, None
    return int(d["traffic_bytes"]), os.path.relpath(paths[-1], REPO)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def config_params(abi, name, max_cycles=256):
    """Engine parameters of a BASELINE config (what the tool derives from its command line)."""
    p = abi.default_params(paired=name != "C2", max_cycles=max_cycles)
    p.qual_filter_enabled = 1
    if name in ("C3", "C4", "C5"):
        p.adapter_trimming = 1
        p.polyg_enabled = 1
    if name in ("C4", "C5"):
        p.cut_right = 1
    if name == "C4":
        p.merge_enabled = 1
        p.max_cycles = max(max_cycles, 320)  # merged reads reach len1 + len2
    if name == "C5":
        p.polyx_enabled = 1
    return p


def c3_params(abi, max_cycles=256):
    return config_params(abi, "C3", max_cycles)


def write_fastq_pair(seq1, qual1, seq2, qual2, first_index, d):
    """Format pairs as FASTQ files (for the reference CPU baseline run)."""
    paths = []
    for mate, (s, q) in enumerate(((seq1, qual1), (seq2, qual2)), start=1):
        path = os.path.join(d, f"r{mate}.fq")
        with open(path, "wb") as f:
            chunks = []
            for i in range(s.shape[0]):
                idx = first_index + i
                chunks.append(b"@SYN:1:1101:%d:%d %d:N:0:ACGTACGT\n%s\n+\n%s\n"
                              % (idx % 100000, idx // 100000, mate, s[i].tobytes(), q[i].tobytes()))
                if len(chunks) >= 65536:
                    f.write(b"".join(chunks))
                    chunks = []
            f.write(b"".join(chunks))
        paths.append(path)
    return paths


def cpu_baseline(lib, abi, torch, pairs):
    """Time the reference CPU path on a bounded sample of the same workload on this host."""
    import numpy as np

    ref = os.path.join(REPO, "oracle", "_ref", "fqtool_ref")
    dev = torch.device("cuda:0")
    bufs = [torch.empty(abi.batch_bytes(pairs, STRIDE), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.empty(pairs, dtype=torch.int16, device=dev) for _ in range(2)]
    b = abi.FqBatch()
    b.n, b.stride = pairs, STRIDE
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    first = 10 ** 12  # a disjoint index range
    assert lib.fq_synth_fill_device(ctypes.byref(b), SEED, first, READ_LEN, None) == 0
    torch.cuda.synchronize()
    arr = [abi.untile_rows(t.cpu().numpy(), pairs, STRIDE)[:, :READ_LEN] for t in bufs]
    del bufs
    tmp = tempfile.mkdtemp(prefix="fqbench_")
    try:
        r1, r2 = write_fastq_pair(arr[0], arr[1], arr[2], arr[3], first, tmp)
        if os.path.exists(ref):
            workers = min(16, os.cpu_count() or 1)
            cmd = [ref, "-i", r1, "-I", r2, "-o", os.path.join(tmp, "o1.fq"), "-O", os.path.join(tmp, "o2.fq"),
                   "-q", "-a", "--detect_pe_adapter", "-g", "-w", str(workers),
                   "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
            t0 = time.perf_counter()
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
            return {"value": round(2 * pairs / dt / 1e6, 4), "unit": "Mreads/s", "cores": workers,
                    "kind": "reference",
                    "sample": f"{pairs} pairs ({2 * pairs} reads) of the same synthetic workload as FASTQ on "
                              f"local disk, oracle/_ref/fqtool_ref -w {workers} (+1 reader, 2 writer threads), "
                              f"wall {dt:.2f}s incl. its adapter-detection pre-pass"}
        # no reference build: time the C restatement (single thread) on the packed sample
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from oracle_lib import load_oracle
        from batch_util import Pack, run_oracle

        oracle = load_oracle()
        pk = Pack(pairs, STRIDE, True)
        pk.seq1[:, :READ_LEN], pk.qual1[:, :READ_LEN] = arr[0], arr[1]
        pk.seq2[:, :READ_LEN], pk.qual2[:, :READ_LEN] = arr[2], arr[3]
        pk.len1[:] = READ_LEN
        pk.len2[:] = READ_LEN
        p = c3_params(abi)
        t0 = time.perf_counter()
        run_oracle(oracle, p, pk)
        dt = time.perf_counter() - t0
        return {"value": round(2 * pairs / dt / 1e6, 4), "unit": "Mreads/s", "cores": 1, "kind": "port",
                "sample": f"{pairs} pairs, oracle/fq_oracle.c single thread, in-memory packs"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=100_000_000, help="pairs per GPU (BASELINE: 100 M)")
    ap.add_argument("--cpu-pairs", type=int, default=1_000_000, help="CPU-baseline sample size (pairs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", default="C3", choices=sorted(WORKLOADS),
                    help="workload (BASELINE.json configs); the headline metric is C3")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from fqtool_amd import abi
    from fqtool_amd.dist import reduce_accumulator, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    lib = abi.load_engine()
    p = config_params(abi, args.config)
    paired = bool(p.paired)
    h = ctypes.c_void_p()
    if lib.fq_engine_create(ctypes.byref(p), local, 0, 0, ctypes.byref(h)) != 0:
        raise SystemExit("fq_engine_create: " + lib.fq_engine_last_error(None).decode())

    first, n = shard(rank, world, args.pairs)
    log(f"rank {rank}/{world}: allocating {4 * n * STRIDE / 1e9:.1f} GB of reads for {n} pairs")
    bufs = [torch.empty(abi.batch_bytes(n, STRIDE), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
    results = torch.empty(n * 2 * 16, dtype=torch.uint8, device=dev)
    acc = torch.zeros(lib.fq_engine_acc_words(h), dtype=torch.int64, device=dev)
    assert lib.fq_engine_set_acc_buffer(h, acc.data_ptr()) == 0
    b = abi.FqBatch()
    b.n, b.stride = n, STRIDE
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    stream = torch.cuda.current_stream(dev)
    sb = abi.FqBatch()  # single-end view (C2): read 1 planes only
    sb.n, sb.stride, sb.seq1, sb.qual1, sb.len1 = b.n, b.stride, b.seq1, b.qual1, b.len1
    t0 = time.time()
    assert lib.fq_synth_fill_device(ctypes.byref(b), SEED, first, READ_LEN, ctypes.c_void_p(stream.cuda_stream)) == 0
    torch.cuda.synchronize(dev)
    log(f"synthetic data generated in {time.time() - t0:.2f}s")

    def step(ev=None):
        acc.zero_()
        if ev:
            ev[0].record(stream)
        rc = lib.fq_engine_process_device(h, ctypes.byref(b if paired else sb), results.data_ptr(),
                                          ctypes.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(lib.fq_engine_last_error(h).decode())
        if ev:
            ev[1].record(stream)
        reduce_accumulator(acc)  # Stats/FilterResult/insert-size sum over RCCL (xGMI) when world > 1

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize(dev)
        log(f"warmup {i + 1}/{args.warmup}")
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = [e0.elapsed_time(e1) for e0, e1 in events]
    kavg = sum(kernel_ms) / len(kernel_ms)
    if lib.fq_engine_sync(h) != 0:
        raise RuntimeError(lib.fq_engine_last_error(h).decode())

    acc_host = acc.cpu().numpy().view("uint64")
    total_pairs = n * world
    reads = (2 if paired else 1) * total_pairs
    # sanity: every pair (read) was counted by the pre-filter stats and by FilterResult
    st0 = abi.acc_stats_offset(p.insert_size_max, p.max_cycles, 0)
    assert int(acc_host[st0 + abi.FQ_ST_READS]) == total_pairs, "accumulator lost pairs"
    assert int(acc_host[abi.FQ_ACC_FILTER:abi.FQ_ACC_FILTER + 32].sum()) == reads

    value = reads * args.steps / elapsed / 1e6
    traffic, traffic_src = pmc_traffic(args.config, args.pairs) if world == 1 else (None, None)
    bytes_per_pair = (2 if paired else 1) * (2 * READ_LEN + 16)  # seq+qual uint8 + 16 B result per read
    achieved = n * bytes_per_pair / (kavg / 1e3) / 1e9
    out = {
        "metric": "Mreads/s (150 bp PE, q+adapter+polyG)" if args.config == "C3" else f"Mreads/s ({args.config})",
        "value": round(value, 2),
        "unit": "Mreads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded counter-based generator in HBM, SURVEY.md 8(d))",
        "config": {"workload": WORKLOADS[args.config], ("pairs_per_gpu" if paired else "reads_per_gpu"): n, "read_len": READ_LEN, "row_stride": STRIDE,
                   "parallelism": f"dp{world} (pairs sharded, RCCL sum of the accumulator block)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_unit": "bytes per launch (PMC)", "traffic_src": traffic_src,
                     "algorithmic_bytes": n * bytes_per_pair,
                     "kernel_ms_avg": round(kavg, 3),
                     ("bytes_per_pair" if paired else "bytes_per_read"): bytes_per_pair},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "C3":
        del bufs, lens, results
        torch.cuda.empty_cache()
        log(f"CPU baseline on {args.cpu_pairs} pairs ...")
        out["cpu_baseline"] = cpu_baseline(lib, abi, torch, args.cpu_pairs)
    lib.fq_engine_destroy(h)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
