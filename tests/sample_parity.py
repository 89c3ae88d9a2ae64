"""Large-batch parity checker: the HIP engine's output on a big HBM-resident batch against the
CPU restatement (oracle/fq_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by the full-size GPU parity tests (tests/test_fullsize_gpu.py) and by bench.py's
`parity_sample` leg, which runs after the timed region (the oracle is the checker there, never
the thing measured).

* `oracle_parallel` runs the oracle over a tiled host batch in tile-aligned chunks on a thread
  pool (ctypes releases the GIL; the oracle keeps its scratch rows thread-local) and sums the
  chunk accumulators -- the accumulator is a sum of per-read contributions, so this equals one
  sequential run (reference semantics: per-thread Stats/FilterResult merged at the end,
  src/peprocessor.cpp:179-217).
* `choose_tiles` picks a stratified tile sample of a batch: the first and last tile (ragged when
  n % 32 != 0), every k-th tile, and a few seeded random ones.
* `check_sample` gathers those tiles out of the device batch into a compact device sub-batch,
  (1) compares the full-size run's records of those tiles with the oracle's, and (2) runs the
  engine again on the sub-batch alone with a fresh accumulator and compares every record and
  every accumulator word with the oracle's over the same tiles.
"""
import concurrent.futures as cf
import ctypes
import os

import numpy as np

from fqtool_amd import abi

TILE = abi.TILE_READS


def host_threads():
    # one GPU's share of the box's host cores (gpurun: 16), whatever os.cpu_count() reports
    return max(1, min(16, os.cpu_count() or 1))


def oracle_parallel(oracle, p, planes, len1, len2, n, stride, threads=None):
    """Oracle over a tiled host batch. planes: dict seq1/qual1[/seq2/qual2] -> uint8 arrays
    (tiled, >= batch_bytes(n, stride)); returns (records, accumulator)."""
    paired = bool(p.paired)
    rpp = 2 if paired else 1
    res = np.zeros(n * rpp, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS))
    words = abi.acc_words(p.insert_size_max, p.max_cycles)
    threads = threads or host_threads()
    ntiles = -(-n // TILE)
    per = max(1, -(-ntiles // (threads * 4)))  # several chunks per thread for balance
    chunks = [(t * TILE, min(n, (t + per) * TILE)) for t in range(0, ntiles, per)]

    def run(lo_hi):
        lo, hi = lo_hi
        b = abi.FqBatch()
        b.n, b.stride = hi - lo, stride
        b.seq1 = planes["seq1"].ctypes.data + lo * stride
        b.qual1 = planes["qual1"].ctypes.data + lo * stride
        b.len1 = len1.ctypes.data + lo * 2
        if paired:
            b.seq2 = planes["seq2"].ctypes.data + lo * stride
            b.qual2 = planes["qual2"].ctypes.data + lo * stride
            b.len2 = len2.ctypes.data + lo * 2
        acc = np.zeros(words, np.uint64)
        rc = oracle.orc_process_batch(ctypes.byref(p), ctypes.byref(b), res.ctypes.data + lo * rpp * 16,
                                      acc.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"oracle rc {rc}")
        return acc

    total = np.zeros(words, np.uint64)
    with cf.ThreadPoolExecutor(threads) as ex:
        for acc in ex.map(run, chunks):
            total += acc  # u64 wrap-around addition, like the engine's atomics
    return res, total


def choose_tiles(n, target_pairs, seed=1):
    ntiles = -(-n // TILE)
    want = min(ntiles, max(2, -(-target_pairs // TILE)))
    if want >= ntiles:
        return np.arange(ntiles, dtype=np.int64)
    step = max(1, ntiles // want)
    ids = set(range(0, ntiles, step))
    rng = np.random.default_rng(seed)
    ids.update(int(x) for x in rng.integers(0, ntiles, 64))
    ids.update((0, ntiles - 1))
    return np.array(sorted(ids), dtype=np.int64)  # the (possibly ragged) last tile comes last


def gather_sample(torch, planes_dev, lens_dev, results_dev, n, stride, tile_ids, paired):
    """Device sub-batch of the given tiles: tiled planes, lengths, and the full run's records."""
    dev = planes_dev[0].device
    ntiles = -(-n // TILE)
    tb = TILE * stride
    T = torch.from_numpy(tile_ids).to(dev)
    sub_planes = [pl[: ntiles * tb].view(ntiles, tb).index_select(0, T).reshape(-1).contiguous() for pl in planes_dev]
    pidx = (T[:, None] * TILE + torch.arange(TILE, device=dev)[None, :]).reshape(-1)
    pidx = pidx[pidx < n]
    sub_lens = [l.index_select(0, pidx).contiguous() for l in lens_dev]
    rpp = 2 if paired else 1
    sub_res = None
    if results_dev is not None:
        sub_res = results_dev[: n * rpp * 16].view(n, rpp * 16).index_select(0, pidx).reshape(-1).contiguous()
    return sub_planes, sub_lens, sub_res, int(pidx.numel())


def device_batch(planes, lens, n, stride, paired):
    b = abi.FqBatch()
    b.n, b.stride = n, stride
    b.seq1, b.qual1, b.len1 = planes[0].data_ptr(), planes[1].data_ptr(), lens[0].data_ptr()
    if paired:
        b.seq2, b.qual2, b.len2 = planes[2].data_ptr(), planes[3].data_ptr(), lens[1].data_ptr()
    return b


def host_copy(torch, planes, lens, paired):
    names = ("seq1", "qual1", "seq2", "qual2") if paired else ("seq1", "qual1")
    hp = {k: t.cpu().numpy() for k, t in zip(names, planes)}
    l1 = lens[0].cpu().numpy().view(np.uint16)
    l2 = lens[1].cpu().numpy().view(np.uint16) if paired else None
    return hp, l1, l2


def first_diff(a, b):
    bad = np.nonzero(a != b)[0]
    return len(bad), (int(bad[0]) if len(bad) else None)


def engine_run(lib, torch, p, planes, lens, n, stride, paired, device_index):
    """The engine alone over a device batch: fresh accumulator, records on the device."""
    dev = planes[0].device
    h = ctypes.c_void_p()
    if lib.fq_engine_create(ctypes.byref(p), device_index, 0, 0, ctypes.byref(h)) != 0:
        raise RuntimeError(lib.fq_engine_last_error(None).decode())
    try:
        res = torch.zeros(n * (2 if paired else 1) * 16, dtype=torch.uint8, device=dev)
        b = device_batch(planes, lens, n, stride, paired)
        if lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None) != 0:
            raise RuntimeError(lib.fq_engine_last_error(h).decode())
        if lib.fq_engine_sync(h) != 0:
            raise RuntimeError(lib.fq_engine_last_error(h).decode())
        acc = np.zeros(lib.fq_engine_acc_words(h), np.uint64)
        if lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size) != 0:
            raise RuntimeError(lib.fq_engine_last_error(h).decode())
        return res, acc
    finally:
        lib.fq_engine_destroy(h)


def check_sample(lib, oracle, torch, p, planes_dev, lens_dev, results_dev, n, stride, target_pairs,
                 device_index=0, seed=1):
    """Stratified-sample parity of a full-size run (see module doc). Returns a summary dict."""
    paired = bool(p.paired)
    tiles = choose_tiles(n, target_pairs, seed)
    sp, sl, sres, ns = gather_sample(torch, planes_dev, lens_dev, results_dev, n, stride, tiles, paired)
    eres, eacc = engine_run(lib, torch, p, sp, sl, ns, stride, paired, device_index)
    hp, l1, l2 = host_copy(torch, sp, sl, paired)
    ores, oacc = oracle_parallel(oracle, p, hp, l1, l2, ns, stride)
    full = sres.cpu().numpy().view(ores.dtype) if sres is not None else None
    sub = eres.cpu().numpy().view(ores.dtype)
    nbad_full, i_full = first_diff(full, ores) if full is not None else (0, None)
    nbad_sub, i_sub = first_diff(sub, ores)
    nbad_acc, i_acc = first_diff(eacc, oacc)
    out = {
        "pairs" if paired else "reads": ns,
        "tiles": int(len(tiles)),
        "of_tiles": int(-(-n // TILE)),
        "full_run_records_equal": nbad_full == 0,
        "sample_run_records_equal": nbad_sub == 0,
        "sample_run_acc_equal": nbad_acc == 0,
        "ok": nbad_full == 0 and nbad_sub == 0 and nbad_acc == 0,
    }
    if not out["ok"]:
        out["detail"] = {"full_bad": nbad_full, "full_first": i_full, "sub_bad": nbad_sub, "sub_first": i_sub,
                         "acc_bad": nbad_acc, "acc_first": i_acc}
    return out
