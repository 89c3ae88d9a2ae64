#!/usr/bin/env python3
"""Headline benchmark: Mreads/s of the per-read hot path on MI355X.

Workload (BASELINE.json configs[2]): synthetic 150 bp paired-end reads, options
`-q -a --detect_pe_adapter -g` (quality filter + overlap adapter trimming + polyG), generated
directly in HBM by the engine's counter-based generator.  A *step* is one pass of the hot
path (fq_engine_process_device: one persistent kernel launch) over the whole resident batch,
i.e. every pair's trim/filter result record and the Stats x4 / FilterResult / insert-size
accumulators; with N ranks the accumulator block is then summed over RCCL (the only exchange
the path has).  Scaling is weak: each rank owns `--pairs` pairs (its own index range).

Launch:  python bench.py [--gpus N --steps K --warmup W] [--config C2|C3|C4|C5]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Without a launcher, --gpus N > 1 spawns the N rank processes itself (before any GPU call); under
a launcher WORLD_SIZE must equal N or the run stops.  Rank 0 prints ONE JSON line.  After the
timed region each rank checks a stratified sample of its shard against the CPU restatement
(`parity_sample`: the oracle as checker, never timed) and the run fails if any rank differs.
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
SIMDS = 1024  # 256 CUs x 4 SIMD-32
CLOCK_HZ = 2.4e9  # MI355X max shader clock
PCIE_PEAK_GBS = 64.0  # PCIe 5.0 x16, one direction (host <-> MI355X)
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


def e2e_path(tool_log, gz_input=False):
    """What the e2e run did, from the tool's own log lines: the raw stream (GPU record indexing and
    output text), text packs (host parse, device planes and text) or host packs."""
    text = " ".join(tool_log or [])
    if "raw stream" in text:
        mid = "pread into page-locked windows -> GPU record indexing -> kernels -> GPU output text"
    elif "text packs" in text:
        mid = "host parse -> text packs -> device planes -> kernels -> GPU output text"
    else:
        mid = "host parse -> pinned tile packs -> kernels -> records -> host formatting"
    src = "gzip FASTQ (page cache) -> chunks inflated on several threads" if gz_input else "FASTQ (page cache)"
    return f"fqtool binary: {src} -> {mid} -> /dev/null + JSON"


def sq_profile(cfg, pairs):
    """VALU wave-instructions per launch of the fast kernel for this workload, from the latest
    committed SQ counter profile (tools/pmc_sq.sh + tools/pmc_sq_summary.py: rocprofv3 --pmc
    SQ_INSTS_VALU ... passes of this bench command); (None, None) when no profile matches."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_sq_{cfg}.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    if int(d.get("pairs", d.get("reads", -1))) != pairs:
        return None, None
    return d, os.path.relpath(paths[-1], REPO)


def isa_cpi(cfg):
    """Average issue cycles per VALU instruction of this workload's fast-kernel instantiation, from the
    latest committed static ISA budget (tools/isa_budget.py: every instruction of the tile loop priced
    with the opcode costs measured on gfx950, profiles/r04_micro_opcost2.txt): (value, source) or
    (None, None)."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_isa_cpi.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    e = d.get(cfg)
    return (e["cycles_per_valu"], os.path.relpath(paths[-1], REPO)) if e else (None, None)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def config_params(abi, name, max_cycles=256):
    """Engine parameters of a BASELINE config (what the tool derives from its command line)."""
    max_cycles = max(max_cycles, READ_LEN)
    p = abi.default_params(paired=name != "C2", max_cycles=max_cycles)
    p.qual_filter_enabled = 1
    if name in ("C3", "C4", "C5"):
        p.adapter_trimming = 1
        p.polyg_enabled = 1
    if name in ("C4", "C5"):
        p.cut_right = 1
    if name == "C4":
        p.merge_enabled = 1
        p.max_cycles = max(max_cycles, 2 * READ_LEN, 320)  # merged reads reach len1 + len2
    if name == "C5":
        p.polyx_enabled = 1
    return p


def c3_params(abi, max_cycles=256):
    return config_params(abi, "C3", max_cycles)


def write_fastq_fast(planes, n, first_index, d, tag=""):
    """Format n pairs (tiled device planes: seq1, qual1, seq2, qual2) as two FASTQ files of
    fixed-width records, vectorised (numpy), chunk by chunk:
    @SYN:1:1101:<idx % 100000, 5 digits>:<idx // 100000, 7 digits> <mate>:N:0:ACGTACGT"""
    import numpy as np

    from fqtool_amd import abi

    L = READ_LEN
    head = b"@SYN:1:1101:"
    name_len = len(head) + 5 + 1 + 7 + len(b" 1:N:0:ACGTACGT")
    rec_len = name_len + 1 + L + 3 + L + 1
    paths = [os.path.join(d, f"{tag}r{m}.fq") for m in (1, 2)]
    files = [open(p_, "wb") for p_ in paths]
    try:
        step = 1 << 20  # pairs per chunk (multiple of the tile size)
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            k = hi - lo
            idx = np.arange(first_index + lo, first_index + hi, dtype=np.int64)
            digits = []
            for v, w in ((idx % 100000, 5), (idx // 100000, 7)):
                digits.append(np.stack([(v // 10 ** (w - 1 - j)) % 10 + 48 for j in range(w)], 1).astype(np.uint8))
            for m in range(2):
                rec = np.empty((k, rec_len), np.uint8)
                o = 0
                rec[:, o:o + len(head)] = np.frombuffer(head, np.uint8)
                o += len(head)
                rec[:, o:o + 5] = digits[0]
                o += 5
                rec[:, o] = ord(":")
                o += 1
                rec[:, o:o + 7] = digits[1]
                o += 7
                tail = b" %d:N:0:ACGTACGT\n" % (m + 1)
                rec[:, o:o + len(tail)] = np.frombuffer(tail, np.uint8)
                o += len(tail)
                sl = slice(lo * STRIDE, lo * STRIDE + abi.batch_bytes(k, STRIDE))
                seq = abi.untile_rows(planes[2 * m][sl].cpu().numpy(), k, STRIDE)[:, :L]
                qual = abi.untile_rows(planes[2 * m + 1][sl].cpu().numpy(), k, STRIDE)[:, :L]
                rec[:, o:o + L] = seq
                o += L
                rec[:, o:o + 3] = np.frombuffer(b"\n+\n", np.uint8)
                o += 3
                rec[:, o:o + L] = qual
                o += L
                rec[:, o] = 10
                files[m].write(rec)  # (buffer protocol: no extra copy)
    finally:
        for f in files:
            f.flush()
            os.fsync(f.fileno())  # (written back before any timed run reads them: no writeback in the timing)
            f.close()
    return paths


def gzip_single_member(src, dst, nbytes=None, level=6, threads=None, piece=64 << 20):
    """The first `nbytes` of `src` (all of it by default) as ONE gzip member (one deflate stream,
    not BGZF), compressed at `level` by zlib on `threads` threads as pigz does: each 64 MiB piece is
    deflated with the previous piece's last 32 KiB as its dictionary (so matches reach back across
    pieces as in one `gzip -6` stream) and ends in a full flush (an empty stored block), so the
    pieces join into a single stream; CRC32 and ISIZE of the whole.  Made in seconds instead of
    minutes."""
    import concurrent.futures as cf
    import struct
    import zlib

    total = os.path.getsize(src) if nbytes is None else nbytes
    threads = threads or host_cores()

    def deflate(args):
        data, last, dictionary = args
        if dictionary:
            c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, dictionary)
        else:
            c = zlib.compressobj(level, zlib.DEFLATED, -15, 8)
        return c.compress(data) + c.flush(zlib.Z_FINISH if last else zlib.Z_FULL_FLUSH)

    crc = 0
    with open(src, "rb") as f, open(dst, "wb") as g, cf.ThreadPoolExecutor(threads) as ex:
        g.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03")
        pending = []
        done = 0
        tail = b""
        while done < total or pending:
            while done < total and len(pending) < 2 * threads:  # (bounded: 2 pieces a thread in flight)
                data = f.read(min(piece, total - done))
                if not data:
                    raise ValueError(f"{src}: shorter than {total} bytes")
                done += len(data)
                crc = zlib.crc32(data, crc)
                pending.append(ex.submit(deflate, (data, done >= total, tail)))
                tail = data[-32768:]
            g.write(pending.pop(0).result())
        g.write(struct.pack("<II", crc & 0xFFFFFFFF, total & 0xFFFFFFFF))
    return dst


def host_cores():
    """Host cores this process may use (the GPU box's share is 16 per GPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def port_baseline(abi, pairs, first, threads):
    """CPU baseline leg (checker code, never the product): oracle/fq_oracle.c, the C restatement of
    the per-read path, on `pairs` synthetic pairs split over `threads` threads (ctypes drops the
    GIL, so the slices run in parallel), in-memory packs, no FASTQ parse or formatting."""
    import threading

    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_lib import load_oracle
    from batch_util import Pack, run_oracle

    oracle = load_oracle()
    per = -(-pairs // threads)
    packs = []
    for t in range(threads):
        n = min(per, pairs - t * per)
        if n <= 0:
            break
        pk = Pack(n, STRIDE, True)
        oracle.orc_synth_fill(ctypes.byref(pk.batch()), SEED, first + t * per, READ_LEN)
        pk.load_batch()
        packs.append(pk)
    p = c3_params(abi)
    th = [threading.Thread(target=run_oracle, args=(oracle, p, pk)) for pk in packs]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    return {"value": round(2 * pairs / dt / 1e6, 4), "unit": "Mreads/s", "cores": len(packs), "kind": "port",
            "sample": f"{pairs} pairs of the same synthetic workload, oracle/fq_oracle.c on {len(packs)} threads "
                      f"(no -w cap), in-memory packs, wall {dt:.2f}s"}


E2E_PAUSE_S = 2.0  # between e2e runs (host_legs)
GZ_IN_PAIRS = 10_000_000  # pairs of the gzip-input e2e leg


def host_legs(lib, abi, torch, cpu_pairs, e2e_pairs, workers):
    """Rank 0 at N=1, after the timed region: both host-side legs on FASTQ files of the same
    synthetic workload (fixed-width records, page cache):
      e2e          -- the fqtool-amd binary end to end (parse, pinned packs, engine on cuda:0,
                      formatting, writers, JSON) on `e2e_pairs` pairs, outputs to /dev/null;
      cpu_baseline -- the reference binary (oracle/_ref/fqtool_ref, -w <= 16) on the first
                      `cpu_pairs` pairs (or, without it, the C restatement single-threaded)."""
    n = max(cpu_pairs, e2e_pairs)
    gz_pairs = min(GZ_IN_PAIRS, e2e_pairs)
    tmp = tempfile.mkdtemp(prefix="fqbench_")
    rec_bytes = 2 * (40 + 2 * READ_LEN + 5)
    free = shutil.disk_usage(tmp).free
    if (e2e_pairs + cpu_pairs) * rec_bytes * 1.2 > free:  # keep to the space the box has
        e2e_pairs = max(0, min(e2e_pairs, int(free / 1.2 / rec_bytes) - cpu_pairs))
        n = max(cpu_pairs, e2e_pairs)
    dev = torch.device("cuda:0")
    bufs = [torch.empty(abi.batch_bytes(n, STRIDE), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
    b = abi.FqBatch()
    b.n, b.stride = n, STRIDE
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    first = 10 ** 12  # a disjoint index range
    assert lib.fq_synth_fill_device(ctypes.byref(b), SEED, first, READ_LEN, None) == 0
    torch.cuda.synchronize()
    out = {"e2e": None, "cpu_baseline": None}
    shm = None
    try:
        t0 = time.perf_counter()
        small = write_fastq_fast(bufs, cpu_pairs, first, tmp, "cpu_")
        big = write_fastq_fast(bufs, e2e_pairs, first, tmp, "e2e_") if e2e_pairs else None
        del bufs, lens
        torch.cuda.empty_cache()
        os.sync()  # (the files' dirty pages written back now, not during the first timed run)
        log(f"FASTQ written in {time.perf_counter() - t0:.1f}s ({cpu_pairs} + {e2e_pairs} pairs)")
        # the file leg's outputs go beside the inputs: room for one run's outputs (about the inputs' size)
        free = shutil.disk_usage(tmp).free
        file_legs = e2e_pairs * rec_bytes * 1.1 < free
        # tmpfs for the output legs without disk write-back: room for one run's plain outputs
        # (about the inputs' size) besides what the box's memory holds already
        shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
        if shm and shutil.disk_usage(shm).free < e2e_pairs * rec_bytes * 1.3:
            log(f"tmpfs legs skipped: {shutil.disk_usage(shm).free / 1e9:.1f} GB free in /dev/shm")
            shm = None
        if shm:
            shm = tempfile.mkdtemp(prefix="fqbench_", dir=shm)
        if not file_legs:
            log(f"file legs skipped: {free / 1e9:.1f} GB free beside the inputs")
        opts = ["-q", "-a", "--detect_pe_adapter", "-g"]

        def e2e(extra, outputs="null", inp=None, pairs=None):
            """outputs: "null" (/dev/null), "file" (plain FASTQ files beside the inputs: the writer
            threads put every output byte into the page cache), "gz" (BGZF .gz files, members
            compressed on the pool; src/writer.cpp's gzip output)"""
            tool = os.path.join(REPO, "fqtool_amd", "bin", "fqtool")
            inp = inp or big
            pairs = pairs or e2e_pairs
            outs = {"null": ["/dev/null", "/dev/null"],
                    "file": [os.path.join(tmp, "out1.fq"), os.path.join(tmp, "out2.fq")],
                    "gz": [os.path.join(tmp, "out1.fq.gz"), os.path.join(tmp, "out2.fq.gz")],
                    "shm": [os.path.join(shm or tmp, "out1.fq"), os.path.join(shm or tmp, "out2.fq")],
                    "gz_shm": [os.path.join(shm or tmp, "out1.fq.gz"), os.path.join(shm or tmp, "out2.fq.gz")]}[outputs]
            if "--merge_output" in extra and outputs != "null":
                extra = [outs[0] if (k > 0 and extra[k - 1] == "--merge_output") else a for k, a in enumerate(extra)]
            cmd = [tool, "-i", inp[0], "-I", inp[1], "-o", outs[0], "-O", outs[1], *extra, "-w", str(workers),
                   "-J", os.path.join(tmp, "amd.json"), "-H", os.path.join(tmp, "amd.html")]
            # one untimed run first, on the small sample: the binary's first start on a box (its
            # libraries and code objects read in, the GPU's first process setup) is not the pipeline
            warm = [tool, "-i", small[0], "-I", small[1], "-o", "/dev/null", "-O", "/dev/null", *extra, "-w", str(workers),
                    "-J", os.path.join(tmp, "warm.json"), "-H", os.path.join(tmp, "warm.html")]
            subprocess.run(warm if small else cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            runs = []  # three runs (the copy pipeline's run-to-run spread is wide): the median is reported
            for _ in range(3):
                # each run starts as a separate invocation would: the kernel's GPU driver releases a finished
                # process's GPU memory and page-locked pages after its exit, and a process started
                # while that is still going finds HIP's start-up 0.1-0.15 s slower
                # (profiles/r04_e2e_pause_50M.txt)
                time.sleep(E2E_PAUSE_S)
                for f in outs:  # (each run writes its outputs afresh)
                    if f != "/dev/null" and os.path.exists(f):
                        os.remove(f)
                t0 = time.perf_counter()
                p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
                dt = time.perf_counter() - t0
                if p.returncode != 0:
                    raise RuntimeError("fqtool failed: " + p.stderr[-2000:])
                runs.append((dt, [l for l in p.stderr.splitlines() if "fqtool-amd:" in l]))
            out_bytes = sum(os.path.getsize(f) for f in set(outs) if f != "/dev/null" and os.path.exists(f))
            for f in outs:
                if f != "/dev/null" and os.path.exists(f):
                    os.remove(f)
            dt, tool_log = sorted(runs, key=lambda r: r[0])[1]
            gb = (os.path.getsize(inp[0]) + os.path.getsize(inp[1])) / 1e9
            r = {"value": round(2 * pairs / dt / 1e6, 3), "unit": "Mreads/s", "pairs": pairs,
                 "fastq_GB_s": round(gb / dt, 3), "wall_s": round(dt, 3), "workers": workers,
                 "runs_wall_s": [round(r[0], 3) for r in runs], "pause_between_runs_s": E2E_PAUSE_S,
                 "options": " ".join(extra), "outputs": outputs, "affinity_cpus": host_cores(),
                 "path": e2e_path(tool_log, gz_input=inp[0].endswith(".gz")),
                 "tool_log": tool_log[-1].split("] ", 1)[-1] if tool_log else None}
            if outputs != "null":
                r["output_GB"] = round(out_bytes / 1e9, 3)
            return r

        if big:
            out["e2e"] = e2e(opts)
            # BASELINE config 4 (-m): every pair's output is the merged stream (to /dev/null)
            out["e2e_c4"] = e2e(["-q", "-a", "-g", "--enable_cut_right", "-m", "--merge_output", "/dev/null"])
            # gzip inputs: the first GZ_IN_PAIRS pairs as single-member gzip -6 files (one deflate
            # stream each, as gzip writes -- not BGZF), inflated by the tool on several threads
            if os.environ.get("FQ_BENCH_GZ_IN", "1") != "0" and gz_pairs:
                t0 = time.perf_counter()
                gzin = [gzip_single_member(p_, p_ + ".gz", nbytes=os.path.getsize(p_) // e2e_pairs * gz_pairs)
                        for p_ in big]
                gz_gb = sum(os.path.getsize(p_) for p_ in gzin) / 1e9
                log(f"gzip -6 inputs made in {time.perf_counter() - t0:.1f}s ({gz_pairs} pairs, {gz_gb:.2f} GB)")
                out["e2e_gzin"] = e2e(opts, inp=gzin, pairs=gz_pairs)
                out["e2e_gzin"]["input"] = (f"{gz_pairs} pairs as two single-member gzip -6 files ({gz_gb:.2f} GB "
                                            f"compressed; 64 MiB pieces joined by full flushes)")
                for p_ in gzin:
                    os.remove(p_)
            # the writers timed: the same C3 run with plain FASTQ output files (page cache), and
            # BGZF .gz outputs (-z 4, the reference's default level) on the CPU-baseline sample
            if os.environ.get("FQ_BENCH_FILE_LEGS", "1") != "0":
                if file_legs:
                    out["e2e_file"] = e2e(opts, outputs="file")
                if shm:
                    # the same outputs on tmpfs (no disk write-back in the timing), and BGZF .gz
                    # outputs at -z 4 on the whole e2e input (members compressed with libdeflate
                    # on the pool)
                    out["e2e_file_shm"] = e2e(opts, outputs="shm")
                    out["e2e_gz"] = e2e(opts, outputs="gz_shm")
                elif file_legs:
                    out["e2e_gz"] = e2e(opts, outputs="gz", inp=small, pairs=cpu_pairs)
        ref = os.path.join(REPO, "oracle", "_ref", "fqtool_ref")
        if os.path.exists(ref):
            w = min(16, workers)
            cmd = [ref, "-i", small[0], "-I", small[1], "-o", "/dev/null", "-O", "/dev/null", *opts, "-w", str(w),
                   "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
            t0 = time.perf_counter()
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {
                "value": round(2 * cpu_pairs / dt / 1e6, 4), "unit": "Mreads/s", "cores": w, "kind": "reference",
                "sample": f"{cpu_pairs} pairs ({2 * cpu_pairs} reads) of the same synthetic workload as FASTQ in the "
                          f"page cache, oracle/_ref/fqtool_ref -w {w} (+1 reader, 2 writer threads), wall {dt:.2f}s "
                          f"incl. its adapter-detection pre-pass"}
            # the reference on the same sample as single-member gzip -6 inputs (zlib's gzread, one
            # thread per file): the baseline of the e2e_gzin leg
            if os.environ.get("FQ_BENCH_GZ_IN", "1") != "0":
                sgz = [gzip_single_member(p_, p_ + ".gz") for p_ in small]
                cmd = [ref, "-i", sgz[0], "-I", sgz[1], "-o", "/dev/null", "-O", "/dev/null", *opts, "-w", str(w),
                       "-J", os.path.join(tmp, "r.json"), "-H", os.path.join(tmp, "r.html")]
                t0 = time.perf_counter()
                subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                dt = time.perf_counter() - t0
                out["cpu_baseline"]["gzin"] = {
                    "value": round(2 * cpu_pairs / dt / 1e6, 4), "unit": "Mreads/s", "wall_s": round(dt, 3),
                    "sample": f"the same {cpu_pairs} pairs as single-member gzip -6 files, oracle/_ref/fqtool_ref -w {w}"}
            # the same sample through the C restatement's per-read path (no parse/format) on one
            # thread per host core of the box's share -- the reference CLI caps -w at 16
            # (src/main.cpp:110); this run has no cap
            out["cpu_baseline"]["port_threads"] = port_baseline(abi, cpu_pairs, first, host_cores())
        else:  # no reference build: the C restatement on the packed sample
            out["cpu_baseline"] = port_baseline(abi, cpu_pairs, first, host_cores())
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
        if shm:
            shutil.rmtree(shm, ignore_errors=True)
    return out


class HipRunner:
    """One rank of the product path: libfqengine.so (HIP kernels for gfx950) on one GPU, its
    shard of the synthetic workload resident in HBM (generated in place)."""

    backend = "nccl"

    def __init__(self, args, local):
        import torch

        from fqtool_amd import abi

        self.torch, self.abi, self.args = torch, abi, args
        ndev = torch.cuda.device_count()
        if local >= ndev:  # each rank checks its own device (the launcher never touches the GPU)
            raise SystemExit(f"bench: rank needs cuda:{local} but only {ndev} GPUs are visible")
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.local = local
        self.lib = abi.load_engine()
        self.p = config_params(abi, args.config)
        self.paired = bool(self.p.paired)
        h = ctypes.c_void_p()
        if self.lib.fq_engine_create(ctypes.byref(self.p), local, 0, 0, ctypes.byref(h)) != 0:
            raise SystemExit("fq_engine_create: " + self.lib.fq_engine_last_error(None).decode())
        self.h = h
        self.events = []

    def alloc(self, first, n):
        torch, abi = self.torch, self.abi
        self.first, self.n = first, n
        np_ = 4 if self.paired else 2
        log(f"cuda:{self.local}: allocating {np_ * abi.batch_bytes(n, STRIDE) / 1e9:.1f} GB of reads for {n} "
            f"{'pairs' if self.paired else 'reads'}")
        self.planes = [torch.empty(abi.batch_bytes(n, STRIDE), dtype=torch.uint8, device=self.dev) for _ in range(np_)]
        self.lens = [torch.empty(n, dtype=torch.int16, device=self.dev) for _ in range(np_ // 2)]
        self.results = torch.empty(n * (2 if self.paired else 1) * 16, dtype=torch.uint8, device=self.dev)
        self.acc = torch.zeros(self.lib.fq_engine_acc_words(self.h), dtype=torch.int64, device=self.dev)
        assert self.lib.fq_engine_set_acc_buffer(self.h, self.acc.data_ptr()) == 0
        b = abi.FqBatch()
        b.n, b.stride = n, STRIDE
        b.seq1, b.qual1, b.len1 = self.planes[0].data_ptr(), self.planes[1].data_ptr(), self.lens[0].data_ptr()
        if self.paired:
            b.seq2, b.qual2, b.len2 = self.planes[2].data_ptr(), self.planes[3].data_ptr(), self.lens[1].data_ptr()
        self.batch = b
        self.stream = torch.cuda.current_stream(self.dev)
        t0 = time.time()
        assert self.lib.fq_synth_fill_device(ctypes.byref(b), SEED, first, READ_LEN,
                                             ctypes.c_void_p(self.stream.cuda_stream)) == 0
        torch.cuda.synchronize(self.dev)
        log(f"cuda:{self.local}: synthetic shard generated in {time.time() - t0:.2f}s")

    def step(self, timed):
        """One pass of the hot path over the whole resident shard: every record + accumulators.
        HIP events on the launch stream bracket the engine launch (kernel time for roofline)."""
        self.acc.zero_()
        ev = None
        if timed:
            ev = (self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True))
            ev[0].record(self.stream)
        rc = self.lib.fq_engine_process_device(self.h, ctypes.byref(self.batch), self.results.data_ptr(),
                                               ctypes.c_void_p(self.stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(self.lib.fq_engine_last_error(self.h).decode())
        if ev:
            ev[1].record(self.stream)
            self.events.append(ev)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def elapsed_tensor(self, x):
        return self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)

    def kernel_ms(self):
        ms = [a.elapsed_time(b) for a, b in self.events]
        return sum(ms) / len(ms) if ms else None

    def finish(self):
        if self.lib.fq_engine_sync(self.h) != 0:
            raise RuntimeError(self.lib.fq_engine_last_error(self.h).decode())

    def acc_host(self):
        return self.acc.cpu().numpy().view("uint64")

    def parity_sample(self, target):
        """CHECKER leg (after the timed region): a stratified tile sample of this rank's shard,
        the full run's records and a re-run's accumulator vs the CPU restatement (oracle/)."""
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from oracle_lib import load_oracle
        from sample_parity import check_sample

        return check_sample(self.lib, load_oracle(), self.torch, self.p, self.planes, self.lens, self.results,
                            self.n, STRIDE, target, device_index=self.local, seed=self.first + 1)

    def engine_leg(self, pack_pairs, packs=4, rounds=4):
        """The host-pack path (what the fqtool binary drives): page-locked host packs of
        `pack_pairs` pairs go through fq_engine_submit/poll -- H2D on a copy stream, kernels,
        D2H of the 16-byte records -- with up to 3 packs in flight, so copies of pack k+1
        overlap the kernels of pack k.  Rate includes PCIe both ways; parse/format excluded."""
        import numpy as np

        abi, lib, torch = self.abi, self.lib, self.torch
        pp = min(pack_pairs, self.n) // abi.TILE_READS * abi.TILE_READS
        packs = max(1, min(packs, self.n // pp))
        h = ctypes.c_void_p()
        if lib.fq_engine_create(ctypes.byref(self.p), self.local, pp, STRIDE, ctypes.byref(h)) != 0:
            raise RuntimeError(lib.fq_engine_last_error(None).decode())
        rpp = 2 if self.paired else 1
        plane_bytes = abi.batch_bytes(pp, STRIDE)
        host = []
        try:
            for k in range(packs):
                bufs = []
                for nbytes in [plane_bytes] * len(self.planes) + [pp * 2] * len(self.lens) + [pp * rpp * 16]:
                    ptr = ctypes.c_void_p()
                    if lib.fq_host_alloc(nbytes, ctypes.byref(ptr)) != 0:
                        raise RuntimeError("fq_host_alloc failed")
                    host.append(ptr)
                    bufs.append((ptr, nbytes))
                lo = k * pp  # pack k = pairs [k*pp, (k+1)*pp) of the resident shard (tile aligned)
                srcs = [pl[lo * STRIDE: lo * STRIDE + plane_bytes] for pl in self.planes] + \
                       [l[lo: lo + pp] for l in self.lens]
                for (ptr, nbytes), t in zip(bufs, srcs):
                    a = t.cpu().numpy()
                    ctypes.memmove(ptr.value, a.ctypes.data, nbytes)
                b = abi.FqBatch()
                b.n, b.stride = pp, STRIDE
                b.seq1, b.qual1 = bufs[0][0].value, bufs[1][0].value
                if self.paired:
                    b.seq2, b.qual2 = bufs[2][0].value, bufs[3][0].value
                    b.len1, b.len2 = bufs[4][0].value, bufs[5][0].value
                else:
                    b.len1 = bufs[2][0].value
                host.append((b, bufs[-1][0]))

            batches = [x for x in host if isinstance(x, tuple)]

            def run(n_rounds):
                seq = ctypes.c_uint64()
                for r in range(n_rounds):
                    for k, (b, res) in enumerate(batches):
                        if lib.fq_engine_pending(h) >= min(3, len(batches)):
                            if lib.fq_engine_poll(h, 1, ctypes.byref(seq)) != 1:
                                raise RuntimeError(lib.fq_engine_last_error(h).decode())
                        if lib.fq_engine_submit(h, ctypes.byref(b), res, r * len(batches) + k) != 0:
                            raise RuntimeError(lib.fq_engine_last_error(h).decode())
                while lib.fq_engine_pending(h) > 0:
                    if lib.fq_engine_poll(h, 1, ctypes.byref(seq)) != 1:
                        raise RuntimeError(lib.fq_engine_last_error(h).decode())

            run(1)
            t0 = time.perf_counter()
            run(rounds)
            dt = time.perf_counter() - t0
            pairs = pp * len(batches) * rounds
            h2d = pairs * (len(self.planes) * STRIDE + len(self.lens) * 2)
            d2h = pairs * rpp * 16
            return {"value": round(rpp * pairs / dt / 1e6, 2), "unit": "Mreads/s",
                    "pack_pairs" if self.paired else "pack_reads": pp, "packs": pairs // pp,
                    "h2d_GBps": round(h2d / dt / 1e9, 2), "d2h_GBps": round(d2h / dt / 1e9, 2),
                    "pcie_peak_GBps": PCIE_PEAK_GBS,
                    "path": "page-locked host packs: fq_engine_submit (H2D on a copy stream) -> kernels -> "
                            "D2H of the records, <= 3 packs in flight; FASTQ parse/format not included"}
        finally:
            lib.fq_engine_destroy(h)
            for x in host:
                if not isinstance(x, tuple):
                    lib.fq_host_free(x)

    def paths_leg(self, pairs):
        """Off the BASELINE configs: C3's options with explicit adapter sequences (C3b, trimBySequence),
        with UMI (8 + 8), with -c, C4's with -c, and with 1 % of the
        pairs holding a lowercase base, then an IUPAC code (handed to the general kernel), on the first
        `pairs` pairs of the resident shard; kernel ms per launch from HIP events on the launch
        stream (median of 3 after a warm-up).  Runs after every check: -c rewrites corrected
        bases in place and the lowercase bases are written into the shard."""
        abi, lib, torch = self.abi, self.lib, self.torch
        n = min(pairs, self.n) // abi.TILE_READS * abi.TILE_READS
        b = abi.FqBatch()
        for f, _ in abi.FqBatch._fields_:
            setattr(b, f, getattr(self.batch, f))
        b.n = n
        out = {"pairs": n, "unit": "Mreads/s (kernels, HBM-resident)"}

        def timed(p, label):
            h = ctypes.c_void_p()
            if lib.fq_engine_create(ctypes.byref(p), self.local, 0, 0, ctypes.byref(h)) != 0:
                raise RuntimeError(lib.fq_engine_last_error(None).decode())
            try:
                ms = []
                for i in range(4):
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record(self.stream)
                    if lib.fq_engine_process_device(h, ctypes.byref(b), self.results.data_ptr(),
                                                    ctypes.c_void_p(self.stream.cuda_stream)) != 0:
                        raise RuntimeError(lib.fq_engine_last_error(h).decode())
                    ev[1].record(self.stream)
                    torch.cuda.synchronize(self.dev)
                    if i:
                        ms.append(ev[0].elapsed_time(ev[1]))
                ms.sort()
                out[label] = {"ms": round(ms[1], 3), "value": round(2 * n / ms[1] / 1e3, 1)}
            finally:
                lib.fq_engine_destroy(h)

        timed(config_params(abi, "C3"), "c3")
        p = config_params(abi, "C3")  # C3b: explicit adapters (-a/--adapter_sequence_r2: trimBySequence)
        abi.set_adapter(p, 1, "AGATCGGAAGAGCACACGTCTGAACTCCAGTCA")
        abi.set_adapter(p, 2, "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT")
        timed(p, "c3b_adapter_seq")
        p = config_params(abi, "C3")
        p.umi_front1 = p.umi_front2 = 8
        timed(p, "c3_umi8")
        p = config_params(abi, "C3")
        p.correction_enabled = 1
        timed(p, "c3_correct")
        p = config_params(abi, "C4")  # -m with -c: the merge variant's -c instantiation
        p.correction_enabled = 1
        timed(p, "c4_correct")
        i = torch.arange(0, n, 100, device=self.dev, dtype=torch.int64)
        self.planes[0][(i // abi.TILE_READS) * abi.TILE_READS * STRIDE + (i % abi.TILE_READS) * 16 + 5] = ord("a")
        timed(config_params(abi, "C3"), "c3_lowercase_1pct")
        # the same pairs with an IUPAC code instead (R: neither ACGTN nor lowercase)
        self.planes[0][(i // abi.TILE_READS) * abi.TILE_READS * STRIDE + (i % abi.TILE_READS) * 16 + 5] = ord("R")
        timed(config_params(abi, "C3"), "c3_iupac_1pct")
        return out

    def host_legs(self, cpu_pairs, e2e_pairs, workers):
        del self.planes, self.lens, self.results
        self.torch.cuda.empty_cache()
        return host_legs(self.lib, self.abi, self.torch, cpu_pairs, e2e_pairs, workers)

    def close(self):
        self.lib.fq_engine_destroy(self.h)


def make_runner(spec, args, local):
    if spec == "hip":
        return HipRunner(args, local)
    # CPU rehearsal of the rank orchestration (tests/test_bench_cpu.py): "module:Class" on sys.path
    import importlib

    mod, cls = spec.split(":")
    sys.path.insert(0, os.path.join(REPO, "tests"))
    return getattr(importlib.import_module(mod), cls)(args, local)


def free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def set_read_len(args):
    """--read-len: synthetic mates of this length (rows padded to a multiple of 16)."""
    global READ_LEN, STRIDE
    READ_LEN = int(getattr(args, "read_len", 150))
    STRIDE = (READ_LEN + 15) // 16 * 16


def run_rank(args):
    set_read_len(args)
    """One rank: shard, warm up, time exactly `steps` passes between barriers + device syncs,
    max over ranks, RCCL sum of the accumulator block, parity sample, rank 0 prints the line."""
    import hashlib

    import torch.distributed as dist

    from fqtool_amd.dist import reduce_accumulator, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    runner = make_runner(args.runner, args, local)
    if world > 1 or args.pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        kw = {"device_id": runner.dev} if runner.backend == "nccl" else {}
        dist.init_process_group(runner.backend, **kw)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    shard_rank, shard_world = rank, world
    if args.shard:  # rehearse one rank of a larger job: its index range, on this one process
        if world != 1:
            raise SystemExit("bench: --shard is for a single process")
        shard_rank, shard_world = (int(x) for x in args.shard.split("/"))
    first, n = shard(shard_rank, shard_world, args.pairs)
    runner.alloc(first, n)

    def step(timed):
        runner.step(timed)
        reduce_accumulator(runner.acc)  # Stats/FilterResult/insert-size sum over RCCL (xGMI) when world > 1

    for i in range(args.warmup):
        step(False)
        runner.sync()
        log(f"rank {rank}: warmup {i + 1}/{args.warmup}")
    if world > 1:
        dist.barrier()
    runner.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    runner.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = runner.elapsed_tensor(elapsed)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kavg = runner.kernel_ms()
    runner.finish()
    log(f"rank {rank}: {args.steps} steps in {elapsed:.3f}s")

    abi = runner.abi
    p = runner.p
    paired = runner.paired
    acc_host = runner.acc_host()
    total_pairs = n * world
    reads = (2 if paired else 1) * total_pairs
    # size-independent invariants of the reduced block: every pair (read) counted once by the
    # pre-filter stats and once by FilterResult
    st0 = abi.acc_stats_offset(p.insert_size_max, p.max_cycles, 0)
    assert int(acc_host[st0 + abi.FQ_ST_READS]) == total_pairs, "accumulator lost pairs"
    assert int(acc_host[abi.FQ_ACC_FILTER:abi.FQ_ACC_FILTER + 32].sum()) == reads, "FilterResult lost reads"
    acc_digest = hashlib.sha256(acc_host.tobytes()).hexdigest()

    sample = None
    if args.sample_pairs > 0:
        t1 = time.time()
        sample = runner.parity_sample(args.sample_pairs)
        if sample is not None:
            log(f"rank {rank}: parity sample {sample} ({time.time() - t1:.1f}s)")
            if world > 1:  # every rank checks its own shard; all must agree
                ok = runner.elapsed_tensor(1.0 if sample["ok"] else 0.0)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                sample["all_ranks_ok"] = bool(ok.item() == 1.0)
                sample["ranks"] = world

    engine = None
    if args.engine_pairs > 0 and hasattr(runner, "engine_leg"):
        log(f"rank {rank}: engine leg (pinned host packs of {args.engine_pairs}) ...")
        engine = runner.engine_leg(args.engine_pairs)
        log(f"rank {rank}: engine leg {engine}")
        if world > 1:
            t = runner.elapsed_tensor(engine["value"])
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            engine["value_all_ranks"] = round(float(t.item()), 2)

    paths = None
    if rank == 0 and world == 1 and args.config == "C3" and args.paths_pairs > 0 and hasattr(runner, "paths_leg"):
        try:
            paths = runner.paths_leg(args.paths_pairs)
            log(f"paths {paths}")
        except Exception as ex:  # a side leg: report, never fail the bench line
            paths = {"error": str(ex)}

    value = reads * args.steps / elapsed / 1e6
    traffic, traffic_src = pmc_traffic(args.config, args.pairs) if world == 1 else (None, None)
    sq, sq_src = sq_profile(args.config, args.pairs) if world == 1 else (None, None)
    valu = None
    sq_ms = (sq or {}).get("kernel_ms_trace") or (sq or {}).get("kernel_ms_bench")
    if sq and kavg and sq_ms and abs(sq_ms / kavg - 1) > 0.05:
        # the committed SQ counters were taken on another build (its kernel time differs from this
        # run's by more than 5 %): not reported as this build's
        log(f"SQ profile {sq_src} is stale ({sq_ms:.3f} ms vs this run's {kavg:.3f} ms): not used")
        valu = {"stale_profile": sq_src, "profile_kernel_ms": sq_ms, "run_kernel_ms": round(kavg, 3)}
        sq = None
    if sq and kavg and sq.get("counters_per_launch", {}).get("SQ_INSTS_VALU") and sq.get("kernel_cycles"):
        # VALU issue: the profiled launch's VALU wave-instructions (SQ_INSTS_VALU, per launch) over the
        # SIMD cycles of that launch (1024 SIMDs x its kernel cycles, GRBM_GUI_ACTIVE per XCD: the
        # clock the kernel actually ran at).  `frac_at_2_cycles` prices every VALU at the nominal 2
        # cycles per wave64 instruction (a lower bound); `issue_frac` at the tile loop's static
        # average cost per VALU (isa_cpi: VOP3 forms take ~4.4 cycles, VOP2 ~2.3) -- an estimate of
        # the share of SIMD cycles spent issuing VALU, <= 1 by construction of both counts.
        n_valu = sq["counters_per_launch"]["SQ_INSTS_VALU"]
        simd_cycles = SIMDS * sq["kernel_cycles"]
        cpi, cpi_src = isa_cpi(args.config)
        valu = {"insts_per_launch": n_valu, "per_tile": sq.get("valu_per_tile"),
                "frac_at_2_cycles": round(n_valu * 2 / simd_cycles, 4),
                "cycles_per_valu_static": cpi, "cpi_src": cpi_src,
                "issue_frac": round(n_valu * cpi / simd_cycles, 4) if cpi else None,
                "kernel_clock_GHz": round(sq["kernel_cycles"] / (sq_ms * 1e-3) / 1e9, 3) if sq_ms else None,
                "src": sq_src, "wait_frac": sq.get("wait_frac"), "inst_stall_frac": sq.get("inst_stall_frac"),
                "active_frac": sq.get("active_frac")}
    bytes_per_pair = (2 if paired else 1) * (2 * READ_LEN + 16)  # seq+qual uint8 + 16 B result per read
    achieved = n * bytes_per_pair / (kavg / 1e3) / 1e9 if kavg else None
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
        "config": {"workload": WORKLOADS[args.config].replace("150bp", f"{READ_LEN}bp"), ("pairs_per_gpu" if paired else "reads_per_gpu"): n,
                   "first_index": first,
                   "read_len": READ_LEN, "row_stride": STRIDE,
                   "parallelism": f"dp{world} (pairs sharded, RCCL sum of the accumulator block)"},
        # frac / achieved / peak are the HBM roofline (algorithmic bytes over the kernel time);
        # `bound` names what limits the kernel: VALU issue when the estimated VALU issue share of the
        # SIMD cycles (valu.issue_frac) is >= 0.75 and above the HBM fraction, else HBM
        "roofline": {"bound": ("valu_issue" if valu and valu.get("issue_frac") and achieved and
                               valu["issue_frac"] >= 0.75 and valu["issue_frac"] > achieved / HBM_PEAK_GBS else "hbm"),
                     "frac_of": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "traffic_unit": "bytes per launch (PMC)", "traffic_src": traffic_src,
                     "algorithmic_bytes": n * bytes_per_pair,
                     "kernel_ms_avg": round(kavg, 3) if kavg else None,
                     ("bytes_per_pair" if paired else "bytes_per_read"): bytes_per_pair,
                     "valu": valu},
        "cpu_baseline": None,
        "engine_mreads_s": engine["value"] if engine else None,
        "engine": engine,
        "paths": paths,
        "e2e": None,
        "e2e_c4": None,
        "e2e_file": None,
        "e2e_gz": None,
        "e2e_file_shm": None,
        "e2e_gzin": None,
        "acc_sha256": acc_digest,
        "parity_sample": sample,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "C3" and hasattr(runner, "host_legs"):
        log(f"host legs: e2e on {args.e2e_pairs} pairs, CPU baseline on {args.cpu_pairs} pairs ...")
        legs = runner.host_legs(args.cpu_pairs, args.e2e_pairs, min(16, os.cpu_count() or 1))
        out["cpu_baseline"] = legs["cpu_baseline"]
        out["e2e"] = legs["e2e"]
        out["e2e_c4"] = legs.get("e2e_c4")
        out["e2e_file"] = legs.get("e2e_file")
        out["e2e_gz"] = legs.get("e2e_gz")
        out["e2e_gzin"] = legs.get("e2e_gzin")
        out["e2e_file_shm"] = legs.get("e2e_file_shm")
        log(f"e2e {legs['e2e']}")
        log(f"e2e_c4 {legs.get('e2e_c4')}")
    runner.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        out_pg = dist.get_backend()
        dist.destroy_process_group()
        log(f"rank {rank}: process group ({out_pg}) closed")
    if sample is not None and not sample.get("all_ranks_ok", sample["ok"]):
        raise SystemExit("bench: parity sample FAILED (the engine's records/accumulator differ from the oracle)")


def _spawned_rank(i, args, port):
    os.environ.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run_rank(args)


def launch(args):
    """`--gpus N` without a launcher: start N rank processes here (spawn, before this process
    touches any GPU), one per GPU. Under torchrun WORLD_SIZE must equal N."""
    if "WORLD_SIZE" in os.environ or args.gpus == 1:
        run_rank(args)
        return
    # No torch.cuda / HIP call here: this process only forks+execs the ranks (a GPU-initialised
    # process must never replace its program on this pool); each rank checks its own device.
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_spawned_rank, args=(i, args, port)) for i in range(args.gpus)]
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join()
    bad = [(i, p_.exitcode) for i, p_ in enumerate(procs) if p_.exitcode != 0]
    if bad:
        raise SystemExit(f"bench: rank(s) failed: {bad}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=None,
                    help="pairs (SE: reads) per GPU; default 100 M (BASELINE configs 1-3), 125 M for C5 "
                         "(config 4's 1 B pairs over 8 GPUs)")
    ap.add_argument("--cpu-pairs", type=int, default=1_000_000, help="CPU-baseline sample size (pairs)")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip both host legs (e2e and CPU baseline)")
    ap.add_argument("--e2e-pairs", type=int, default=50_000_000, help="pairs of the end-to-end tool leg (0: off)")
    ap.add_argument("--paths-pairs", type=int, default=20_000_000,
                    help="pairs of the off-baseline path leg (C3 + UMI / -c / 1 %% lowercase; 0: off)")
    ap.add_argument("--sample-pairs", type=int, default=1_000_000,
                    help="per-rank parity sample checked against the oracle after the timed region (0: off)")
    ap.add_argument("--engine-pairs", type=int, default=1_048_576,
                    help="pairs per host pack of the PCIe-inclusive engine leg (0: off)")
    ap.add_argument("--config", default="C3", choices=sorted(WORKLOADS),
                    help="workload (BASELINE.json configs); the headline metric is C3")
    ap.add_argument("--read-len", type=int, default=150,
                    help="synthetic read length (default 150, the BASELINE configs); longer reads exercise "
                         "the long-read kernel variant")
    ap.add_argument("--runner", default="hip", help=argparse.SUPPRESS)  # tests: CPU rehearsal of the ranks
    ap.add_argument("--shard", default=None,
                    help="R/W: process rank R's index range of a W-rank job on this single process "
                         "(e.g. 7/8 with --config C5: the last shard of config 5)")
    ap.add_argument("--pg", action="store_true",
                    help="create the process group (RCCL on the GPU) and run the accumulator all-reduce "
                         "even with one rank")
    args = ap.parse_args()
    if args.pairs is None:
        args.pairs = 125_000_000 if args.config == "C5" else 100_000_000
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if not 1 <= args.read_len <= 1000:
        raise SystemExit("--read-len must be in 1..1000")
    set_read_len(args)
    launch(args)


if __name__ == "__main__":
    main()
