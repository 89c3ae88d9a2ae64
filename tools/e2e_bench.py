#!/usr/bin/env python3
"""End-to-end (FASTQ file -> FASTQ files + JSON) timing of the fqtool-amd binary on the GPU box.

Not the headline metric (bench.py is: device-resident batches).  This measures the whole tool:
reader/parse, pinned H2D, engine, D2H, formatting and writers, on plain FASTQ in the page
cache, next to the reference binary (oracle/_ref/fqtool_ref) on the same files and options,
and checks that both produce byte-identical FASTQ and JSON (Software block masked).

    python tools/e2e_bench.py [--pairs 2000000] [--workers 16] [--no-ref]
Prints one JSON line per run plus a parity verdict.
"""
import argparse
import ctypes
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (write_fastq_pair, SEED, READ_LEN, STRIDE)

OPTS = {
    "C3": ["-q", "-a", "--detect_pe_adapter", "-g"],
    "C5": ["-q", "-a", "-g", "-x", "--enable_cut_right"],
    "C4": ["-q", "-a", "-g", "--enable_cut_right", "-m"],
}


def gen_fastq(pairs, d):
    import torch

    from fqtool_amd import abi

    lib = abi.load_engine()
    dev = torch.device("cuda:0")
    bufs = [torch.empty(abi.batch_bytes(pairs, bench.STRIDE), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.empty(pairs, dtype=torch.int16, device=dev) for _ in range(2)]
    b = abi.FqBatch()
    b.n, b.stride = pairs, bench.STRIDE
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    first = 10 ** 12
    assert lib.fq_synth_fill_device(ctypes.byref(b), bench.SEED, first, bench.READ_LEN, None) == 0
    torch.cuda.synchronize()
    paths = bench.write_fastq_fast(bufs, pairs, first, d)
    del bufs
    torch.cuda.empty_cache()
    return paths


def digest(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 22), b""):
            h.update(blk)
    return h.hexdigest()


def same_records(a, b):
    """Order-insensitive FASTQ comparison (the reference writes packs in completion order at -w > 1)."""
    def sorted_digest(p):
        cmd = f"paste - - - - < '{p}' | LC_ALL=C sort -S 2G | sha256sum"
        return subprocess.run(["bash", "-c", cmd], stdout=subprocess.PIPE, check=True, text=True).stdout.split()[0]
    return sorted_digest(a) == sorted_digest(b)


def masked_json(path):
    j = json.load(open(path))
    j.pop("Software", None)
    return j


def run(tool, r1, r2, d, tag, cfg, workers, extra=(), null_out=False):
    o = {k: os.path.join(d, f"{tag}_{k}") for k in ("o1.fq", "o2.fq", "m.fq", "r.json", "r.html")}
    if null_out:
        for k in ("o1.fq", "o2.fq", "m.fq"):
            o[k] = "/dev/null"
    cmd = [tool, "-i", r1, "-I", r2, "-o", o["o1.fq"], "-O", o["o2.fq"], *OPTS[cfg], "-w", str(workers),
           "-J", o["r.json"], "-H", o["r.html"], *extra]
    if cfg == "C4":
        cmd += ["--merge_output", o["m.fq"]]
    env = dict(os.environ)
    if os.environ.get("E2E_TEARDOWN_TIMING"):  # (FQ_TIMING keeps the teardown the binary otherwise skips)
        env["FQ_TIMING"] = "1"
    for tok in [t for t in cmd if re.fullmatch(r"[A-Z_]+=\S*", t)]:  # KEY=VALUE extras: environment
        k, v = tok.split("=", 1)
        env[k] = v
        cmd.remove(tok)
    env["FQ_TIMING_MONO"] = "1"  # (the tool's steady-clock stamps: exec and exit time from outside)
    for k in ("o1.fq", "o2.fq", "m.fq"):  # (a fresh file each run: rewriting a truncated one makes
        if o[k] != "/dev/null" and os.path.exists(o[k]):  # some file systems write it back at close)
            os.remove(o[k])
    t0 = time.perf_counter()
    m0 = time.monotonic()
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    m1 = time.monotonic()
    wall = time.perf_counter() - t0
    if p.returncode != 0:
        raise SystemExit(f"{tag} failed rc={p.returncode}: {p.stderr[-2000:]}")
    m = re.search(r"fqtool-amd: (.*)", p.stderr)
    t = re.search(r"fqtool-amd timing: (.*)", p.stderr)
    ec = re.findall(r"fq_engine_create: (.*)", p.stderr)  # (FQ_ENGINE_TIMING=1)
    rb = re.findall(r"fq_engine_raw_begin: ([\d.]+) ms", p.stderr)
    rs = [float(x) for x in re.findall(r"fq_engine_raw_enqueue: slot \d+ set up in ([\d.]+) ms", p.stderr)]
    if rb or rs:
        ec.append(f"raw_begin {'+'.join(rb)} ms, {len(rs)} raw slots set up in {sum(rs):.1f} ms (max {max(rs or [0]):.1f})")
    mm = re.search(r"fqtool-amd mono: t0 ([\d.]+) end ([\d.]+)(.*)", p.stderr)
    if mm:  # before the tool's clock starts (exec, loading, static init) and after its last line (exit)
        ec.append(f"exec {float(mm.group(1)) - m0:.3f} s, exit {m1 - float(mm.group(2)):.3f} s;{mm.group(3)}")
    return wall, (m.group(1) if m else "(no fqtool-amd summary line)") + ((" | " + t.group(1)) if t else "") + \
        ((" | engine: " + "; ".join(ec)) if ec else ""), o


def _bgzf_chunk(arg):
    path, off, n = arg
    import struct
    import zlib
    with open(path, "rb") as f:
        f.seek(off)
        raw = f.read(n)
    out = bytearray()
    for o in range(0, len(raw), 0xFF00):
        blk = raw[o:o + 0xFF00]
        c = zlib.compressobj(1, zlib.DEFLATED, -15)
        d = c.compress(blk) + c.flush()
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", len(d) + 25)
        out += d + struct.pack("<II", zlib.crc32(blk), len(blk))
    return bytes(out)


def compress_inputs(paths, kind):
    """The generated FASTQ as BGZF (level 1, on a process pool) or as one gzip stream (gzip -1)."""
    import multiprocessing as mp
    import subprocess

    out = []
    for p in paths:
        gz = p + ".gz"
        if kind == "bgzf":
            size, step = os.path.getsize(p), 0xFF00 * 64
            with mp.Pool(16) as pool, open(gz, "wb") as f:
                for blob in pool.imap(_bgzf_chunk, [(p, o, min(step, size - o)) for o in range(0, size, step)], 4):
                    f.write(blob)
                f.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
        else:
            with open(gz, "wb") as f:
                subprocess.run(["gzip", "-1", "-c", p], stdout=f, check=True)
        os.remove(p)
        out.append(gz)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2_000_000)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--config", default="C3", choices=sorted(OPTS))
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--devices", default=None, help="--devices of the fqtool-amd run (e.g. 0,0,0,0)")
    ap.add_argument("--repeat", type=int, default=1, help="runs of the fqtool-amd binary (all printed)")
    ap.add_argument("--extra", default="", help="extra fqtool-amd options (space separated)")
    ap.add_argument("--variants", default=None, help="';'-separated list of --extra strings, each run in turn")
    ap.add_argument("--null-out", action="store_true", help="FASTQ outputs to /dev/null (as bench.py's e2e leg)")
    ap.add_argument("--workers-list", default=None, help="comma list of -w values to run (overrides --workers)")
    ap.add_argument("--pause", type=float, default=0.0, help="seconds between fqtool-amd runs")
    ap.add_argument("--gz", default=None, choices=["bgzf", "gzip"], help="compressed inputs: BGZF or one gzip stream")
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="fqe2e_")
    try:
        t0 = time.perf_counter()
        r1, r2 = gen_fastq(args.pairs, tmp)
        gb = (os.path.getsize(r1) + os.path.getsize(r2)) / 1e9
        os.sync()
        print(f"[e2e] wrote {args.pairs} pairs ({gb:.2f} GB FASTQ) in {time.perf_counter() - t0:.1f}s", flush=True)
        if args.gz:
            t0 = time.perf_counter()
            r1, r2 = compress_inputs([r1, r2], args.gz)
            gzb = (os.path.getsize(r1) + os.path.getsize(r2)) / 1e9
            print(f"[e2e] compressed to {args.gz} ({gzb:.2f} GB) in {time.perf_counter() - t0:.1f}s", flush=True)
        reads = 2 * args.pairs
        ours = os.path.join(REPO, "fqtool_amd", "bin", "fqtool")
        variants = args.variants.split(";") if args.variants else [args.extra]
        wl = [int(x) for x in args.workers_list.split(",")] if args.workers_list else [args.workers]
        for _, w, v in [(r, w, v) for v in variants for w in wl for r in range(args.repeat)]:
            if args.pause:
                time.sleep(args.pause)
            extra = (["--devices", args.devices] if args.devices else []) + v.split()
            wall, inner, o_ours = run(ours, r1, r2, tmp, "amd", args.config, w, extra, args.null_out)
            line = {"tool": "fqtool-amd", "config": args.config, "pairs": args.pairs, "fastq_GB": round(gb, 3),
                    "wall_s": round(wall, 3), "Mreads_s": round(reads / wall / 1e6, 3),
                    "fastq_GB_s": round(gb / wall, 3), "workers": w, "devices": args.devices, "extra": v,
                    "text_mode": os.environ.get("FQ_TEXT_MODE", "1") != "0", "tool_log": inner}
            print(json.dumps(line), flush=True)
        ref = os.path.join(REPO, "oracle", "_ref", "fqtool_ref")
        if not args.no_ref and not args.null_out and os.path.exists(ref):
            w = min(16, args.workers)
            wall_r, _, o_ref = run(ref, r1, r2, tmp, "ref", args.config, w)
            print(json.dumps({"tool": "reference", "config": args.config, "pairs": args.pairs, "wall_s": round(wall_r, 3),
                              "Mreads_s": round(reads / wall_r / 1e6, 3), "workers": w}), flush=True)
            same = {}
            for k in ("o1.fq", "o2.fq", "m.fq"):
                if os.path.exists(o_ref[k]) or os.path.exists(o_ours[k]):
                    if not (os.path.exists(o_ours[k]) and os.path.exists(o_ref[k])):
                        same[k] = False
                    elif digest(o_ours[k]) == digest(o_ref[k]):
                        same[k] = "identical"
                    else:
                        same[k] = "same records, pack order differs" if same_records(o_ours[k], o_ref[k]) else False
            jr, jo = masked_json(o_ref["r.json"]), masked_json(o_ours["r.json"])
            # the reference counts InsertSize on worker thread 0 only; compare it at -w 1 only
            if w > 1:
                jr.pop("InsertSize", None)
                jo.pop("InsertSize", None)
            same["json"] = jr == jo
            print(json.dumps({"parity": same, "speedup_vs_reference": round(wall_r / wall, 2)}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
