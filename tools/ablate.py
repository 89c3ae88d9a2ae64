"""Profiling aid: time the fast PE kernel with phases switched off (fq_params.reserved[0] bits,
see pe_fast.hip).  Outputs are NOT valid in ablated runs; only the timings matter."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fqtool_amd import abi

lib = abi.load_engine()
dev = torch.device("cuda:0")
n, stride = int(os.environ.get("PAIRS", 20_000_000)), 160
bufs = [torch.empty(abi.batch_bytes(n, stride), dtype=torch.uint8, device=dev) for _ in range(4)]
lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
b = abi.FqBatch(); b.n, b.stride = n, stride
b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
assert lib.fq_synth_fill_device(ctypes.byref(b), 20261015, 0, 150, None) == 0
res = torch.empty(n * 32, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
variants = [("full", 0), ("no_overlap", 1), ("no_filter", 2), ("no_stats", 4), ("no_polyg", 8),
            ("no_lds_atomics", 16), ("no_overlap_filter_stats", 7), ("stage_only", 15), ("no_polyg_counters", 32),
            ("no_ov_exact", 64), ("no_ov_scan", 128),
            ("plus_512_valu", 256), ("one_wg_per_cu", 70 << 16)]
only = os.environ.get("VARIANTS")
if only:
    variants = [v for v in variants if v[0] in only.split(",")]
results = {}
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import config_params  # (the BASELINE config's engine parameters, CONFIG=C3 by default)
CFG = os.environ.get("CONFIG", "C3")
for rep in range(int(os.environ.get("REPS", 3))):
    for name, bits in variants:
        p = config_params(abi, CFG)
        p.reserved[0] = bits & 0xFFFF
        p.reserved[2] = (bits >> 16) * 1024  # extra LDS KiB per workgroup (occupancy probe)
        h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
        lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
        lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
        ms = lib.fq_engine_last_kernel_ms(h)
        results.setdefault(name, []).append(ms)
        lib.fq_engine_destroy(h)
for name in results:
    v = sorted(results[name])
    print(f"{name:28s} median {v[len(v)//2]:8.2f} ms  min {v[0]:8.2f}  -> {n / (v[len(v)//2] / 1e3) / 1e9:.2f} G pairs/s", flush=True)

# per-phase wave cycles (fq_params.reserved[1] = 1)
names = ["staging", "trim", "polyG", "overlap", "polyX/maxlen", "filter", "stats", "store"]
from bench import config_params
p = config_params(abi, os.environ.get("CONFIG", "C3"))
p.reserved[1] = 1
h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
lib.fq_debug_phase_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = (ctypes.c_ulonglong * 8)()
lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
lib.fq_debug_phase_cycles(out, 8)
lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
print("stamped run ms", lib.fq_engine_last_kernel_ms(h))
lib.fq_debug_phase_cycles(out, 8)
tot = sum(out)
if tot == 0:
    print("no phase stamps (build with make STAMPS=1)")
for nm, v in (zip(names, out) if tot else []):
    print(f"phase {nm:14s} {100.0 * v / tot:6.1f}%  {v / 2048:14.0f} cycles/wave")
lib.fq_engine_destroy(h)
