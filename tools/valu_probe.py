"""Profiling aid: one launch of the fast PE kernel per ablation variant (fq_params.reserved[0]
bits, see pe_fast.hip), meant to run under `rocprofv3 --pmc SQ_INSTS_VALU ...` so the per-dispatch
counters give each phase's dynamic instruction count (dispatch order = VARIANTS order)."""
import ctypes, os, sys
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
bits = {"full": 0, "no_overlap": 1, "no_filter": 2, "no_stats": 4, "no_polyg": 8, "stage_only": 15,
        "no_ov_exact": 64, "no_ov_scan": 128, "no_trim": 1024, "no_polyx": 2048}
import bench
CFG = os.environ.get("CONFIG", "C3")
for name in os.environ.get("VARIANTS", "full,no_overlap,no_filter,no_stats,no_polyg,stage_only").split(","):
    p = bench.config_params(abi, CFG)
    p.reserved[0] = bits[name]
    h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
    lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
    print(name, lib.fq_engine_last_kernel_ms(h), flush=True)
    lib.fq_engine_destroy(h)
if os.environ.get("COUNT_EXACT"):
    p = abi.default_params(True, 256); p.qual_filter_enabled = 1; p.adapter_trimming = 1; p.polyg_enabled = 1
    p.reserved[0] = 512
    lib.fq_debug_phase_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_ulonglong * 8)()
    lib.fq_debug_phase_cycles(out, 8)
    h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
    lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
    lib.fq_debug_phase_cycles(out, 8)
    print("exact checks per lane-scan: %.3f (%d checks, %d scanning lanes)" % (out[0] / max(out[1], 1), out[0], out[1]))
