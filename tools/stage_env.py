"""Profiling aid: stage-only fast kernel (build with make ABLATE_STAGE=1) on synthetic vs constant
data, timed like tools/micro/stagebench (best of 5)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fqtool_amd import abi

lib = abi.load_engine()
dev = torch.device("cuda:0")
n, stride = 20_000_000, 160
bufs = [torch.empty(abi.batch_bytes(n, stride), dtype=torch.uint8, device=dev) for _ in range(4)]
lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
b = abi.FqBatch(); b.n, b.stride = n, stride
b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
res = torch.empty(n * 32, dtype=torch.uint8, device=dev)


def run(tag, bits):
    p = abi.default_params(True, 256); p.qual_filter_enabled = 1; p.adapter_trimming = 1; p.polyg_enabled = 1
    p.reserved[0] = bits
    h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
    best = 1e9
    for _ in range(5):
        lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
        best = min(best, lib.fq_engine_last_kernel_ms(h))
    lib.fq_engine_destroy(h)
    print(f"{tag:30s} best {best:7.3f} ms", flush=True)


assert lib.fq_synth_fill_device(ctypes.byref(b), 20261015, 0, 150, None) == 0
torch.cuda.synchronize()
run("synthetic stage_only", 15)
run("synthetic full", 0)
for i, t in enumerate(bufs):
    t.fill_(0x41 if i % 2 == 0 else 0x49)
for t in lens:
    t.fill_(150)
torch.cuda.synchronize()
run("constant stage_only", 15)
run("constant full", 0)
