import ctypes, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fqtool_amd import abi
lib = abi.load_engine()
dev = torch.device("cuda:0")
p = abi.default_params(True, 256); p.qual_filter_enabled = 1; p.adapter_trimming = 1; p.polyg_enabled = 1
h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
for n in [10**4, 10**5, 10**6, 4*10**6, 16*10**6, 64*10**6]:
    bufs = [torch.empty(abi.batch_bytes(n, 160), dtype=torch.uint8, device=dev) for _ in range(4)]
    lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
    b = abi.FqBatch(); b.n, b.stride = n, 160
    b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
    b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
    assert lib.fq_synth_fill_device(ctypes.byref(b), 1, 0, 150, None) == 0
    torch.cuda.synchronize()
    assert lib.fq_engine_reset_acc(h) == 0
    t = time.time()
    assert lib.fq_engine_process_device(h, ctypes.byref(b), None, None) == 0
    rc = lib.fq_engine_sync(h); dt = time.time() - t
    acc = torch.zeros(lib.fq_engine_acc_words(h), dtype=torch.int64).numpy()
    rc2 = lib.fq_engine_read_acc(h, acc.ctypes.data, acc.size)
    st0 = abi.acc_stats_offset(512, 256, 0)
    print(n, rc, rc2, "reads", acc[st0], "filtersum", acc[:32].sum(), "pre2", acc[st0 + abi.acc_stats_words(256)], "dt %.3f" % dt, "kms", lib.fq_engine_last_kernel_ms(h), flush=True)
    del bufs, lens
