"""Profiling aid: median kernel ms of the fast kernel over several launches (after one warm-up)
for each config in CONFIGS, with the engine library FQ_ENGINE_LIB (A/B builds, tools/ab.sh)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fqtool_amd import abi
import bench

lib = abi.load_engine()
dev = torch.device("cuda:0")
n, stride = int(os.environ.get("PAIRS", 20_000_000)), int(os.environ.get("STRIDE", 160))
RL = int(os.environ.get("L", 150))  # read length (long rows: STRIDE 256 / 304 with L 250 / 300)
bufs = [torch.empty(abi.batch_bytes(n, stride), dtype=torch.uint8, device=dev) for _ in range(4)]
lens = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(2)]
b = abi.FqBatch(); b.n, b.stride = n, stride
b.seq1, b.qual1, b.seq2, b.qual2 = [t.data_ptr() for t in bufs]
b.len1, b.len2 = lens[0].data_ptr(), lens[1].data_ptr()
assert lib.fq_synth_fill_device(ctypes.byref(b), 20261015, 0, RL, None) == 0
res = torch.empty(n * 32, dtype=torch.uint8, device=dev)
fe = int(os.environ.get("INDEX_EVERY", 0))
if fe:  # every fe-th pair dropped by the host's index filter (fq_batch.flags)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    flags[::fe] = abi.FQ_BF_INDEX_FILTERED
    b.flags = flags.data_ptr()
ev = int(os.environ.get("EXOTIC_EVERY", 0))
if ev:  # every ev-th pair gets a lowercase base in read 1 (position 5): a hand-off to the general kernel
    i = torch.arange(0, n, ev, device=dev, dtype=torch.int64)
    off = (i // 32) * 32 * stride + (i % 32) * 16 + 5
    bufs[0][off] = ord("a")
torch.cuda.synchronize()
tag = os.environ.get("TAG", "")
for cfg in os.environ.get("CONFIGS", "C3").split():
    p = bench.config_params(abi, cfg)
    p.max_cycles = max(p.max_cycles, 2 * RL + 16)
    p.correction_enabled = int(os.environ.get("CORRECT", 0))  # -c on top of the config
    p.umi_front1 = p.umi_front2 = int(os.environ.get("UMI", 0))  # UMI cut from both reads
    if os.environ.get("ADAPTERS"):  # explicit adapters (trimBySequence), as bench's c3b_adapter_seq
        abi.set_adapter(p, 1, "AGATCGGAAGAGCACACGTCTGAACTCCAGTCA")
        abi.set_adapter(p, 2, "AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT")
    p.reserved[0] = int(os.environ.get("ABL", 0))  # ablation bits (pe_fast.hip; results invalid when set)
    if cfg == "C2":
        b.seq2 = b.qual2 = None
    h = ctypes.c_void_p(); assert lib.fq_engine_create(ctypes.byref(p), 0, 0, 0, ctypes.byref(h)) == 0
    ms = []
    for i in range(int(os.environ.get("LAUNCHES", 6))):
        lib.fq_engine_process_device(h, ctypes.byref(b), res.data_ptr(), None); lib.fq_engine_sync(h)
        if i: ms.append(lib.fq_engine_last_kernel_ms(h))
    lib.fq_engine_destroy(h)
    ms.sort()
    print(f"{tag} {cfg} median {ms[len(ms)//2]:.3f} min {ms[0]:.3f}", flush=True)
    if cfg == "C2":
        b.seq2, b.qual2 = bufs[2].data_ptr(), bufs[3].data_ptr()
