"""ctypes mirror of the engine's C-ABI (include/fqengine.h).

Python is plumbing here: the product is the C-ABI library ``libfqengine.so`` (HIP kernels
for gfx950) and the C++ host tool ``fqtool``.  This module only lets bench.py / tests /
__graft_entry__ call the same entry points a reference-side binding would.
"""
import ctypes
import os

FQ_MAX_ADAPTER = 128
FQ_OK = 0
FQ_E_INVALID = -1

FQ_ACC_FILTER = 0
FQ_ACC_ADAPTER_READS = 32
FQ_ACC_ADAPTER_BASES = 33
FQ_ACC_POLYX_READS = 34
FQ_ACC_POLYX_BASES = 39
FQ_ACC_MERGED_PAIRS = 44
FQ_ACC_INSERT = 48
FQ_ST_READS, FQ_ST_LENGTH_SUM, FQ_ST_Q20, FQ_ST_Q30 = 0, 1, 2, 3
FQ_ST_CYCLES = 16
FQ_ST_PER_CYCLE = 16

FQ_RF_NULL = 0x01
FQ_RF_AD_OVERLAP = 0x02
FQ_RF_AD_SEQ = 0x04
FQ_RF_AD_NEG = 0x08
FQ_RF_MERGED = 0x10
FQ_RF_OVERLAP = 0x20
FQ_RF_CORRECTED = 0x40
FQ_RF_INDEX_FILTERED = 0x80
FQ_BF_INDEX_FILTERED = 0x01
FQ_ACC_TAIL_CORRECTED_READS = 0
FQ_ACC_TAIL_CORRECTED_BASES = 1
FQ_ACC_TAIL_WORDS = 16

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
ENGINE_LIB = os.environ.get("FQ_ENGINE_LIB") or os.path.join(PKG_DIR, "lib", "libfqengine.so")  # (override: profiling A/B builds)
HOST_LIB = os.path.join(PKG_DIR, "lib", "libfqhost.so")
FQTOOL_BIN = os.path.join(PKG_DIR, "bin", "fqtool")


class FqParams(ctypes.Structure):
    _fields_ = [
        ("paired", ctypes.c_int32),
        ("trim_front1", ctypes.c_int32), ("trim_tail1", ctypes.c_int32),
        ("trim_front2", ctypes.c_int32), ("trim_tail2", ctypes.c_int32),
        ("cut_front", ctypes.c_int32), ("cut_right", ctypes.c_int32), ("cut_tail", ctypes.c_int32),
        ("cut_front_window", ctypes.c_int32), ("cut_right_window", ctypes.c_int32),
        ("cut_tail_window", ctypes.c_int32),
        ("cut_front_quality", ctypes.c_int32), ("cut_right_quality", ctypes.c_int32),
        ("cut_tail_quality", ctypes.c_int32),
        ("polyg_enabled", ctypes.c_int32),
        ("polyg_compare_req", ctypes.c_int32), ("polyg_max_mismatch", ctypes.c_int32),
        ("polyg_one_mismatch_per", ctypes.c_int32),
        ("polyx_enabled", ctypes.c_int32), ("polyx_mask", ctypes.c_int32),
        ("polyx_compare_req", ctypes.c_int32), ("polyx_max_mismatch", ctypes.c_int32),
        ("polyx_one_mismatch_per", ctypes.c_int32),
        ("adapter_trimming", ctypes.c_int32),
        ("adapter1_len", ctypes.c_int32), ("adapter2_len", ctypes.c_int32),
        ("adapter1", ctypes.c_uint8 * FQ_MAX_ADAPTER),
        ("adapter2", ctypes.c_uint8 * FQ_MAX_ADAPTER),
        ("overlap_diff_limit", ctypes.c_int32), ("overlap_require", ctypes.c_int32),
        ("insert_size_max", ctypes.c_int32),
        ("max_len1", ctypes.c_int32), ("max_len2", ctypes.c_int32),
        ("merge_enabled", ctypes.c_int32), ("discard_unmerged", ctypes.c_int32),
        ("qual_filter_enabled", ctypes.c_int32),
        ("low_qual_limit", ctypes.c_int32), ("low_qual_base_limit", ctypes.c_int32),
        ("n_base_limit", ctypes.c_int32),
        ("avg_qual_limit", ctypes.c_double),
        ("length_filter_enabled", ctypes.c_int32), ("min_len", ctypes.c_int32),
        ("max_len", ctypes.c_int32),
        ("complexity_enabled", ctypes.c_int32),
        ("complexity_threshold", ctypes.c_double),
        ("max_cycles", ctypes.c_int32),
        ("correction_enabled", ctypes.c_int32),
        ("umi_front1", ctypes.c_int32), ("umi_front2", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 4),
    ]


class FqBatch(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("stride", ctypes.c_int32),
        ("seq1", ctypes.c_void_p), ("qual1", ctypes.c_void_p), ("len1", ctypes.c_void_p),
        ("seq2", ctypes.c_void_p), ("qual2", ctypes.c_void_p), ("len2", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
    ]


class FqTextRec(ctypes.Structure):  # fq_text_rec (include/fqengine.h), 24 bytes
    _fields_ = [("name_off", ctypes.c_uint32), ("seq_off", ctypes.c_uint32), ("strand_off", ctypes.c_uint32),
                ("qual_off", ctypes.c_uint32), ("name_len", ctypes.c_uint16), ("strand_len", ctypes.c_uint16),
                ("len", ctypes.c_uint16), ("pad", ctypes.c_uint16)]


TEXT_REC_DTYPE = [("name_off", "<u4"), ("seq_off", "<u4"), ("strand_off", "<u4"), ("qual_off", "<u4"),
                  ("name_len", "<u2"), ("strand_len", "<u2"), ("len", "<u2"), ("pad", "<u2")]


class FqTextBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("stride", ctypes.c_int32), ("text", ctypes.c_void_p * 2),
                ("text_bytes", ctypes.c_uint64 * 2), ("rec", ctypes.c_void_p * 2)]


class FqTextOut(ctypes.Structure):
    _fields_ = [("text", ctypes.c_void_p * 2), ("bytes", ctypes.c_uint64 * 2)]


class FqRawWindow(ctypes.Structure):  # fq_raw_window
    _fields_ = [("bytes", ctypes.c_void_p * 2), ("n", ctypes.c_uint64 * 2)]


class FqRawResult(ctypes.Structure):  # fq_raw_result
    _fields_ = [("pairs", ctypes.c_int32), ("stop", ctypes.c_int32), ("max_len", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("carry", ctypes.c_uint64 * 2), ("text_bytes", ctypes.c_uint64 * 2)]


class FqRawOut(ctypes.Structure):  # fq_raw_out
    _fields_ = [("text", FqTextOut), ("adapter_bytes", ctypes.c_uint64 * 2),
                ("results", ctypes.c_void_p), ("rec", ctypes.c_void_p * 2)]


# Batch planes hold rows in chunk-interleaved tiles (include/fqengine.h): byte j of read i at
# (i // 32) * 32 * stride + (j // 16) * 512 + (i % 32) * 16 + j % 16.
TILE_READS = 32
CHUNK = 16


def batch_bytes(n, stride):
    """Bytes of one batch plane for n reads (whole tiles), fq_batch_bytes."""
    return -(-n // TILE_READS) * TILE_READS * stride


def batch_offset(stride, i, j=0):
    """fq_batch_offset: plane offset of byte j of read i."""
    return (i // TILE_READS) * TILE_READS * stride + (j // CHUNK) * TILE_READS * CHUNK + (i % TILE_READS) * CHUNK + j % CHUNK


def tile_rows(rows):
    """(n, stride) uint8 rows -> flat batch plane (numpy), padded to whole tiles."""
    import numpy as np

    n, stride = rows.shape
    nt = -(-n // TILE_READS)
    buf = np.zeros((nt * TILE_READS, stride), np.uint8)
    buf[:n] = rows
    return np.ascontiguousarray(buf.reshape(nt, TILE_READS, stride // CHUNK, CHUNK).transpose(0, 2, 1, 3)).reshape(-1)


def untile_rows(plane, n, stride):
    """Flat batch plane (numpy, >= batch_bytes(n, stride) bytes) -> (n, stride) rows."""
    nt = -(-n // TILE_READS)
    v = plane[: nt * TILE_READS * stride].reshape(nt, stride // CHUNK, TILE_READS, CHUNK).transpose(0, 2, 1, 3)
    return v.reshape(nt * TILE_READS, stride)[:n]


class FqReadResult(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_uint16), ("len", ctypes.c_uint16),
        ("code", ctypes.c_uint8), ("flags", ctypes.c_uint8),
        ("ad_pos", ctypes.c_uint16), ("ad_len", ctypes.c_uint16),
        ("m_len1", ctypes.c_uint16), ("m_len2", ctypes.c_uint16),
        ("reserved", ctypes.c_uint16),
    ]


RESULT_DTYPE_FIELDS = [("start", "<u2"), ("len", "<u2"), ("code", "u1"), ("flags", "u1"),
                       ("ad_pos", "<u2"), ("ad_len", "<u2"), ("m_len1", "<u2"), ("m_len2", "<u2"),
                       ("reserved", "<u2")]


def acc_stats_words(max_cycles):
    return FQ_ST_CYCLES + max_cycles * FQ_ST_PER_CYCLE


def acc_stats_offset(insert_size_max, max_cycles, k):
    base = FQ_ACC_INSERT + insert_size_max + 1
    base = (base + 15) & ~15
    return base + k * acc_stats_words(max_cycles)


def acc_tail_offset(insert_size_max, max_cycles):
    return acc_stats_offset(insert_size_max, max_cycles, 4)


def acc_words(insert_size_max, max_cycles):
    return acc_tail_offset(insert_size_max, max_cycles) + FQ_ACC_TAIL_WORDS


def default_params(paired=True, max_cycles=256):
    """Reference defaults after Options::update (reference src/options.h, src/options.cpp:24-58)
    with every CLI flag off (CLI11 resets bool flags to false)."""
    p = FqParams()
    p.paired = 1 if paired else 0
    p.cut_front_window = p.cut_right_window = p.cut_tail_window = 4
    p.cut_front_quality = p.cut_right_quality = p.cut_tail_quality = 20
    p.polyg_compare_req, p.polyg_max_mismatch, p.polyg_one_mismatch_per = (1, 10, 10) if paired else (10, 1, 10)
    p.polyx_mask = 0x1F
    p.polyx_compare_req, p.polyx_max_mismatch, p.polyx_one_mismatch_per = 10, 1, 10
    p.overlap_diff_limit, p.overlap_require, p.insert_size_max = 5, 30, 512
    p.low_qual_limit = 20 + 33
    p.low_qual_base_limit = int(0.15 * 151)
    p.n_base_limit = 5
    p.min_len = 15
    p.complexity_threshold = 0.3
    p.max_cycles = max_cycles
    return p


def set_adapter(p, which, seq):
    data = seq.encode() if isinstance(seq, str) else bytes(seq)
    if len(data) > FQ_MAX_ADAPTER:
        raise ValueError("adapter too long")
    arr = getattr(p, "adapter%d" % which)
    for i, c in enumerate(data):
        arr[i] = c
    setattr(p, "adapter%d_len" % which, len(data))


def load_engine(path=ENGINE_LIB):
    """Load libfqengine.so and declare its prototypes.  Raises OSError when it is missing:
    there is no CPU fallback."""
    # torch bundles its own HIP runtime (libamdhip64.so.7 / libhsa-runtime64.so.1); loading it
    # first makes the engine bind to that same runtime instead of a second copy from /opt/rocm
    # (two HIP runtimes in one process cannot share device memory or the device).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    vp, i32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
    lib.fq_engine_create.argtypes = [ctypes.POINTER(FqParams), ctypes.c_int, i32, i32, ctypes.POINTER(vp)]
    lib.fq_engine_create.restype = ctypes.c_int
    lib.fq_engine_destroy.argtypes = [vp]
    lib.fq_engine_process.argtypes = [vp, ctypes.POINTER(FqBatch), vp]
    lib.fq_engine_process_device.argtypes = [vp, ctypes.POINTER(FqBatch), vp, vp]
    lib.fq_engine_acc_words.argtypes = [vp]
    lib.fq_engine_acc_words.restype = ctypes.c_size_t
    lib.fq_engine_acc_device_ptr.argtypes = [vp, ctypes.POINTER(vp)]
    lib.fq_engine_read_acc.argtypes = [vp, vp, ctypes.c_size_t]
    lib.fq_engine_reset_acc.argtypes = [vp]
    lib.fq_engine_set_acc_buffer.argtypes = [vp, vp]
    lib.fq_engine_sync.argtypes = [vp]
    lib.fq_engine_last_error.argtypes = [vp]
    lib.fq_engine_last_error.restype = ctypes.c_char_p
    lib.fq_engine_device_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_size_t]
    lib.fq_synth_fill_device.argtypes = [ctypes.POINTER(FqBatch), u64, u64, i32, vp]
    lib.fq_engine_last_kernel_ms.argtypes = [vp]
    lib.fq_engine_last_kernel_ms.restype = ctypes.c_double
    lib.fq_engine_submit.argtypes = [vp, ctypes.POINTER(FqBatch), vp, u64]
    lib.fq_engine_submit_text.argtypes = [vp, ctypes.POINTER(FqTextBatch), vp, ctypes.POINTER(FqTextOut), u64]
    lib.fq_engine_poll.argtypes = [vp, ctypes.c_int, ctypes.POINTER(u64)]
    lib.fq_engine_pending.argtypes = [vp]
    lib.fq_engine_raw_begin.argtypes = [vp, u64, u64]
    lib.fq_engine_raw_enqueue.argtypes = [vp, ctypes.POINTER(FqRawWindow)]
    lib.fq_engine_raw_launch.argtypes = [vp, ctypes.POINTER(FqRawResult), ctypes.POINTER(FqRawOut), u64]
    lib.fq_engine_raw_wait.argtypes = [vp, ctypes.POINTER(FqRawResult)]
    lib.fq_engine_raw_end.argtypes = [vp]
    lib.fq_host_register.argtypes = [vp, ctypes.c_size_t]
    lib.fq_host_unregister.argtypes = [vp]
    lib.fq_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
    lib.fq_host_free.argtypes = [vp]
    lib.fq_dup_create.argtypes = [ctypes.c_int, i32, ctypes.POINTER(vp)]
    lib.fq_dup_destroy.argtypes = [vp]
    lib.fq_dup_reset.argtypes = [vp]
    lib.fq_engine_set_dup.argtypes = [vp, vp]
    lib.fq_dup_merge.argtypes = [vp, vp]
    lib.fq_dup_stat.argtypes = [vp, i32, vp, vp, vp]
    lib.fq_kmer_open.argtypes = [ctypes.c_int, vp, vp, i32, ctypes.POINTER(vp)]
    lib.fq_kmer_close.argtypes = [vp]
    lib.fq_kmer_count.argtypes = [vp, i32, i32, i32, vp]
    lib.fq_kmer_find.argtypes = [vp, i32, i32, i32, ctypes.c_uint32, vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    return lib


ENGINE_SYMBOLS = [
    "fq_engine_create", "fq_engine_destroy", "fq_engine_process", "fq_engine_process_device",
    "fq_engine_acc_words", "fq_engine_acc_device_ptr", "fq_engine_read_acc", "fq_engine_reset_acc",
    "fq_engine_sync", "fq_engine_set_acc_buffer", "fq_engine_last_error", "fq_engine_device_info", "fq_synth_fill_device",
    "fq_engine_last_kernel_ms", "fq_engine_submit", "fq_engine_submit_text", "fq_engine_poll", "fq_engine_pending", "fq_host_alloc",
    "fq_host_free", "fq_dup_create", "fq_dup_destroy", "fq_dup_reset", "fq_engine_set_dup", "fq_dup_merge",
    "fq_dup_stat", "fq_kmer_open", "fq_kmer_close", "fq_kmer_count", "fq_kmer_find",
    "fq_engine_raw_begin", "fq_engine_raw_enqueue", "fq_engine_raw_launch", "fq_engine_raw_wait", "fq_engine_raw_end", "fq_host_register", "fq_host_unregister",
]


def load_host(path=HOST_LIB):
    """Load libfqhost.so (include/fqhost.h) after the engine (it links libfqengine.so)."""
    load_engine()
    lib = ctypes.CDLL(path)
    vp, ci, cs = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    argv_t = ctypes.POINTER(ctypes.c_char_p)
    lib.fqh_run.argtypes = [ci, argv_t]
    lib.fqh_json_double.argtypes = [ctypes.c_double, ctypes.c_char_p, cs]
    lib.fqh_merged_name.argtypes = [ctypes.c_char_p, ci, ci, ctypes.c_char_p, cs]
    lib.fqh_evaluate_read_len.argtypes = [ctypes.c_char_p]
    lib.fqh_detect_adapter.argtypes = [ctypes.c_char_p, ci, ctypes.c_char_p, cs]
    lib.fqh_report_json.argtypes = [ci, ctypes.c_char_p, vp, ci, ctypes.c_char_p]
    lib.fqh_report_json.restype = vp
    lib.fqh_free.argtypes = [vp]
    lib.fqh_session_open.argtypes = [ci, argv_t, ctypes.POINTER(vp)]
    lib.fqh_session_error.argtypes = [vp]
    lib.fqh_session_error.restype = ctypes.c_char_p
    lib.fqh_session_params.argtypes = [vp, ci, ctypes.POINTER(FqParams)]
    lib.fqh_session_next.argtypes = [vp, ci, ctypes.POINTER(FqBatch)]
    lib.fqh_session_consume.argtypes = [vp, vp, ci]
    lib.fqh_session_add_acc.argtypes = [vp, vp, ci]
    lib.fqh_session_dup_params.argtypes = [vp, ctypes.POINTER(ci), ctypes.POINTER(ci), ctypes.POINTER(ci)]
    lib.fqh_session_set_dup.argtypes = [vp, vp, vp, vp]
    lib.fqh_session_finish.argtypes = [vp]
    lib.fqh_session_finish.restype = vp
    lib.fqh_session_close.argtypes = [vp]
    lib.fqh_set_kmer_backend.argtypes = [vp]
    lib.fqh_debug_records.argtypes = [ctypes.c_char_p, ci, ci, ci, ci]
    lib.fqh_debug_records.restype = vp
    return lib


def take_string(lib, ptr):
    """Copy and free a malloc'd string returned by libfqhost."""
    s = ctypes.string_at(ptr).decode()
    lib.fqh_free(ptr)
    return s


HOST_SYMBOLS = [
    "fqh_run", "fqh_json_double", "fqh_merged_name", "fqh_evaluate_read_len", "fqh_detect_adapter",
    "fqh_report_json", "fqh_free", "fqh_session_open", "fqh_session_error", "fqh_session_params",
    "fqh_session_next", "fqh_session_consume", "fqh_session_add_acc", "fqh_session_finish",
    "fqh_session_close", "fqh_debug_records", "fqh_session_dup_params", "fqh_session_set_dup",
    "fqh_set_kmer_backend", "fqh_pargz_read_all", "fqh_gzread_all", "fqh_gz_drain",
]
