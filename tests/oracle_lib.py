"""Loads the CPU restatement (oracle/build/liboracle.so) -- the parity CHECKER.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

from fqtool_amd import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")


class OrcOverlap(ctypes.Structure):
    _fields_ = [("overlapped", ctypes.c_int), ("offset", ctypes.c_int), ("overlap_len", ctypes.c_int),
                ("diff", ctypes.c_int)]


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load_oracle():
    build_oracle()
    lib = ctypes.CDLL(ORACLE_LIB)
    P = ctypes.POINTER(abi.FqParams)
    cp, ci = ctypes.c_char_p, ctypes.c_int
    ip = ctypes.POINTER(ctypes.c_int)
    lib.orc_pass_filter.argtypes = [P, cp, cp, ci, ci]
    lib.orc_trim_and_cut.argtypes = [P, cp, cp, ci, ci, ci, ip, ip]
    lib.orc_trim_polyg.argtypes = [cp, ci, ci, ci, ci, ip]
    lib.orc_trim_polyx.argtypes = [cp, ci, ci, ci, ci, ci, ip, ip]
    lib.orc_analyze.argtypes = [cp, ci, cp, ci, ci, ci]
    lib.orc_analyze.restype = OrcOverlap
    lib.orc_trim_by_sequence.argtypes = [cp, ci, cp, ci, ip]
    lib.orc_process_batch.argtypes = [P, ctypes.POINTER(abi.FqBatch), ctypes.c_void_p, ctypes.c_void_p]
    lib.orc_synth_fill.argtypes = [ctypes.POINTER(abi.FqBatch), ctypes.c_uint64, ctypes.c_uint64, ci]
    vp = ctypes.c_void_p
    lib.orc_dup_create.argtypes = [ci]
    lib.orc_dup_create.restype = vp
    lib.orc_dup_destroy.argtypes = [vp]
    lib.orc_dup_add_batch.argtypes = [vp, ctypes.POINTER(abi.FqBatch), ci]
    lib.orc_dup_stat.argtypes = [vp, ci, vp, vp, vp]
    lib.orc_kmer_open.argtypes = [ci, vp, vp, ctypes.c_int32, ctypes.POINTER(vp)]
    lib.orc_kmer_close.argtypes = [vp]
    lib.orc_kmer_count.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp]
    lib.orc_kmer_find.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, vp, ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_size_t)]
    lib.orc_sizeof_params.restype = ctypes.c_size_t
    lib.orc_sizeof_result.restype = ctypes.c_size_t
    assert lib.orc_sizeof_params() == ctypes.sizeof(abi.FqParams), "fq_params ABI mismatch"
    assert lib.orc_sizeof_result() == ctypes.sizeof(abi.FqReadResult) == 16
    return lib
