"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/fqengine.h
declares, agrees with the Python mirror of its structs, and refuses to run without a gfx950
device (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

from fqtool_amd import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "fqengine.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*|double)\s+(fq_\w+)\s*\(", text, re.M)))


def test_engine_exports_every_declared_symbol():
    if not os.path.exists(abi.ENGINE_LIB):
        subprocess.run(["make", "-s", "-C", REPO, "engine"], check=True)
    lib = abi.load_engine()
    declared = header_functions()
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(abi.ENGINE_SYMBOLS) == sorted(n for n in declared if not n.startswith("fq_acc_"))


def test_struct_sizes_match_oracle(oracle):
    assert ctypes.sizeof(abi.FqReadResult) == 16
    assert oracle.orc_sizeof_params() == ctypes.sizeof(abi.FqParams)


def test_no_device_no_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = abi.load_engine()
    p = abi.default_params()
    h = ctypes.c_void_p()
    rc = lib.fq_engine_create(ctypes.byref(p), 0, 16, 160, ctypes.byref(h))
    assert rc == -2, rc
    assert b"no HIP device" in lib.fq_engine_last_error(None) or b"gfx950" in lib.fq_engine_last_error(None)


def host_functions():
    text = open(os.path.join(REPO, "include", "fqhost.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|char\*|void|const char\*)\s+(fqh_\w+)\s*\(", text, re.M)))


def test_host_exports_every_declared_symbol():
    if not os.path.exists(abi.HOST_LIB) or not os.path.exists(abi.FQTOOL_BIN):
        subprocess.run(["make", "-s", "-C", REPO, "host"], check=True)
    lib = abi.load_host()
    declared = host_functions()
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(abi.HOST_SYMBOLS) == declared


def test_tool_refuses_to_run_without_device(tmp_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    inp = os.path.join(REPO, "tests", "golden", "inputs", "polygr1.fq")
    p = subprocess.run([abi.FQTOOL_BIN, "-i", inp, "-o", str(tmp_path / "o.fq"), "-J", str(tmp_path / "r.json")],
                       capture_output=True, cwd=tmp_path)
    assert p.returncode == 255
    assert b"no CPU fallback" in p.stderr
