"""The host's JSON number formatter against the reference's own writer (nlohmann 3.5.0 Grisu2 as
vendored in src/json.hpp): tests/golden/grisu2_vectors.tsv was produced by compiling that header
(tests/golden/make_grisu.py); plus the small host helpers the report depends on."""
import ctypes
import os
import struct

import pytest

from fqtool_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def host():
    return abi.load_host()


def test_grisu2_vectors(host):
    buf = ctypes.create_string_buffer(64)
    bad = []
    n = 0
    with open(os.path.join(GOLDEN, "grisu2_vectors.tsv")) as f:
        for line in f:
            hx, want = line.rstrip("\n").split("\t")
            v = struct.unpack("<d", bytes.fromhex(hx)[::-1])[0]
            host.fqh_json_double(v, buf, 64)
            n += 1
            if buf.value.decode() != want:
                bad.append((hx, want, buf.value.decode()))
    assert n > 40000
    assert not bad, bad[:10]


@pytest.mark.parametrize("name,l1,l2,want", [
    ("@A00399:61:HG 1:N:0:ACGT", 120, 30, "@A00399:61:H_merged_120_30 1:N:0:ACGT"),
    ("@SYN:7:FC1:12 1:N:0", 151, 0, "@SYN:7:FC1:1_merged_151_0 1:N:0"),
    ("@noSpace", 5, 7, "_merged_5_7"),
    ("@ x", 1, 2, "_merged_1_2 x"),
])
def test_merged_name(host, name, l1, l2, want):
    # OverlapAnalysis::merge drops the character before the first space (src/overlapanalysis.cpp)
    buf = ctypes.create_string_buffer(256)
    host.fqh_merged_name(name.encode(), l1, l2, buf, 256)
    assert buf.value.decode() == want


def test_evaluate_read_len(host):
    assert host.fqh_evaluate_read_len(os.path.join(GOLDEN, "inputs", "r1.fq.gz").encode()) == 150
    assert host.fqh_evaluate_read_len(os.path.join(GOLDEN, "inputs", "edge_r1.fq").encode()) == 300
