"""The parallel single-stream gzip inflater (fqtool_amd/host/pargz.cpp) against zlib's gzread in the
reference's 1 MiB calls (src/fqreader.cpp:28-47), byte for byte, on the CPU.

The stream it hands out must be exactly the bytes the reference's reader gets -- on clean files
(gzip levels 1, 6, 9, stored blocks, fixed-Huffman blocks, the golden inputs), and on corrupt ones
(truncation, flipped bytes, a bad CRC32 or ISIZE, trailing garbage, several members), where the
reference's stream ends at the start of the gzread call that fails.  Small chunks (4-64 KiB of
compressed data) make every file span many chunks, so the block-start search, the verification of
each chunk's start against the previous chunk's end, the re-decode of chunks whose start is wrong or
missing, the marker resolution and the fallback to zlib are all exercised."""
import ctypes
import gzip
import os
import random
import subprocess
import zlib

import pytest

from fqtool_amd import abi
import e2e_util as E

LIB = os.path.join(abi.REPO_DIR, "fqtool_amd", "lib", "libfqhost.so")
CALL = 1 << 20


@pytest.fixture(scope="module")
def host():
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "host"], check=True)
    lib = ctypes.CDLL(LIB)
    lib.fqh_pargz_read_all.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(ctypes.c_int)]
    lib.fqh_gzread_all.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
    lib.fqh_free.argtypes = [ctypes.c_void_p]
    return lib


def par(lib, path, chunk, threads, call=CALL):
    p, n, ok = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_int()
    rc = lib.fqh_pargz_read_all(str(path).encode(), call, threads, chunk, ctypes.byref(p), ctypes.byref(n),
                                ctypes.byref(ok))
    if rc <= 0:
        return rc, None, None
    b = ctypes.string_at(p, n.value)
    lib.fqh_free(p)
    return rc, b, ok.value


def ref(lib, path, call=CALL):
    p, n, ok = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_int()
    assert lib.fqh_gzread_all(str(path).encode(), call, ctypes.byref(p), ctypes.byref(n), ctypes.byref(ok)) == 0
    b = ctypes.string_at(p, n.value)
    lib.fqh_free(p)
    return b, ok.value


def fastq_text(n, seed, L=150):
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        seq = "".join(rnd.choice("ACGT") for _ in range(L))
        qual = "".join(chr(33 + min(41, max(2, int(rnd.gauss(30, 8))))) for _ in range(L))
        out.append(f"@SYN:{seed}:{i} 1:N:0:ACGTACGT\n{seq}\n+\n{qual}\n")
    return "".join(out).encode()


def gz_member(data, level, strategy=zlib.Z_DEFAULT_STRATEGY, mtime=0):
    c = zlib.compressobj(level, zlib.DEFLATED, 31, 8, strategy)
    return c.compress(data) + c.flush()


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("pargz")
    text = fastq_text(6000, 7)
    made = {}
    for name, blob in [("l1", gz_member(text, 1)), ("l6", gz_member(text, 6)), ("l9", gz_member(text, 9)),
                       ("fixed", gz_member(text, 6, zlib.Z_FIXED)), ("stored", gz_member(text, 0)),
                       ("huffonly", gz_member(text, 6, zlib.Z_HUFFMAN_ONLY)), ("rle", gz_member(text, 6, zlib.Z_RLE))]:
        p = d / (name + ".fq.gz")
        p.write_bytes(blob)
        made[name] = p
    for g in ("r1.fq.gz", "r2.fq.gz", "synth_r1.fq.gz"):
        made[g] = os.path.join(E.INPUTS, g)
    return d, made, text


@pytest.mark.parametrize("name", ["l1", "l6", "l9", "fixed", "stored", "huffonly", "rle", "r1.fq.gz", "r2.fq.gz",
                                  "synth_r1.fq.gz"])
@pytest.mark.parametrize("chunk,threads", [(4096, 3), (16384, 2), (65536, 4), (65536, 1)])
def test_clean_streams_match_gzread(host, files, name, chunk, threads):
    _, made, _ = files
    path = made[name]
    want, wok = ref(host, path)
    rc, got, ok = par(host, path, chunk, threads)
    if rc == 0:
        assert os.path.getsize(path) < 2 * chunk  # (too small to split)
        return
    assert rc == 1, "a clean single-member file stays on the parallel path"
    assert ok == wok == 1
    assert got == want


def corrupt_variants(blob):
    """(label, bytes) of damaged copies of one gzip member"""
    n = len(blob)
    out = [("truncated_mid", blob[: n // 2]), ("truncated_tail", blob[: n - 3]), ("no_trailer", blob[: n - 8])]
    for frac in (0.1, 0.37, 0.5, 0.83, 0.97):
        b = bytearray(blob)
        b[int(n * frac)] ^= 0x5A
        out.append((f"flip_{frac}", bytes(b)))
    b = bytearray(blob)
    b[-8] ^= 1  # CRC32
    out.append(("bad_crc", bytes(b)))
    b = bytearray(blob)
    b[-4] ^= 1  # ISIZE
    out.append(("bad_isize", bytes(b)))
    out.append(("trailing_garbage", blob + b"garbage after the member\n"))
    out.append(("trailing_zeros", blob + bytes(4096)))
    return out


@pytest.mark.parametrize("chunk", [4096, 32768])
def test_corrupt_streams_match_gzread(host, files, chunk):
    d, _, text = files
    blob = gz_member(text, 6)
    for label, data in corrupt_variants(blob):
        p = d / f"bad_{label}_{chunk}.fq.gz"
        p.write_bytes(data)
        want, wok = ref(host, p)
        rc, got, ok = par(host, p, chunk, 3)
        if rc == 0:
            continue
        assert (got, ok) == (want, wok), f"{label}: {len(got)} bytes ok={ok} vs gzread {len(want)} ok={wok}"


def test_several_members_match_gzread(host, files):
    d, _, text = files
    half = len(text) // 2
    p = d / "two_members.fq.gz"
    p.write_bytes(gz_member(text[:half], 6) + gz_member(text[half:], 1))
    want, wok = ref(host, p)
    rc, got, ok = par(host, p, 8192, 3)
    assert rc == 2  # (handed to zlib's reader: the parallel path takes one member)
    assert (got, ok) == (want, wok) and wok == 1 and want == text


def test_small_calls(host, files):
    """a gzread call smaller than a chunk: bytes go out call by call"""
    _, made, _ = files
    want, wok = ref(host, made["l6"], call=1000)
    rc, got, ok = par(host, made["l6"], 16384, 3, call=1000)
    assert rc == 1 and (got, ok) == (want, wok)


def _gz_cases():
    return [c for c in E.ok_cases() if any(a.endswith(".gz") for a in E.argv_for("x", c, "/o")[1:] if a.startswith(E.INPUTS))]


@pytest.mark.parametrize("case", _gz_cases())
def test_tool_with_small_chunks_cpu(case, tmp_path):
    """The tool itself (CPU stand-in engine) reading the golden gzip inputs through 4 KiB chunks:
    outputs and JSON as the reference's."""
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "cpuhost"], check=True)
    binp = os.path.join(abi.REPO_DIR, "build", "cpuhost", "fqtool")
    outd = tmp_path / "out"
    outd.mkdir()
    argv = E.argv_for(binp, case, str(outd))
    env = dict(os.environ, FQ_PARGZ_CHUNK="4096")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    E.check_outputs(case, str(outd))


REF_BIN = os.path.join(abi.REPO_DIR, "oracle", "_ref", "fqtool_ref")


@pytest.mark.parametrize("label", ["flip_0.37", "flip_0.83", "bad_crc", "truncated_mid", "trailing_garbage"])
def test_tool_matches_reference_on_corrupt_gzip(label, tmp_path):
    """Read 1 as one re-compressed gzip member with damage: the tool (CPU stand-in engine, parallel
    inflate on 8 KiB chunks) and the reference binary built here (oracle/_ref) give the same outputs,
    JSON sections and the reference's error message."""
    if not os.path.exists(REF_BIN):
        pytest.skip("reference binary not built (oracle/Makefile.ref)")
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "cpuhost"], check=True)
    cpu_bin = os.path.join(abi.REPO_DIR, "build", "cpuhost", "fqtool")
    ind = tmp_path / "in"
    ind.mkdir()
    # several MiB of text, so the reference's 1 MiB gzread calls matter (the golden pair repeated)
    with gzip.open(os.path.join(E.INPUTS, "r1.fq.gz"), "rb") as f:
        t1 = f.read() * 3
    with gzip.open(os.path.join(E.INPUTS, "r2.fq.gz"), "rb") as f:
        t2 = f.read() * 3
    bad = dict(corrupt_variants(gz_member(t1, 6)))[label]
    (ind / "r1.fq.gz").write_bytes(bad)
    (ind / "r2.fq.gz").write_bytes(gz_member(t2, 6))
    outs = {}
    for tool in ("ours", "ref"):
        od = tmp_path / tool
        od.mkdir()
        argv = [cpu_bin if tool == "ours" else REF_BIN, "-w", "1", "-i", str(ind / "r1.fq.gz"), "-I",
                str(ind / "r2.fq.gz"), "-o", str(od / "o1.fq"), "-O", str(od / "o2.fq"), "-q", "-g",
                "-J", str(od / "r.json"), "-H", str(od / "r.html")]
        env = dict(os.environ, FQ_PARGZ_CHUNK="8192")
        p = subprocess.run(argv, capture_output=True, cwd=od, timeout=300, env=env)
        outs[tool] = (od, p.returncode, p.stderr.decode(errors="replace"))
    assert outs["ours"][1] == outs["ref"][1], (outs["ours"][2][-1500:], outs["ref"][2][-1500:])
    assert ("Error to read gzip file" in outs["ours"][2]) == ("Error to read gzip file" in outs["ref"][2])
    for n in ("o1.fq", "o2.fq"):
        a, b = (outs[t][0] / n for t in ("ours", "ref"))
        assert a.exists() == b.exists()
        if a.exists():
            assert a.read_bytes() == b.read_bytes(), n
    import json
    if (outs["ref"][0] / "r.json").exists():
        a, b = (json.loads((outs[t][0] / "r.json").read_text()) for t in ("ours", "ref"))
        for k in ("summary", "filtering_result", "read1_before_filtering", "read2_after_filtering"):
            assert a.get(k) == b.get(k), k


def test_pigz_style_stream(host, files, tmp_path):
    """bench.py's gzip -6 inputs: pieces deflated apart (each primed with the previous 32 KiB) and
    joined by full flushes into one member -- empty stored blocks at byte boundaries mid-stream"""
    import sys
    sys.path.insert(0, abi.REPO_DIR)
    import bench
    _, _, text = files
    src = tmp_path / "t.fq"
    src.write_bytes(text)
    p = bench.gzip_single_member(str(src), str(tmp_path / "t.fq.gz"), threads=3, piece=65536)
    assert gzip.open(p).read() == text
    want, wok = ref(host, p)
    for chunk in (4096, 16384):
        rc, got, ok = par(host, p, chunk, 3)
        assert rc == 1 and (got, ok) == (want, wok)


@pytest.mark.parametrize("where", [0.3, 0.7])
def test_tool_resumes_gzip_stream_after_irregular_record(where, tmp_path):
    """A "\\r\\n" record part way into read 1 (a clean gzip member): the raw stream stops there and the
    host reader resumes on the gzip stream (read again from its start up to the stop) -- outputs and
    JSON as the reference binary's."""
    if not os.path.exists(REF_BIN):
        pytest.skip("reference binary not built (oracle/Makefile.ref)")
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "cpuhost"], check=True)
    cpu_bin = os.path.join(abi.REPO_DIR, "build", "cpuhost", "fqtool")
    ind = tmp_path / "in"
    ind.mkdir()
    with gzip.open(os.path.join(E.INPUTS, "r1.fq.gz"), "rb") as f:
        t1 = f.read() * 3
    with gzip.open(os.path.join(E.INPUTS, "r2.fq.gz"), "rb") as f:
        t2 = f.read() * 3
    lines = t1.split(b"\n")
    k = int(len(lines) * where) // 4 * 4
    for j in range(k, k + 4):
        lines[j] += b"\r"
    (ind / "r1.fq.gz").write_bytes(gz_member(b"\n".join(lines), 6))
    (ind / "r2.fq.gz").write_bytes(gz_member(t2, 6))
    outs = {}
    for tool in ("ours", "ref"):
        od = tmp_path / tool
        od.mkdir()
        argv = [cpu_bin if tool == "ours" else REF_BIN, "-w", "2", "-i", str(ind / "r1.fq.gz"), "-I",
                str(ind / "r2.fq.gz"), "-o", str(od / "o1.fq"), "-O", str(od / "o2.fq"), "-q", "-g",
                "-J", str(od / "r.json"), "-H", str(od / "r.html")]
        env = dict(os.environ, FQ_PARGZ_CHUNK="8192", FQ_RAW_WINDOW0="65536")
        p = subprocess.run(argv, capture_output=True, cwd=od, timeout=300, env=env)
        outs[tool] = (od, p.returncode, p.stderr.decode(errors="replace"))
    assert outs["ours"][1] == outs["ref"][1] == 0, (outs["ours"][2][-1500:], outs["ref"][2][-1500:])
    assert "irregular record" in outs["ours"][2], outs["ours"][2][-1500:]
    for n in ("o1.fq", "o2.fq"):
        assert (outs["ours"][0] / n).read_bytes() == (outs["ref"][0] / n).read_bytes(), n
    import json
    a, b = (json.loads((outs[t][0] / "r.json").read_text()) for t in ("ours", "ref"))
    for k in ("summary", "filtering_result", "read1_before_filtering", "read2_after_filtering"):
        assert a.get(k) == b.get(k), k


def test_highly_compressible_stream_goes_to_zlib(host, tmp_path):
    """A stream that inflates far beyond FASTQ's ratios (runs of one byte, ~1000:1) exceeds the
    per-chunk output cap (16 times the chunk's compressed bytes, at least 16 MiB): the file goes to
    zlib's reader, byte for byte as gzread, instead of holding gigabytes per chunk in flight."""
    text = (b"@r\n" + b"A" * 100000 + b"\n+\n" + b"F" * 100000 + b"\n") * 500
    p = tmp_path / "runs.fq.gz"
    p.write_bytes(gz_member(text, 6))
    want, wok = ref(host, p)
    rc, got, ok = par(host, p, 32768, 3)
    assert rc == 2 and (got, ok) == (want, wok) and want == text
