"""The tool's raw-stream and text-pack pipelines on the CPU (build/cpuhost/fqtool: the real host
sources linked against oracle/cpu_engine.cpp, which restates raw.hip's record cut / carry / stop and
text.hip's output text and merged stream on the CPU -- test infrastructure, never the product).

The GPU twin is tests/test_host_e2e.py::test_fqtool_raw_stream_small_windows_matches_reference;
here the same stress runs without a GPU, so the host side of the raw stream (the window reader,
one thread per engine, the ordered enqueue / launch hand-offs of RawMulti, the host reader's
resume where the stream stops, the writers) is covered by the CPU suite: 4 KiB first windows,
7-pair packs, 1 and 3 engines, and the records-only egress (FQ_RAW_EGRESS=host).  Outputs and
JSON must equal the reference's -w 1 outputs (tests/golden/e2e).  Irregular records placed inside
a later engine's window are checked against the reference binary built here (oracle/_ref)."""
import gzip
import os
import shutil
import subprocess

import pytest

import e2e_util as E
from fqtool_amd import abi

CPU_BIN = os.path.join(abi.REPO_DIR, "build", "cpuhost", "fqtool")
REF_BIN = os.path.join(abi.REPO_DIR, "oracle", "_ref", "fqtool_ref")


@pytest.fixture(scope="module")
def cpu_build():
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "cpuhost"], check=True)


def plain_inputs(argv, ind):
    """gzip inputs decompressed to plain files, so every case with plain outputs takes the raw stream"""
    for k, a in enumerate(argv):
        if a.startswith(E.INPUTS) and a.endswith(".fq.gz"):
            plain = os.path.join(ind, os.path.basename(a)[:-3])
            if not os.path.exists(plain):
                with gzip.open(a, "rb") as f, open(plain, "wb") as g:
                    shutil.copyfileobj(f, g)
            argv[k] = plain
    return argv


RAW_CASES = ("td_pe_qag", "td_pe_plain", "td_pe_detect", "synth_pe_c3", "synth_pe_c5", "synth_se_c2", "polygr_pe",
             "edge_pe_dup", "td_se_q", "td_pe_merge", "synth_pe_c4", "edge_pe_merge")


@pytest.mark.parametrize("devices", ["0", "0,0,0", "0,0,0,0"])
@pytest.mark.parametrize("case", E.ok_cases())
def test_raw_stream_small_windows_cpu(case, devices, cpu_build, tmp_path):
    ind, outd = tmp_path / "in", tmp_path / "out"
    ind.mkdir()
    outd.mkdir()
    argv = plain_inputs(E.argv_for(CPU_BIN, case, str(outd)), str(ind))
    argv += ["--pack_pairs", "7"]
    m = E.manifest()[case]
    multi = devices != "0" and not E.is_split(case) and " -d" not in m["args"]  # (-d tables merge on the GPU only)
    if multi:
        argv += ["--devices", devices]
    env = dict(os.environ, FQ_RAW_WINDOW0="4096")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=300, env=env)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 0, err[-2000:]
    if case in RAW_CASES:
        assert "raw stream" in err, err[-1000:]
        if multi:
            assert "raw stream on %d engines" % len(devices.split(",")) in err, err[-1000:]
    E.check_outputs(case, str(outd))


@pytest.mark.parametrize("devices", ["0,0,0,0", "0,0,0,0,0,0,0,0"])
@pytest.mark.parametrize("case", ["synth_pe_c3", "td_pe_merge"])
def test_raw_stream_slow_engines_cpu(case, devices, cpu_build, tmp_path):
    """Engines slower than the host (each pack >= 2 ms on the stand-in), 4 KiB first windows and 7-pair
    packs: every engine keeps its packs in flight, so the spare packs and staging windows run out
    while engines wait for their turns.  Each wait polls the engine's own packs, so the stream must
    finish (bounded by the timeout) with the reference's outputs (the turn holder waiting
    for a spare pack while every pack sat unpolled in an engine)."""
    ind, outd = tmp_path / "in", tmp_path / "out"
    ind.mkdir()
    outd.mkdir()
    argv = plain_inputs(E.argv_for(CPU_BIN, case, str(outd)), str(ind))
    argv += ["--pack_pairs", "7", "--devices", devices]
    env = dict(os.environ, FQ_RAW_WINDOW0="4096", FQ_CPU_ENGINE_DELAY_US="2000")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=240, env=env)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 0, err[-2000:]
    assert "raw stream on %d engines" % len(devices.split(",")) in err, err[-1000:]
    E.check_outputs(case, str(outd))


@pytest.mark.parametrize("devices", ["0", "0,0,0"])
def test_detection_error_after_pipeline_cpu(devices, cpu_build, tmp_path):
    """The PE adapter detection runs concurrently and is joined after the pipeline; when it fails
    there (the stand-in's k-mer device refuses, FQ_CPU_KMER_FAIL) the tool must report it as the
    reference reports a failed pre-pass -- "ERROR: ..." and exit status 255, no outputs left behind
    (src/main.cpp:137-141) -- not end in std::terminate (its completion promise was once set twice)."""
    ind, outd = tmp_path / "in", tmp_path / "out"
    ind.mkdir()
    outd.mkdir()
    argv = plain_inputs(E.argv_for(CPU_BIN, "td_pe_detect", str(outd)), str(ind)) + ["--devices", devices]
    env = dict(os.environ, FQ_CPU_KMER_FAIL="1")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=120, env=env)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 255, err[-2000:]
    assert "ERROR: adapter detection" in err and "terminate" not in err, err[-2000:]
    assert not (outd / "o1.fq").exists() and not (outd / "o2.fq").exists()


@pytest.mark.parametrize("zc", ["1", "0"])
@pytest.mark.parametrize("case", ["td_pe_qag", "synth_pe_c3", "td_pe_merge", "synth_se_c2", "edge_pe_all", "td_pe_plain",
                                  "td_se_q", "polygr_pe"])
def test_records_only_egress_cpu(case, zc, cpu_build, tmp_path):
    """FQ_RAW_EGRESS=host (one engine): the engine returns records and line offsets, the host formats
    from its staging windows (the carry in front of each window included) -- with plain outputs as
    byte ranges of the windows written by writev (FQ_RAW_ZC=1, the default), or copied (0)."""
    ind, outd = tmp_path / "in", tmp_path / "out"
    ind.mkdir()
    outd.mkdir()
    argv = plain_inputs(E.argv_for(CPU_BIN, case, str(outd)), str(ind)) + ["--pack_pairs", "7"]
    env = dict(os.environ, FQ_RAW_WINDOW0="4096", FQ_RAW_EGRESS="host", FQ_RAW_ZC=zc)
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    err = p.stderr.decode(errors="replace")
    if case in RAW_CASES:
        assert "raw stream" in err, err[-1000:]
        import re
        m = re.search(r"records-only egress: (\d+) packs, (\d+) as byte ranges", err)
        if "-m" not in E.manifest()[case]["args"].split():
            assert m and int(m.group(1)) > 0, err[-1000:]
            plain = not any(a.endswith(".gz") for a in argv if a.startswith(str(outd)))
            assert int(m.group(2)) == (int(m.group(1)) if zc == "1" and plain else 0), err[-1000:]
    E.check_outputs(case, str(outd))


@pytest.mark.parametrize("case", ["td_pe_gz", "td_pe_qag", "td_pe_merge", "td_se_q"])
def test_text_packs_cpu(case, cpu_build, tmp_path):
    """Text packs (the host parses, the engine builds the planes and writes the output text): gzip
    inputs as they are, on two engines."""
    outd = tmp_path / "out"
    outd.mkdir()
    argv = E.argv_for(CPU_BIN, case, str(outd)) + ["--pack_pairs", "7", "--devices", "0,0"]
    env = dict(os.environ, FQ_RAW_MODE="0")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    E.check_outputs(case, str(outd))


@pytest.mark.parametrize("kind", ["crlf", "empty_line"])
@pytest.mark.parametrize("merge", [False, True])
def test_irregular_record_mid_stream_second_engine(kind, merge, cpu_build, tmp_path):
    """An irregular record (a CRLF line end, or an empty line after a record) placed in the middle of
    the stream, inside a window owned by the second of three engines: the GPU path stops there, every
    later window is dropped unlaunched, and the host reader resumes at the reported offsets.  Outputs
    and JSON against the reference binary on the same input."""
    if not os.path.exists(REF_BIN):
        pytest.skip("reference binary not built (oracle/Makefile.ref)")
    src = {}
    for name in ("r1.fq.gz", "r2.fq.gz"):
        with gzip.open(os.path.join(E.INPUTS, name), "rb") as f:
            src[name] = f.read()
    ind = tmp_path / "in"
    ind.mkdir()
    # windows: the first is 4 KiB, later ones sized from the 7-pair packs -- record 30 of read 1
    # lies in window 4, which engine 1 of 3 takes
    for name, data in src.items():
        recs = _records_bytes(data)
        k = 30 if name == "r1.fq.gz" else None
        out = []
        for i, r in enumerate(recs):
            if k is not None and i == k:
                if kind == "crlf":
                    r = [r[0] + b"\r", r[1], r[2], r[3]]
                else:
                    r = r + [b""]
            out.append(b"\n".join(r) + b"\n")
        (ind / name[:-3]).write_bytes(b"".join(out))
    outs = {}
    for tool in ("ours", "ref"):
        od = tmp_path / tool
        od.mkdir()
        binary = CPU_BIN if tool == "ours" else REF_BIN
        argv = [binary, "-w", "1", "-i", str(ind / "r1.fq"), "-I", str(ind / "r2.fq"), "-J", str(od / "r.json"),
                "-H", str(od / "r.html"), "-q", "-a", "-g"]
        argv += ["-o", str(od / "o1.fq"), "-O", str(od / "o2.fq")]
        if merge:
            argv += ["-m", "--merge_output", str(od / "m.fq")]
        if tool == "ours":
            argv += ["--pack_pairs", "7", "--devices", "0,0,0"]
        env = dict(os.environ, FQ_RAW_WINDOW0="4096")
        p = subprocess.run(argv, capture_output=True, cwd=od, timeout=300, env=env)
        assert p.returncode == 0, p.stderr.decode()[-2000:]
        outs[tool] = (od, p.stderr.decode(errors="replace"))
    err = outs["ours"][1]
    assert "raw stream on 3 engines" in err, err[-1500:]
    import re
    mw = re.search(r"ended: irregular record in window (\d+)", err)
    assert mw and int(mw.group(1)) % 3 == 1, err[-1500:]  # (window k goes to engine k mod 3)
    for n in ["o1.fq", "o2.fq"] + (["m.fq"] if merge else []):
        assert (outs["ours"][0] / n).read_bytes() == (outs["ref"][0] / n).read_bytes(), n
    import json
    a, b = (json.loads((outs[t][0] / "r.json").read_text()) for t in ("ours", "ref"))
    for k in ("summary", "filtering_result", "adapter_cutting", "read1_before_filtering", "read2_after_filtering"):
        assert a.get(k) == b.get(k), k


def _records_bytes(data):
    lines = data.split(b"\n")
    return [lines[i:i + 4] for i in range(0, len(lines) - 3, 4)]
