"""End-to-end parity of the tool against the reference binary's outputs (tests/golden/e2e, made
by tests/golden/make_e2e.py from oracle/_ref/fqtool_ref runs with -w 1).

CPU: the host pipeline (CLI, FASTQ packing, output formatting/writers, JSON report) driven through
the libfqhost session API with the CPU oracle standing in for the engine, and the CLI's error
behaviour (exit status + message) of the real binary, which fails before touching a device.
GPU: the real `fqtool` binary, engine on MI355X, byte-identical outputs and JSON.
"""
import ctypes
import gzip
import os
import struct
import subprocess
import zlib

import pytest

import e2e_util as E
from fqtool_amd import abi


@pytest.fixture(scope="module")
def host(oracle):
    """libfqhost with the adapter-detection k-mer work on the CPU restatement (the tool itself
    runs it on the GPU; the CPU suite has no device)."""
    if not (os.path.exists(abi.HOST_LIB) and os.path.exists(abi.FQTOOL_BIN)):
        subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "host"], check=True)
    lib = abi.load_host()
    backend = E.oracle_kmer_backend(oracle)
    lib.fqh_set_kmer_backend(ctypes.addressof(backend))
    yield lib
    lib.fqh_set_kmer_backend(None)


@pytest.mark.parametrize("case", E.ok_cases())
def test_host_pipeline_with_oracle_engine(case, host, oracle, tmp_path):
    argv = E.argv_for("fqtool", case, str(tmp_path))
    report = E.run_session_with_oracle(host, oracle, argv)
    E.check_outputs(case, str(tmp_path), report)


@pytest.mark.parametrize("case", E.ok_cases())
def test_host_pipeline_threaded(case, host, oracle, tmp_path):
    """Same with -w 4 and small packs: tile packing, output formatting (blocks) and gzip members
    run on the host pool; outputs and JSON must not change."""
    argv = E.argv_for("fqtool", case, str(tmp_path))
    assert argv[1:3] == ["-w", "1"]
    if not E.is_split(case):  # with -s / -S, -w is the number of file sequences
        argv[2] = "4"
    report = E.run_session_with_oracle(host, oracle, argv, max_n=700)
    E.check_outputs(case, str(tmp_path), report)


def bgzf(raw, level=6, member=0xff00):
    """BGZF (SAM/BAM spec 4.1) members of `member` input bytes each, then the empty EOF member."""
    out = bytearray()
    for o in range(0, len(raw), member):
        blk = raw[o:o + member]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        d = c.compress(blk) + c.flush()
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", len(d) + 25)
        out += d + struct.pack("<II", zlib.crc32(blk), len(blk))
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    d = c.compress(b"") + c.flush()
    out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", len(d) + 25)
    return bytes(out + d + struct.pack("<II", 0, 0))


@pytest.mark.parametrize("case,kind", [("td_pe_qag", "bgzf"), ("td_pe_gz", "bgzf"), ("td_se_q", "bgzf"),
                                       ("td_pe_split_num_gz", "bgzf"), ("td_pe_qag", "multi"), ("td_pe_qag", "bgzf_bad")])
def test_bgzf_and_multi_member_inputs(case, kind, host, oracle, tmp_path):
    """The testdata inputs recompressed as BGZF (members inflated on several threads by the bulk
    reader), as plain multi-member gzip (zlib's stream reader), and as BGZF whose last member's
    size field is off by one (not a BGZF chain: zlib's reader): the same outputs and JSON as the
    reference run on the original files.  The tool's own .gz outputs are BGZF."""
    inp, out = tmp_path / "in", tmp_path / "out"
    inp.mkdir()
    out.mkdir()
    for name in ("r1.fq.gz", "r2.fq.gz"):
        with open(os.path.join(E.INPUTS, name), "rb") as f:
            raw = gzip.decompress(f.read())
        if kind == "multi":
            data = b"".join(gzip.compress(raw[o:o + 100_000], 6) for o in range(0, len(raw), 100_000))
        else:
            data = bgzf(raw, member=30_000 if kind == "bgzf_bad" else 0xFF00)
            if kind == "bgzf_bad":  # BSIZE of the EOF member one too large: the chain overruns the file
                data = bytearray(data)
                data[-28 + 16] += 1
                data = bytes(data)
        (inp / name).write_bytes(data)
    argv = [a.replace(E.INPUTS, str(inp)) for a in E.argv_for("fqtool", case, str(out))]
    report = E.run_session_with_oracle(host, oracle, argv)
    E.check_outputs(case, str(out), report)
    for name in os.listdir(out):
        if name.endswith(".gz"):
            with open(out / name, "rb") as f:
                head = f.read(18)
            assert head[:4] == bytes([0x1F, 0x8B, 8, 4]) and head[12:14] == b"BC", name


@pytest.mark.parametrize("case", E.err_cases())
def test_cli_errors_match_reference(case, tmp_path):
    if not os.path.exists(abi.FQTOOL_BIN):
        subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "host"], check=True)
    m = E.manifest()[case]
    p = subprocess.run(E.argv_for(abi.FQTOOL_BIN, case, str(tmp_path)), capture_output=True, cwd=tmp_path,
                       timeout=120)
    assert p.returncode == m["exit"], p.stderr
    err = p.stderr.decode().replace(E.INPUTS, "{in}").replace(str(tmp_path), "{out}")
    if m["exit"] == 255:
        assert [l for l in err.splitlines() if l.startswith("ERROR:")] == \
            [l for l in m["stderr"].splitlines() if l.startswith("ERROR:")]
    else:
        assert err == m["stderr"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", E.ok_cases())
def test_fqtool_binary_matches_reference(case, tmp_path):
    p = subprocess.run(E.argv_for(abi.FQTOOL_BIN, case, str(tmp_path)), capture_output=True, cwd=tmp_path,
                       timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    E.check_outputs(case, str(tmp_path))


@pytest.mark.gpu
@pytest.mark.parametrize("case", E.ok_cases())
def test_fqtool_multi_engine_matches_reference(case, tmp_path):
    """Packs dealt round-robin over three engines (virtual devices on one GPU, each with its
    asynchronous pinned pipeline), small packs so every engine gets several, -w 4: the writer
    reorders by pack sequence number and the accumulators are summed, so the FASTQ and JSON
    must still equal the reference's -w 1 outputs."""
    argv = E.argv_for(abi.FQTOOL_BIN, case, str(tmp_path))
    if not E.is_split(case):
        argv[2] = "4"
    argv += ["--devices", "0,0,0", "--pack_pairs", "777"]
    p = subprocess.run(argv, capture_output=True, cwd=tmp_path, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert "on 3 engine(s)" in p.stderr.decode()
    E.check_outputs(case, str(tmp_path))


@pytest.mark.parametrize("case", ["td_pe_split_num", "td_se_split_lines", "td_se_split_num_many"])
def test_split_with_several_workers(case, host, oracle, tmp_path):
    """-s / -S with -w 3: each worker writes its own file sequence (t+1, t+1+3, ...; the
    reference's ThreadConfig).  Whatever the schedule, the files together hold exactly the
    records of the -w 1 run, each file a run of whole packs in input order."""
    import glob

    one, three = tmp_path / "w1", tmp_path / "w3"
    one.mkdir()
    three.mkdir()
    E.run_session_with_oracle(host, oracle, E.argv_for("fqtool", case, str(one)))
    argv = E.argv_for("fqtool", case, str(three))
    argv[2] = "3"
    E.run_session_with_oracle(host, oracle, argv)

    def records(d, mate):
        out = []
        for f in sorted(glob.glob(str(d / ("*." + mate)))):
            lines = open(f, "rb").read().split(b"\n")[:-1]
            out += [b"\n".join(lines[k:k + 4]) for k in range(0, len(lines), 4)]
        return out

    for mate in ("o1.fq", "o2.fq"):
        assert sorted(records(one, mate)) == sorted(records(three, mate))
    names = sorted(os.path.basename(f) for f in glob.glob(str(three / "0*")))
    assert names[0].startswith("0001.") and len(names) >= len(glob.glob(str(one / "0*")))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["0", "0,0,0", "0,0,0,0"])
@pytest.mark.parametrize("case", E.ok_cases())
def test_fqtool_raw_stream_small_windows_matches_reference(case, devices, tmp_path):
    """GPU record indexing (fq_engine_raw_*) under stress: gzip inputs are decompressed to plain
    files so every case with plain outputs takes the raw stream, the first window is 4 KiB and packs
    hold 7 pairs, so records straddle windows (the device carry), the mates' windows are sized
    apart, and irregular records (CR line ends, empty lines, long or lowercase reads, lines without
    '@') stop the stream mid-file for the host reader to resume at the reported offsets.  Outputs
    and JSON must still equal the reference's -w 1 outputs."""
    import gzip
    import shutil

    ind, outd = tmp_path / "in", tmp_path / "out"
    ind.mkdir()
    outd.mkdir()
    argv = E.argv_for(abi.FQTOOL_BIN, case, str(outd))
    for k, a in enumerate(argv):
        if a.startswith(E.INPUTS) and a.endswith(".fq.gz"):
            plain = ind / os.path.basename(a)[:-3]
            with gzip.open(a, "rb") as f, open(plain, "wb") as g:
                shutil.copyfileobj(f, g)
            argv[k] = str(plain)
    argv += ["--pack_pairs", "7"]
    if devices != "0" and not E.is_split(case):  # (-d tables merge across engines; split keeps -w)
        argv += ["--devices", devices]
    env = dict(os.environ, FQ_RAW_WINDOW0="4096")
    p = subprocess.run(argv, capture_output=True, cwd=outd, timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    if case in ("td_pe_qag", "td_pe_plain", "td_pe_detect", "synth_pe_c3", "synth_pe_c5", "synth_se_c2", "polygr_pe",
                "edge_pe_dup", "td_se_q", "td_pe_merge", "synth_pe_c4", "edge_pe_merge"):
        assert "raw stream" in p.stderr.decode(), p.stderr.decode()[-1000:]
        if devices != "0":
            assert "raw stream on %d engines" % len(devices.split(",")) in p.stderr.decode(), p.stderr.decode()[-1000:]
    E.check_outputs(case, str(outd))


@pytest.mark.parametrize("kind", ["bgzf", "bgzf_small_batches", "multi"])
def test_corrupt_member_keeps_the_good_prefix(kind, host, oracle, tmp_path, monkeypatch):
    """A CRC32 flipped in a middle member of read 1's .gz: the tool processes exactly the bytes the
    reference's stream delivers before the failure and reports the error.  The reference reads every
    gzip file in 1 MiB gzread calls (src/fqreader.cpp:28-35) and the call that meets the bad CRC
    returns -1, so the stream ends at that call's start -- the bad member's bytes before it included.
    Both readers here follow that: BGZF (members inflated in parallel, batches handed out up to their
    last call boundary until the next is known) and any other gzip (zlib's stream reader).
    Expected: the outputs of the same command on plain files holding that prefix (read 2 whole)."""
    member, bad = 0xFF00, 40
    if kind == "bgzf_small_batches":
        # ~256 KiB inflate batches: the bad member lies batches after the one holding the cut, so
        # the hold-back of each batch's bytes past its last 1 MiB boundary is what keeps them out
        monkeypatch.setenv("FQ_BGZF_BATCH", str(1 << 18))
        kind = "bgzf"
    raw = {}
    for name in ("r1.fq.gz", "r2.fq.gz"):
        with open(os.path.join(E.INPUTS, name), "rb") as f:
            raw[name] = gzip.decompress(f.read())
    gz, plain, out_gz, out_plain = (tmp_path / d for d in ("gz", "plain", "out_gz", "out_plain"))
    for d in (gz, plain, out_gz, out_plain):
        d.mkdir()
    for name, data in raw.items():
        if kind == "bgzf":
            comp = bytearray(bgzf(data, member=member))
        else:
            comp = bytearray(b"".join(gzip.compress(data[o:o + member], 6) for o in range(0, len(data), member)))
        keep = len(data)
        if name == "r1.fq.gz":
            # walk to member `bad`: BGZF headers carry BSIZE; plain members are re-compressed to find their sizes
            off = 0
            for k in range(bad):
                if kind == "bgzf":
                    off += struct.unpack("<H", bytes(comp[off + 16:off + 18]))[0] + 1
                else:
                    off += len(gzip.compress(data[k * member:(k + 1) * member], 6))
            if kind == "bgzf":
                end = off + struct.unpack("<H", bytes(comp[off + 16:off + 18]))[0] + 1
            else:
                end = off + len(gzip.compress(data[bad * member:(bad + 1) * member], 6))
            comp[end - 8] ^= 0x5A  # the member's CRC32
            stop = (bad + 1) * member  # decompressed end of the bad member
            keep = (stop - 1) // (1 << 20) * (1 << 20)  # the start of the gzread call that meets the bad CRC
        (gz / name).write_bytes(bytes(comp))
        (plain / name[:-3]).write_bytes(data[:keep])
    argv = E.argv_for("fqtool", "td_pe_qag", str(out_gz))
    argv_gz = [a.replace(E.INPUTS, str(gz)) for a in argv]
    argv_plain = [a.replace(E.INPUTS, str(plain)).replace(".fq.gz", ".fq") if a.startswith(E.INPUTS) else a
                  for a in E.argv_for("fqtool", "td_pe_qag", str(out_plain))]
    rep_gz = E.run_session_with_oracle(host, oracle, argv_gz)
    rep_plain = E.run_session_with_oracle(host, oracle, argv_plain)
    outs = sorted(n for n in os.listdir(out_gz) if not n.startswith("report."))
    assert outs == sorted(n for n in os.listdir(out_plain) if not n.startswith("report."))
    for n in outs:
        assert E.digest(str(out_gz / n)) == E.digest(str(out_plain / n)), n
    import json
    a, b = json.loads(rep_gz), json.loads(rep_plain)
    for k in ("summary", "filtering_result", "adapter_cutting", "read1_before_filtering", "read2_after_filtering"):
        assert a.get(k) == b.get(k), k


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in E.ok_cases() if any(a.endswith(".gz") for a in E.argv_for("x", c, "/o")[1:]
                                                                 if a.startswith(E.INPUTS))])
def test_fqtool_parallel_gzip_inputs_match_reference(case, tmp_path):
    """The golden cases with gzip inputs read through the parallel inflater (4 KiB chunks, so the
    small golden files split into many) -- on one engine straight into the raw stream's windows --
    and 4 KiB first windows: outputs and JSON as the reference's."""
    env = dict(os.environ, FQ_PARGZ_CHUNK="4096", FQ_RAW_WINDOW0="4096")
    p = subprocess.run(E.argv_for(abi.FQTOOL_BIN, case, str(tmp_path)), capture_output=True, cwd=tmp_path,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    E.check_outputs(case, str(tmp_path))
