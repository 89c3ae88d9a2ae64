"""The host pipeline under ThreadSanitizer (the reader, one dispatcher per engine, the
formatter, the writers, the pool and the detection thread run instrumented, with the oracle standing
in for the engine): byte-identical outputs and no TSan report.  A representative subset here; the
full sweep over every golden case at -w 4 and -w 16 is tools/tsan_sweep.py (log under profiles/)."""
import pytest

import tsan_util as T

pytestmark = pytest.mark.skipif(not T.tsan_available(), reason="libtsan not installed")


@pytest.fixture(scope="module")
def tsan_build():
    T.build()


@pytest.mark.parametrize("case,workers", [("td_pe_qag", 4), ("td_pe_gz", 16), ("td_se_split_num_many", 3),
                                          ("td_pe_merge", 4), ("td_pe_correct", 4), ("td_pe_dup", 4),
                                          ("td_pe_umi_perread", 16), ("synth_pe_c5", 16)])
def test_host_pipeline_under_tsan(case, workers, tsan_build, tmp_path):
    err, reports = T.run_case(case, str(tmp_path), workers, devices=2)
    assert reports == 0, err[-6000:]


@pytest.mark.parametrize("workers", [4, 16])
def test_bgzf_inputs_under_tsan(workers, tsan_build, tmp_path):
    """BGZF inputs: members inflated on up to 8 threads per mate, one batch ahead of the parser."""
    import gzip
    import os

    import e2e_util as E
    from test_host_e2e import bgzf

    inp, out = tmp_path / "in", tmp_path / "out"
    inp.mkdir()
    out.mkdir()
    for name in ("r1.fq.gz", "r2.fq.gz"):
        with open(os.path.join(E.INPUTS, name), "rb") as f:
            (inp / name).write_bytes(bgzf(gzip.decompress(f.read()), member=30_000))
    err, reports = T.run_case("td_pe_qag", str(out), workers, devices=2, inputs=str(inp))
    assert reports == 0, err[-6000:]


@pytest.mark.parametrize("case,devices", [("td_pe_qag", 3), ("td_pe_merge", 3), ("synth_pe_c3", 3), ("td_se_q", 3),
                                          ("td_pe_qag", 4), ("td_pe_merge", 4)])
def test_raw_stream_under_tsan(case, devices, tsan_build, tmp_path):
    """The raw stream on three / four engines (plain inputs, 4 KiB first window, 7-pair packs): the
    window reader thread, the per-engine threads with RawMulti's index waits, ordered turns and
    stage queues, end_locked, and the host reader's resume."""
    env = {"FQ_RAW_WINDOW0": "4096"}
    err, reports = T.run_case(case, str(tmp_path), 4, devices=devices, mode="raw", env_extra=env, pack_pairs=7)
    assert "raw stream on %d engines" % devices in err, err[-3000:]
    assert reports == 0, err[-6000:]


@pytest.mark.parametrize("case,zc", [("td_pe_qag", "1"), ("synth_pe_c3", "1"), ("td_se_q", "1"), ("td_pe_qag", "0")])
def test_records_only_egress_under_tsan(case, zc, tsan_build, tmp_path):
    """Records-only egress on one engine (FQ_RAW_EGRESS=host): the formatter copies each carry from
    the previous window and hands windows back through shared holds; with zero copy (FQ_RAW_ZC=1)
    the writer threads write byte ranges of the windows and release them when done."""
    env = {"FQ_RAW_WINDOW0": "4096", "FQ_RAW_EGRESS": "host", "FQ_RAW_ZC": zc}
    err, reports = T.run_case(case, str(tmp_path), 4, devices=1, mode="raw", env_extra=env, pack_pairs=7)
    assert "records-only egress" in err, err[-3000:]
    assert reports == 0, err[-6000:]


@pytest.mark.parametrize("case", ["td_pe_gz", "td_pe_merge"])
def test_text_packs_under_tsan(case, tsan_build, tmp_path):
    err, reports = T.run_case(case, str(tmp_path), 4, devices=2, mode="text", pack_pairs=7)
    assert reports == 0, err[-6000:]


@pytest.mark.parametrize("case,workers", [("td_pe_gz", 4), ("td_pe_qag", 16), ("td_se_q", 4)])
def test_gzip_raw_stream_under_tsan(case, workers, tsan_build, tmp_path):
    """Single-stream gzip inputs on the raw stream (one engine): each mate's parallel inflater (4 KiB
    chunks, so many chunks and workers) read in order by the window reader."""
    env = {"FQ_RAW_WINDOW0": "4096", "FQ_PARGZ_CHUNK": "4096"}
    err, reports = T.run_case(case, str(tmp_path), workers, devices=1, mode="rawgz", env_extra=env, pack_pairs=7)
    assert "gzip inputs inflated" in err, err[-3000:]
    assert reports == 0, err[-6000:]
