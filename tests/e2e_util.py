"""End-to-end helpers: the golden manifest written by tests/golden/make_e2e.py (reference binary
runs), argv construction, and comparison of a run directory against it."""
import ctypes
import gzip
import hashlib
import json
import os
import re

import numpy as np

from fqtool_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INPUTS = os.path.join(GOLDEN, "inputs")
E2E = os.path.join(GOLDEN, "e2e")


def manifest():
    with open(os.path.join(E2E, "manifest.json")) as f:
        return json.load(f)


def ok_cases():
    return sorted(k for k, v in manifest().items() if v["exit"] == 0)


def err_cases():
    return sorted(k for k, v in manifest().items() if v["exit"] != 0)


def argv_for(binary, case, outdir):
    """Same argument order make_e2e.py used for the reference."""
    args = manifest()[case]["args"]
    argv = [binary, "-w", "1", "-J", os.path.join(outdir, "report.json"), "-H", os.path.join(outdir, "report.html")]
    return argv + args.format(**{"in": INPUTS, "out": outdir}).split()


def is_split(case):
    """-s / -S runs: the worker count -w changes which files the packs go to."""
    return " -s " in manifest()[case]["args"] + " " or " -S " in manifest()[case]["args"] + " "


def mask_se_dup(text):
    j = json.loads(text)
    h = j.get("Duplication", {}).get("Histogram")
    if h is not None:
        half = len(h) // 2
        j["Duplication"]["Histogram"] = h[:half] + [0] * (len(h) - half)
        return json.dumps(j, indent=4)
    return text


def mask_software(text):
    text = re.sub(r'"CWD": "[^"]*"', '"CWD": ""', text)
    return re.sub(r'"Command": "[^"]*"', '"Command": ""', text)


def mask_html(text):
    """The footer's time stamp and the Software rows (command line, cwd) vary per run."""
    text = re.sub(r"Fqtool Report @ [^<]*", "Fqtool Report @ ", text)
    text = re.sub(r'(<td class="col1">Command</td><td class="col2">)[^<]*', r"\1", text)
    return re.sub(r'(<td class="col1">CWD</td><td class="col2">)[^<]*', r"\1", text)


def mask_html_se_dup(text):
    """SE duplication percentages come from the partly uninitialised histogram (see mask_se_dup)."""
    return re.sub(r"(<script type=\"text/javascript\">var data=\[\{x:\[[^\]]*\],y:\[)[^\]]*(\],name: 'Read percent)"
                  r"[^<]*", r"\1\2", text)


def golden_html(case):
    with gzip.open(os.path.join(E2E, manifest()[case]["html"]), "rt") as f:
        return f.read()


def golden_json(case):
    with gzip.open(os.path.join(E2E, manifest()[case]["json"]), "rt") as f:
        return f.read()


def digest(path):
    data = open(path, "rb").read()
    if path.endswith(".gz"):
        data = gzip.decompress(data) if data else b""
    return {"sha256": hashlib.sha256(data).hexdigest(), "lines": data.count(b"\n")}


def check_outputs(case, outdir, report_text=None):
    """Asserts every output file and the JSON report equal the reference's."""
    m = manifest()[case]
    present = {}
    for name in sorted(os.listdir(outdir)):  # every output file but the reports
        if not name.startswith("report."):
            present[name] = digest(os.path.join(outdir, name))
    assert sorted(present) == sorted(m["outputs"]), (sorted(present), sorted(m["outputs"]))
    for name, d in m["outputs"].items():
        assert present[name] == d, "%s: %s differs from the reference (%s vs %s lines)" % (
            case, name, present[name]["lines"], d["lines"])
    if m.get("html"):
        with open(os.path.join(outdir, "report.html")) as f:
            got_html = mask_html(f.read())
        ref_html = mask_html(golden_html(case))
        if " -d" in m["args"] and " -I " not in m["args"] and "--in_fq_interleaved" not in m["args"]:
            got_html, ref_html = mask_html_se_dup(got_html), mask_html_se_dup(ref_html)
        if got_html != ref_html:
            k = next(i for i in range(min(len(got_html), len(ref_html)) + 1) if got_html[i:i + 1] != ref_html[i:i + 1])
            raise AssertionError("%s: HTML report differs at %d: ours ...%r... reference ...%r..." % (
                case, k, got_html[max(0, k - 80):k + 80], ref_html[max(0, k - 80):k + 80]))
    if report_text is None:
        with open(os.path.join(outdir, "report.json")) as f:
            report_text = f.read()
    ref = mask_software(golden_json(case))
    got = mask_software(report_text)
    if " -d" in m["args"] and " -I " not in m["args"] and "--in_fq_interleaved" not in m["args"]:
        # SingleEndProcessor zeroes only sizeof(int) * histSize bytes of the size_t histogram
        # (src/seprocessor.cpp:245): its upper half is uninitialised memory -- masked
        ref, got = mask_se_dup(ref), mask_se_dup(got)
    if got != ref:
        a, b = json.loads(got), json.loads(ref)
        for k in sorted(set(a) | set(b)):
            assert a.get(k) == b.get(k), "%s: JSON section %s differs" % (case, k)
        assert got == ref, "%s: JSON text differs (number formatting / key order)" % case


def round16(x):
    return (x + 15) & ~15


def oracle_process(orc):
    def process(p, b, nres, mc):
        res = np.zeros(nres, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS))
        acc = np.zeros(abi.acc_words(p.insert_size_max, mc), np.uint64)
        assert orc.orc_process_batch(ctypes.byref(p), ctypes.byref(b), res.ctypes.data, acc.ctypes.data) == 0
        return res, acc
    return process


class KmerBackend(ctypes.Structure):  # fqh_kmer_backend (include/fqhost.h)
    _fields_ = [("open", ctypes.c_void_p), ("close", ctypes.c_void_p), ("count", ctypes.c_void_p),
                ("find", ctypes.c_void_p)]


def oracle_kmer_backend(orc):
    """The oracle's restatement of the detection k-mer loops as an fqh_kmer_backend."""
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value
    return KmerBackend(addr(orc.orc_kmer_open), addr(orc.orc_kmer_close), addr(orc.orc_kmer_count),
                       addr(orc.orc_kmer_find))


class OracleDup:
    """Duplicate (-d) on the CPU restatement, standing in for the engine's fq_dup table."""

    def __init__(self, orc, keylen):
        self.orc = orc
        self.d = orc.orc_dup_create(keylen)

    def add(self, b, paired):
        self.orc.orc_dup_add_batch(self.d, ctypes.byref(b), int(paired))

    def stat(self, hist_size):
        hist, gcs, tot = np.zeros(hist_size, np.uint64), np.zeros(hist_size, np.uint64), np.zeros(2, np.uint64)
        self.orc.orc_dup_stat(self.d, hist_size, hist.ctypes.data, gcs.ctypes.data, tot.ctypes.data)
        return hist, gcs, tot

    def close(self):
        self.orc.orc_dup_destroy(self.d)


def run_session(host, argv, process, max_n=1500, dup_engine=None):
    """The tool's host pipeline (libfqhost session API) with `process(params, batch, n_results,
    max_cycles) -> (results, accumulator)` standing in for the engine call."""
    enc = [a.encode() for a in argv]
    arr = (ctypes.c_char_p * len(enc))(*enc)
    s = ctypes.c_void_p()
    rc = host.fqh_session_open(len(enc), arr, ctypes.byref(s))
    dup = None
    try:
        assert rc == 0, host.fqh_session_error(s)
        p0 = abi.FqParams()
        host.fqh_session_params(s, 16, ctypes.byref(p0))
        dup_on, keylen, hist_size = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        host.fqh_session_dup_params(s, ctypes.byref(dup_on), ctypes.byref(keylen), ctypes.byref(hist_size))
        if dup_on.value:
            assert dup_engine is not None, "-d needs a duplication engine"
            dup = dup_engine(keylen.value)
        while True:
            b = abi.FqBatch()
            r = host.fqh_session_next(s, max_n, ctypes.byref(b))
            assert r >= 0, host.fqh_session_error(s)
            if r == 0:
                break
            n = b.n
            paired = bool(b.seq2)
            l1 = np.ctypeslib.as_array(ctypes.cast(b.len1, ctypes.POINTER(ctypes.c_uint16)), (n,))
            m1 = int(l1.max()) if n else 0
            m2 = 0
            if paired:
                l2 = np.ctypeslib.as_array(ctypes.cast(b.len2, ctypes.POINTER(ctypes.c_uint16)), (n,))
                m2 = int(l2.max()) if n else 0
            need = m1 + m2 if p0.merge_enabled else max(m1, m2)
            mc = max(16, round16(need))
            p = abi.FqParams()
            host.fqh_session_params(s, mc, ctypes.byref(p))
            if dup is not None:
                dup.add(b, paired)
            res, acc = process(p, b, n * (2 if paired else 1), mc)
            assert host.fqh_session_consume(s, res.ctypes.data, mc) == 0, host.fqh_session_error(s)
            host.fqh_session_add_acc(s, acc.ctypes.data, mc)
        if dup is not None:
            hist, gcs, tot = dup.stat(hist_size.value)
            host.fqh_session_set_dup(s, hist.ctypes.data, gcs.ctypes.data, tot.ctypes.data)
        return abi.take_string(host, host.fqh_session_finish(s))
    finally:
        if dup is not None:
            dup.close()
        host.fqh_session_close(s)


def run_session_with_oracle(host, orc, argv, max_n=1500):
    """Host pipeline with the CPU oracle in the engine's place: checks the host side (parsing,
    packing, formatting, writers, report) on CPU."""
    return run_session(host, argv, oracle_process(orc), max_n, dup_engine=lambda k: OracleDup(orc, k))


def read_row(b, mate, i, length):
    def row(plane):
        return b"".join(ctypes.string_at(plane + abi.batch_offset(b.stride, i, j), min(abi.CHUNK, length - j))
                        for j in range(0, length, abi.CHUNK))

    return row(b.seq1 if mate == 0 else b.seq2), row(b.qual1 if mate == 0 else b.qual2)
