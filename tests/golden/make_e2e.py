#!/usr/bin/env python3
"""Generate end-to-end golden fixtures by running the REFERENCE binary (oracle/_ref/fqtool_ref,
built from /root/reference/src by oracle/Makefile.ref) on fixed inputs.

Inputs under tests/golden/inputs/:
  r1.fq.gz, r2.fq.gz, polygr1.fq, polygr2.fq  -- the reference's own testdata/ files (data)
  synth_r1.fq.gz, synth_r2.fq.gz               -- 3000 pairs from the bench generator (orc_synth_fill)
  edge_r1.fq, edge_r2.fq                       -- ragged/hostile reads (lengths 1..300, IUPAC, lowercase)
  edge64_r1.fq, edge64_r2.fq                   -- the same reads with phred64 qualities
  inter.fq                                     -- first 2000 testdata pairs, interleaved

For every case in CASES: exit status, sha256 + line count of each (decompressed) output and the
JSON report text (gzip) are written under tests/golden/e2e/.  The Software block of the JSON
(command line, cwd) is environment-dependent and is compared with those values masked.

Run from the repo root:  python3 tests/golden/make_e2e.py [case ...]
"""
import ctypes
import gzip
import hashlib
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
INP = os.path.join(HERE, "inputs")
OUT = os.path.join(HERE, "e2e")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "fqtool_ref")
TESTDATA = "/root/reference/testdata"

PE = "-i {in}/%s_r1%s -I {in}/%s_r2%s"

# name -> argument list ({in} = inputs dir, {out} = output dir); outputs are discovered by name
CASES = {
    # BASELINE configs[0]: testdata PE -q -a -g
    "td_pe_qag": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g",
    "td_pe_plain": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq",
    "td_pe_gz": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq.gz -O {out}/o2.fq.gz -q -g -z 6",
    "td_pe_no_O": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -q -a -g",
    "td_se_q": "-i {in}/r1.fq.gz -o {out}/o1.fq -q",
    "td_se_all": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -a -g -x -y -l --min_length 40 --enable_cut_front "
                 "--enable_cut_tail --cut_tail_window 5 --cut_tail_mean_qual 25 -f 2 -t 3 -b 140 "
                 "--failed_out {out}/failed.fq",
    "td_se_adapter": "-i {in}/r1.fq.gz -o {out}/o1.fq -a --adapter_of_read1 AGATCGGAAGAGCACACGTCTGAACTCCAGTCA",
    "td_pe_detect": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a --detect_pe_adapter -g",
    "td_pe_merge": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g --enable_cut_right "
                   "-m --merge_output {out}/merged.fq",
    "td_pe_merge_discard": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g "
                           "-m --discard_unmerged --merge_output {out}/merged.fq",
    "td_pe_all": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -Q 25 -U 0.3 -N 3 -e 28 "
                 "-a -g -x --base_to_trim ACT -y -Y 0.4 -l --min_length 50 --max_length 145 --enable_cut_front "
                 "--enable_cut_tail --enable_cut_right --cut_front_window 3 --cut_front_mean_qual 15 "
                 "--cut_tail_window 6 --cut_tail_mean_qual 22 --cut_right_window 5 --cut_right_mean_qual 18 "
                 "-f 1 -t 2 -F 3 -T 1 -b 147 -B 146 --unpaired_read1 {out}/u1.fq --unpaired_read2 {out}/u2.fq "
                 "--failed_out {out}/failed.fq --min_overlap_len 25 --max_diff_for_overlap 3",
    "td_pe_unpaired_same": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -Q 30 "
                           "--unpaired_read1 {out}/u.fq --unpaired_read2 {out}/u.fq --failed_out {out}/failed.fq",
    "td_pe_failed_only": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -Q 30 -l "
                         "--min_length 120 --failed_out {out}/failed.fq",
    "inter_pe": "-i {in}/inter.fq --in_fq_interleaved -o {out}/o1.fq -q -g -x --unpaired_read1 {out}/u1.fq "
                "--failed_out {out}/failed.fq",
    # -a on an interleaved input forces PE adapter detection on the (empty) read2 file name
    "err_inter_adapter": "-i {in}/inter.fq --in_fq_interleaved -o {out}/o1.fq -q -a",
    "polygr_pe": "-i {in}/polygr1.fq -I {in}/polygr2.fq -o {out}/o1.fq -O {out}/o2.fq -g -x",
    "polygr_se": "-i {in}/polygr1.fq -o {out}/o1.fq -g --min_len_detect_polyG 5 --max_mismatches_polyG 2 "
                 "--one_mismatch_each_polyG 4",
    "synth_pe_c3": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a "
                   "--detect_pe_adapter -g",
    "synth_pe_c4": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g "
                   "--enable_cut_right -m --merge_output {out}/merged.fq",
    "synth_pe_c5": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g -x "
                   "--enable_cut_right",
    "synth_se_c2": "-i {in}/synth_r1.fq.gz -o {out}/o1.fq -q",
    "edge_pe_all": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -q -a -g -x -y -l "
                   "--enable_cut_front --enable_cut_tail --enable_cut_right --unpaired_read1 {out}/u1.fq "
                   "--unpaired_read2 {out}/u2.fq --failed_out {out}/failed.fq",
    "edge_pe_merge": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -q -a -g -m "
                     "--merge_output {out}/merged.fq",
    # -m with the low-complexity filter (merged reads), -c with front trimming, -c + UMI + -m
    "td_pe_merge_complexity": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g -y -Y 0.45 "
                              "-m --merge_output {out}/merged.fq",
    "edge_pe_merge_complexity": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -y -Y 0.3 -m "
                                "--merge_output {out}/merged.fq",
    "td_se_correct": "-i {in}/r1.fq.gz -o {out}/o1.fq -c -q -g",
    "edge_pe_correct_front": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -c -q -a -f 3 -F 2 "
                             "--enable_cut_front --cut_front_window 5 --cut_front_mean_qual 22",
    "synth_pe_correct_umi_merge": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -c -q -a "
                                  "-g -u --umi_location 6 --umi_length 6 -m --merge_output {out}/merged.fq",
    "edge_se_all": "-i {in}/edge_r1.fq -o {out}/o1.fq -q -a -g -x -y -l --enable_cut_front --enable_cut_tail "
                   "--failed_out {out}/failed.fq",
    "edge64_pe": "-i {in}/edge64_r1.fq -I {in}/edge64_r2.fq --phred64 -o {out}/o1.fq -O {out}/o2.fq -q -a -g",
    # base correction (-c), alone, with adapters/merge, on hostile reads
    "td_pe_correct": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -c -q -a -g "
                     "--failed_out {out}/failed.fq",
    "td_pe_correct_only": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -c",
    "synth_pe_correct_merge": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -c -q -a "
                              "-g -m --merge_output {out}/merged.fq",
    "edge_pe_correct": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -c -q -a -g -x "
                       "--adapter_of_read1 AGATCGGAAGAGCACACGTCTGAACTCCAGTCA --unpaired_read1 {out}/u1.fq "
                       "--unpaired_read2 {out}/u2.fq --failed_out {out}/failed.fq",
    # UMI: every location, trim / no trim, comment dropping, SE
    "td_pe_umi_idx1": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -u --umi_location 1",
    "td_pe_umi_idx2": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -u --umi_location 2 "
                      "--umi_drop_comment",
    "td_pe_umi_r1": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g -u --umi_location 3 "
                    "--umi_length 8 --umi_skip_length 2 --failed_out {out}/failed.fq",
    "td_pe_umi_r2_notrim": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -u --umi_location 4 "
                           "--umi_length 5 --umi_not_trim",
    "td_pe_umi_perindex": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -u --umi_location 5",
    "td_pe_umi_perread": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -g -u --umi_location 6 "
                         "--umi_length 6 --umi_skip_length 1 --umi_drop_comment -m --merge_output {out}/merged.fq",
    "edge_pe_umi_perread": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -q -a -g "
                           "--enable_cut_front -u --umi_location 6 --umi_length 12 --umi_skip_length 3 "
                           "--unpaired_read1 {out}/u1.fq --failed_out {out}/failed.fq",
    "td_se_umi_r1": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -u --umi_location 3 --umi_length 7 --failed_out {out}/failed.fq",
    "td_se_umi_perindex": "-i {in}/r1.fq.gz -o {out}/o1.fq -u --umi_location 5",
    "edge_se_umi_r2": "-i {in}/edge_r1.fq -o {out}/o1.fq -q -u --umi_location 4 --umi_length 4",
    # index filter
    "td_pe_index": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g --enable_index_filter "
                   "--index1_file {in}/idx_a.txt --index2_file {in}/idx_b.txt --failed_out {out}/failed.fq",
    "td_pe_index_diff1": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q --enable_index_filter "
                         "--index1_file {in}/idx_c.txt --max_diff_for_match 1 -u --umi_location 1",
    "td_se_index": "-i {in}/r1.fq.gz -o {out}/o1.fq -q --enable_index_filter --index1_file {in}/idx_a.txt",
    "synth_pe_index_all": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q "
                          "--enable_index_filter --index2_file {in}/idx_empty_line.txt",
    "td_pe_index_nofile": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q --enable_index_filter",
    # duplication analysis (-d)
    "td_pe_dup": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -d -q -a -g",
    "td_pe_dup_key13": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -d --dup_ana_key_len 13 "
                       "--dup_ana_hist_size 8 -q",
    "td_pe_dup_hist2": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -d --dup_ana_hist_size 2 "
                       "--enable_index_filter --index1_file {in}/idx_a.txt",
    "td_se_dup": "-i {in}/r1.fq.gz -o {out}/o1.fq -d -q",
    "inter_pe_dup": "-i {in}/inter.fq --in_fq_interleaved -o {out}/o1.fq -d --dup_ana_hist_size 5",
    "edge_pe_dup": "-i {in}/edge_r1.fq -I {in}/edge_r2.fq -o {out}/o1.fq -O {out}/o2.fq -d -q -a -g",
    "synth_pe_dup": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -d -q -a -g -x "
                    "--enable_cut_right",
    # split output (-s by file number from the evaluator's read-count estimate, -S by passed reads)
    "td_pe_split_num": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g -s "
                       "--split_file_number 3 --max_item_in_pack 3000",
    "td_pe_split_num_gz": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq.gz -O {out}/o2.fq.gz -q -s "
                          "--split_file_number 4 --max_item_in_pack 1000 --failed_out {out}/failed.fq",
    "td_se_split_num_many": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -s --split_file_number 9 --max_item_in_pack 4000",
    "td_se_split_lines": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -S --splie_file_line 2000 --max_item_in_pack 1500",
    "synth_pe_split_lines": "-i {in}/synth_r1.fq.gz -I {in}/synth_r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -q -a -g "
                            "-S --splie_file_line 500 --max_item_in_pack 400 --digits_file_name 2",
    "err_index_bad": "-i {in}/r1.fq.gz -o {out}/o1.fq --enable_index_filter --index1_file {in}/idx_bad.txt",
    "err_umi_len0": "-i {in}/r1.fq.gz -o {out}/o1.fq -u --umi_location 3",
    # validation / CLI failures: exit status only (messages are compared for validate errors)
    "err_merge_no_out": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -O {out}/o2.fq -m",
    "err_polyx_chars": "-i {in}/r1.fq.gz -o {out}/o1.fq -x --base_to_trim ACGU",
    "err_missing_o": "-i {in}/r1.fq.gz -q",
    "err_needs": "-i {in}/r1.fq.gz -o {out}/o1.fq -Q 20",
    "err_range": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -Q 61",
    "err_no_file": "-i {in}/nonexistent.fq -o {out}/o1.fq",
    "err_extras": "-i {in}/r1.fq.gz -o {out}/o1.fq -qZ a b",
    "err_extra_long": "-i {in}/r1.fq.gz -o {out}/o1.fq --bogus",
    "err_not_int": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -Q abc",
    "err_conversion": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -e abc",
    "err_excludes": "-i {in}/r1.fq.gz -I {in}/r2.fq.gz -o {out}/o1.fq -s -m",
    "err_requires_I": "-i {in}/r1.fq.gz -o {out}/o1.fq -O {out}/o2.fq",
    "err_size_range": "-i {in}/r1.fq.gz -o {out}/o1.fq --max_item_in_pack -5",
    "err_missing_value": "-i {in}/r1.fq.gz -o {out}/o1.fq -q -w 1 -Q",
}

def make_inputs():
    os.makedirs(INP, exist_ok=True)
    for f in ("r1.fq.gz", "r2.fq.gz", "polygr1.fq", "polygr2.fq"):
        shutil.copyfile(os.path.join(TESTDATA, f), os.path.join(INP, f))
    # synthetic pairs from the bench generator
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    import oracle_lib
    from batch_util import synth_pack
    orc = oracle_lib.load_oracle()
    n = 3000
    pk = synth_pack(orc, n, True, seed=777, first=0, L=150, stride=160)
    for m in (1, 2):
        s, q, ln = getattr(pk, "seq%d" % m), getattr(pk, "qual%d" % m), getattr(pk, "len%d" % m)
        with gzip.GzipFile(os.path.join(INP, "synth_r%d.fq.gz" % m), "wb", compresslevel=6, mtime=0) as f:
            for i in range(n):
                L = int(ln[i])
                f.write(b"@SYN:7:FC1:%d %d:N:0:ACGTAC\n" % (i, m) + bytes(s[i, :L]) + b"\n+\n" +
                        bytes(q[i, :L]) + b"\n")
    # ragged / hostile reads
    rng = random.Random(4242)
    ad = {1: b"AGATCGGAAGAGCACACGTCTGAACTCCAGTCA", 2: b"AGATCGGAAGAGCGTCGTGTAGGGAAAGAGTGT"}
    recs = {1: [], 2: []}
    for i in range(800):
        for m in (1, 2):
            L = rng.choice([1, 2, 5, 9, 10, 11, 14, 15, 16, 30, 31, 50, 51, 75, 100, 149, 150, 151, 160, 161,
                            200, 250, 300])
            alpha = b"ACGT" if rng.random() < 0.6 else (b"ACGTN" if rng.random() < 0.7 else b"ACGTNacgtnRYKM.")
            seq = bytearray(rng.choice(alpha) for _ in range(L))
            kind = rng.random()
            if kind < 0.15 and L > 12:
                g = rng.randint(5, L)
                seq[L - g:] = (b"G" if rng.random() < 0.7 else bytes([rng.choice(b"ACT")])) * g
            elif kind < 0.35 and L > 30:
                k = rng.randint(0, L - 1)
                a = ad[m][: L - k]
                seq[k:k + len(a)] = a
            elif kind < 0.4:
                seq = bytearray(b"N" * L)
            qual = bytearray(33 + (rng.randint(2, 40) if rng.random() > 0.15 else rng.randint(0, 12))
                             for _ in range(L))
            name = b"@EDGE:%d %d:N:0" % (i, m) if rng.random() < 0.8 else b"@EDGE_%d/%d" % (i, m)
            recs[m].append((name, bytes(seq), bytes(qual)))
    for m in (1, 2):
        with open(os.path.join(INP, "edge_r%d.fq" % m), "wb") as f:
            for name, s, q in recs[m]:
                f.write(name + b"\n" + s + b"\n+\n" + q + b"\n")
        with open(os.path.join(INP, "edge64_r%d.fq" % m), "wb") as f:
            for name, s, q in recs[m]:
                f.write(name + b"\n" + s + b"\n+\n" + bytes(c + 31 for c in q) + b"\n")
    # index-filter blacklists (Options::makeListFromFileByLine input)
    for name, text in (("idx_a.txt", b"TAGGTCC\nTAGTTCA\n"), ("idx_b.txt", b"TAGTTAC\n"), ("idx_c.txt", b"TAGGTCA\n"),
                       ("idx_empty_line.txt", b"ACGTAC\n\n"), ("idx_bad.txt", b"ACGT\nacgt\n")):
        with open(os.path.join(INP, name), "wb") as f:
            f.write(text)
    # interleaved
    with gzip.open(os.path.join(INP, "r1.fq.gz")) as f1, gzip.open(os.path.join(INP, "r2.fq.gz")) as f2:
        l1, l2 = f1.read().split(b"\n"), f2.read().split(b"\n")
    with open(os.path.join(INP, "inter.fq"), "wb") as f:
        for i in range(2000):
            f.write(b"\n".join(l1[4 * i:4 * i + 4]) + b"\n" + b"\n".join(l2[4 * i:4 * i + 4]) + b"\n")


def digest(path):
    data = open(path, "rb").read()
    if path.endswith(".gz"):
        data = gzip.decompress(data) if data else b""
    return {"sha256": hashlib.sha256(data).hexdigest(), "lines": data.count(b"\n")}


def run_case(binary, name, args, workdir, extra=()):
    out = os.path.join(workdir, name)
    os.makedirs(out, exist_ok=True)
    argv = [binary, "-w", "1", "-J", os.path.join(out, "report.json"), "-H", os.path.join(out, "report.html")]
    argv += list(extra) + args.format(**{"in": INP, "out": out}).split()
    p = subprocess.run(argv, cwd=out, capture_output=True, timeout=600)
    res = {"args": args, "exit": p.returncode, "outputs": {}}
    for o in sorted(os.listdir(out)):  # every output file but the reports
        if not o.startswith("report."):
            res["outputs"][o] = digest(os.path.join(out, o))
    js = os.path.join(out, "report.json")
    res["json"] = open(js).read() if os.path.exists(js) and p.returncode == 0 else None
    hf = os.path.join(out, "report.html")
    res["html"] = open(hf).read() if os.path.exists(hf) and p.returncode == 0 else None
    # error text of a failed run (CLI11 message or util::errorExit line), with paths relative
    res["stderr"] = p.stderr.decode(errors="replace").replace(INP, "{in}").replace(out, "{out}") \
        if p.returncode != 0 else None
    return res


def main():
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -f oracle/Makefile.ref")
    make_inputs()
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]  # case names: regenerate just these, keeping the other fixtures as they are
    manifest = {}
    if only:
        with open(os.path.join(OUT, "manifest.json")) as f:
            manifest = json.load(f)
    with tempfile.TemporaryDirectory() as tmp:
        for name, args in CASES.items():
            if only and name not in only:
                continue
            r = run_case(REF_BIN, name, args, tmp)
            if r["json"] is not None:
                with gzip.GzipFile(os.path.join(OUT, name + ".json.gz"), "wb", compresslevel=9, mtime=0) as f:
                    f.write(r["json"].encode())
            r["json"] = (name + ".json.gz") if r["json"] is not None else None
            if r["html"] is not None:
                with gzip.GzipFile(os.path.join(OUT, name + ".html.gz"), "wb", compresslevel=9, mtime=0) as f:
                    f.write(r["html"].encode())
            r["html"] = (name + ".html.gz") if r["html"] is not None else None
            manifest[name] = r
            print(name, r["exit"], sorted(r["outputs"]), file=sys.stderr)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
