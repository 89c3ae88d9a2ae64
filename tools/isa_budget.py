#!/usr/bin/env python3
"""Profiling aid: static, cycle-weighted instruction budget of one fast-kernel instantiation, per phase.

    hipcc -std=c++17 -O3 --offload-arch=gfx950 --offload-device-only -S -gline-tables-only \
          -Iinclude fqtool_amd/csrc/pe_fast.hip -o /tmp/pe_fast_g.s
    python tools/isa_budget.py /tmp/pe_fast_g.s 'pe_fast_kernelILb1ELb1ELb0ELb0ELb1E' [--costs profiles/r04_micro_opcost2.txt]

Every instruction of the kernel is attributed to a phase through its `.loc` line: kernel-body lines by
the section they lie in (staging, trimAndCut, polyG, overlap, ...), lines of a phase-specific helper
(ov_candidates, polyg_bits, ...) to that phase, and lines of shared helpers (xor32, field_window,
device_ops.h, the HIP headers) to the phase of the last kernel-body line seen before them.  Each
instruction is priced with the measured per-opcode issue cost (SIMD cycles per wave64 instruction,
4 waves per SIMD: tools/micro/gen_opcost2.py), keyed by opcode and operand kind.  Instructions inside
a loop (a block between a back-edge target and its branch) are reported separately: their dynamic
count is the static count times the trip count, which this static view does not know.
"""
import re
import sys
from collections import defaultdict

# (ISA_SRC: another copy of the source the assembly was built from, e.g. an older revision)
SRC_PATH = __import__("os").environ.get("ISA_SRC") or __import__("os").path.join(
    __import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", "fqtool_amd", "csrc", "pe_fast.hip")
SRC = __import__("os").path.basename(SRC_PATH)
# kernel-body sections: the "// ---------------- <name>" marker comments of pe_fast.hip
MARKERS = [("staging", "staging"), ("trimAndCut", "trim"), ("polyG", "polyG"), ("overlap", "overlap"),
           ("polyX", "polyx_maxlen"), ("merge", "merge"), ("passFilter", "filter"), ("Stats::statRead", "stats"),
           ("flush", "flush")]
# phase-specific helpers of pe_fast.hip (function name -> phase)
HELPER_FUNCS = {"ov_exact": "overlap", "ov_scan": "overlap", "unzip2": "overlap", "csa": "overlap",
                "ov_candidates": "overlap", "adseq_search": "adseq", "polyg_bits": "polyG",
                "polyx_no_trim": "polyx_maxlen", "cut_right_w4": "trim", "lower_flags": "staging",
                "correct_pair_fast": "correct", "count_by_value": "filter"}


def _scan_source():
    import re as _re
    lines = open(SRC_PATH).read().split("\n")
    secs, helpers = [], []
    kstart = next(i for i, l in enumerate(lines) if "pe_fast_kernel(fq_params p" in l) + 1
    secs.append((kstart, "setup"))
    for i, l in enumerate(lines, 1):
        m = _re.match(r"\s*// ---------------- (\S+)", l)
        if m and i > kstart:
            for key, nm in MARKERS:
                if m.group(1).startswith(key):
                    secs.append((i, nm))
        m = _re.match(r"__device__.*?\b(\w+)\(", l)
        if m and m.group(1) in HELPER_FUNCS:
            end = next(j for j in range(i, len(lines)) if lines[j].startswith("}"))
            helpers.append((i, end + 1, HELPER_FUNCS[m.group(1)]))
    kend = next(j for j in range(kstart, len(lines)) if lines[j].startswith("}")) + 1
    secs.append((kend + 1, None))
    return secs, helpers, kstart, kend


SECTIONS, HELPERS, KSTART, KEND = _scan_source()


def section_of(line):
    name = None
    for start, nm in SECTIONS:
        if line >= start:
            name = nm
    return name


def helper_of(line):
    for a, b, nm in HELPERS:
        if a <= line <= b:
            return nm
    return None


def load_costs(path):
    """name -> cycles from an opcost2 result file (lines 'name   X.XX SIMD cycles ...')."""
    costs = {}
    if not path:
        return costs
    for ln in open(path):
        m = re.match(r"(.+?)\s+([\d.]+) SIMD cycles", ln)
        if m:
            costs[m.group(1).strip()] = float(m.group(2))
    return costs


FAST_DEFAULT = {"v_xor_b32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_add_u32_e32", "v_sub_u32_e32",
                "v_subrev_u32_e32", "v_lshrrev_b32_e32", "v_mov_b32_e32", "v_not_b32_e32", "v_lshlrev_b16_e32"}


def price(op, args, costs):
    """issue cycles of one instruction (SIMD cycles per wave-instruction, 4 waves per SIMD)."""
    sgpr = bool(re.search(r"(^|[\s,\[])s\d|(^|[\s,])(vcc|exec|m0)\b", args.split(";")[0]))
    if op.startswith("s_nop"):
        return 0.0, "salu"
    if op.startswith("s_"):
        return 0.0, "salu"
    if op.startswith(("ds_", "global_", "buffer_", "scratch_", "flat_")):
        return 0.0, "mem"
    if not op.startswith("v_"):
        return 0.0, "other"
    if costs:
        for key in (f"{op} vv", f"{op} vvv", f"{op} inline", f"{op} vv+inline", op):
            if key in costs and not (sgpr and key.endswith(("vv", "vvv"))):
                return costs[key], "valu"
        base = op.replace("_e64", "_e32")
        if sgpr and f"{op} sgpr" in costs:
            return costs[f"{op} sgpr"], "valu"
    if op in FAST_DEFAULT and not sgpr:
        return 2.4, "valu"
    if op in ("v_cndmask_b32_e32",):
        return 4.5, "valu"
    return 4.5, "valu"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    cost_path = sys.argv[sys.argv.index("--costs") + 1] if "--costs" in sys.argv else None
    costs = load_costs(cost_path)
    lines = open(path).read().split("\n")
    files = {}
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", ln)
        if m:
            files[int(m.group(1))] = m.group(2).split("/")[-1]
        if start is None and ln.startswith("_Z") and sym in ln and ln.rstrip().endswith(":") is False and ":" in ln:
            start = i
    if start is None:
        sys.exit(f"kernel {sym} not found")
    # instructions and labels of the function
    body = []
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        body.append(ln)
    # pass 1: label positions, for loop detection (a backward branch target .. branch)
    label_at = {}
    insts = []  # (index, op, args, file, line)
    cur_file, cur_line = None, 0
    for ln in body:
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur_file, cur_line = files.get(int(m.group(1)), "?"), int(m.group(2))
            continue
        m = re.match(r"(\.LBB\d+_\d+):", s)
        if m:
            label_at[m.group(1)] = len(insts)
            continue
        if not s or s.startswith((".", ";")):
            continue
        parts = s.split(None, 1)
        op = parts[0]
        args = parts[1] if len(parts) > 1 else ""
        insts.append((op, args, cur_file, cur_line))
    in_loop = [False] * len(insts)
    for i, (op, args, _, _) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = args.split()[0]
            j = label_at.get(tgt)
            if j is not None and j <= i:
                for k in range(j, i + 1):
                    in_loop[k] = True
    # attribution
    phase_of = []
    last_phase = "setup"
    for op, args, f, line in insts:
        ph = None
        if f == SRC:
            ph = helper_of(line)
            if ph is None:
                sec = section_of(line)
                if sec is not None and KSTART <= line <= KEND:
                    ph = sec
                    last_phase = sec
        if ph is None:
            ph = last_phase
        phase_of.append(ph)
    # tally
    tab = defaultdict(lambda: defaultdict(float))
    ops_by_phase = defaultdict(lambda: defaultdict(int))
    order = []
    for (op, args, f, line), ph, lp in zip(insts, phase_of, in_loop):
        if ph not in order:
            order.append(ph)
        cyc, cls = price(op, args, costs)
        key = "loop" if lp else "line"
        tab[ph][f"{cls}_{key}"] += 1
        tab[ph][f"cyc_{key}"] += cyc
        if op == "s_nop":
            m = re.match(r"(\d+)", args)
            tab[ph][f"nop_{key}"] += 1 + int(m.group(1)) if m else 1
        if op.startswith("ds_add"):
            tab[ph][f"ldsatomic_{key}"] += 1
        if cls == "valu":
            ops_by_phase[ph][op] += 1
    hdr = f"{'phase':22s} {'VALU':>6s} {'cyc':>8s} {'c/VALU':>6s} {'SALU':>5s} {'mem':>5s} {'nopcyc':>6s} | {'VALU@loop':>9s} {'cyc@loop':>8s}"
    print(hdr)
    tot = defaultdict(float)
    for ph in order:
        t = tab[ph]
        v, c = t["valu_line"], t["cyc_line"]
        print(f"{ph:22s} {v:6.0f} {c:8.0f} {c / v if v else 0:6.2f} {t['salu_line']:5.0f} {t['mem_line']:5.0f} "
              f"{t['nop_line']:6.0f} | {t['valu_loop']:9.0f} {t['cyc_loop']:8.0f}")
        for k, x in t.items():
            tot[k] += x
    print(f"{'total':22s} {tot['valu_line']:6.0f} {tot['cyc_line']:8.0f} {tot['cyc_line'] / max(tot['valu_line'], 1):6.2f} "
          f"{tot['salu_line']:5.0f} {tot['mem_line']:5.0f} {tot['nop_line']:6.0f} | {tot['valu_loop']:9.0f} {tot['cyc_loop']:8.0f}")
    if "--ops" in sys.argv:
        for ph in order:
            top = sorted(ops_by_phase[ph].items(), key=lambda kv: -kv[1])[:14]
            print(f"\n{ph}: " + ", ".join(f"{o} {n}" for o, n in top))


if __name__ == "__main__":
    main()
