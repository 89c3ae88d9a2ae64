# profiling aid: per-variant dynamic instruction counts of the fast PE kernel (valu_probe.py's ablation
# variants, one launch each), per tile of 32 pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${CONFIG:-C3}
CNT=${COUNTERS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES}
timeout -s KILL 300 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/vprobe_$C -o pmc -- python tools/valu_probe.py > gpurun_out/vprobe_$C.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections, os
C = os.environ.get('CONFIG', 'C3')
rows = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for path in glob.glob(f"gpurun_out/vprobe_{C}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"]); names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
variants = [l.split()[0] for l in open(f"gpurun_out/vprobe_{C}.log") if l.strip() and l.split()[0].islower() and len(l.split()) == 2]
ms = {l.split()[0]: float(l.split()[1]) for l in open(f"gpurun_out/vprobe_{C}.log") if l.strip() and l.split()[0].islower() and len(l.split()) == 2}
fast = [d for d in sorted(rows) if "pe_fast" in names[d]]
tiles = int(os.environ.get("PAIRS", 20_000_000)) / 32
for v, d in zip(variants, fast):
    c = rows[d]
    print(f"{v:12s} ms {ms[v]:7.3f} " + " ".join(f"{k.replace('SQ_','')}/tile {c[k]/tiles:8.1f}" for k in sorted(c) if k != 'SQ_WAVES'))
PY
