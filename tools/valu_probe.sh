# profiling aid: per-variant dynamic instruction counts of the fast PE kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/vprobe_${CONFIG:-C3} -o pmc -- python tools/valu_probe.py > gpurun_out/vprobe_${CONFIG:-C3}.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections, os
rows = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for path in glob.glob(f"gpurun_out/vprobe_{os.environ.get('CONFIG','C3')}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"]); names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
variants = [l.split()[0] for l in open(f"gpurun_out/vprobe_{os.environ.get('CONFIG','C3')}.log") if l.strip() and l.split()[0].islower() and len(l.split()) == 2]
fast = [d for d in sorted(rows) if "pe_fast" in names[d]]
tiles = 20_000_000 / 32
for v, d in zip(variants, fast):
    c = rows[d]
    print(f"{v:14s} VALU/tile {c['SQ_INSTS_VALU']/tiles:8.0f}  SALU/tile {c['SQ_INSTS_SALU']/tiles:7.0f}  LDS/tile {c['SQ_INSTS_LDS']/tiles:6.0f}")
PY
