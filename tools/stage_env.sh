set -u
for m in "SCHED_PIN=1" "SCHED_PIN=1 ABLATE_STAGE=1"; do
touch fqtool_amd/csrc/pe_fast.hip
make $m engine > /dev/null 2>&1 || { echo "build failed"; exit 1; }
echo "== $m"
timeout -k 10 200 python tools/stage_env.py 2>&1 | grep synthetic || exit 1
done
touch fqtool_amd/csrc/pe_fast.hip
