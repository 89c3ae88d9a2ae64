#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-pytest smoke bench prof}"
run() {
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc" >> "gpurun_out/$name.log"
    echo "$name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    return $rc
}
for s in $STEPS; do
    case $s in
    pytest)
        run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread; rc=$?
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)
        run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
        run bench 900 python bench.py ${BENCH_ARGS:-} || exit $? ;;
    prof)
        run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
