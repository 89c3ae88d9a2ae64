#!/bin/bash
# Runs one gpurun command, retrying only while no GPU box is free (gpurun's transient status: nothing
# ran, nothing charged), at most TRIES times, SLEEP seconds apart.  Any real outcome -- success or a
# failure of the command itself -- ends it.  Output: gpurun_out/when_free.log
#   tools/gpurun_when_free.sh <timeout-seconds> '<command>'
set -u
to=$1; shift
cmd=$1
log=gpurun_out/when_free.log
mkdir -p gpurun_out
for i in $(seq 1 ${TRIES:-40}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "GPU-minutes left this round: 0" "$log"; then
    sleep ${SLEEP:-60}
    continue
  fi
  echo "attempt $i rc=$rc" >> "$log"
  exit $rc
done
echo "gave up after $i attempts" >> "$log"
exit 3
