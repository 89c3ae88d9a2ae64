#!/bin/bash
# tools/micro/unpin_cost for a few cases (';'-separated "MiB chunks busy_ms threads"); each under its own time limit
set -e
cd "$(dirname "$0")"
IFS=';' read -ra cases <<< "${CASES:-3000 24 400 1;3000 24 50 1;1500 12 400 1}"
for c in "${cases[@]}"; do
  python3 - $c <<'PY'
import subprocess, sys, time
a = sys.argv[1:]
t0 = time.monotonic()
p = subprocess.run(["timeout", "-k", "5", "60", "./unpin_cost", *a], stdout=subprocess.PIPE, text=True)
t1 = time.monotonic()
lines = p.stdout.strip().splitlines()
print(f"pinned {a[0]} MiB in {a[1]} chunks, busy {a[2]} ms, {a[3] if len(a) > 3 else 1} threads: {lines[0]}; exit {t1 - float(lines[-1].split()[1]):.3f} s"
      if p.returncode == 0 and lines else f"{a}: rc {p.returncode}", flush=True)
PY
done
