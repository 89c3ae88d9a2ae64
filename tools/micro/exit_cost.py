"""Runs tools/micro/exit_cost for a few (pinned MiB, device MiB, chunks) cases; prints the exit time
(the child's last steady-clock stamp to its reaping) and the whole wall, median of 3."""
import os, subprocess, sys, time
exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exit_cost")
cases = [tuple(int(x) for x in c.split()) for c in os.environ["CASES"].split(";")] if os.environ.get("CASES") else \
    [(0, 0, 1, 0), (3000, 0, 1, 0), (3000, 0, 24, 0), (0, 4000, 1, 0), (0, 4000, 40, 0), (3000, 4000, 24, 0)]
for pin, dev, ch, hm in cases:
    ex, wall = [], []
    for _ in range(3):
        t0 = time.monotonic()
        p = subprocess.run([exe, str(pin), str(dev), str(ch), str(hm)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        t1 = time.monotonic()
        if p.returncode:
            print(f"pinned {pin} MiB device {dev} MiB chunks {ch}: rc {p.returncode}")
            break
        ex.append(t1 - float(p.stdout.split()[1]))
        wall.append(t1 - t0)
    if ex:
        print(f"pinned {pin:5d} MiB ({'hipHostMalloc' if hm else 'registered THP'}) device {dev:5d} MiB chunks {ch:3d}: "
              f"exit {sorted(ex)[1]:.3f} s, wall {sorted(wall)[1]:.3f} s, {p.stderr.strip()}", flush=True)
