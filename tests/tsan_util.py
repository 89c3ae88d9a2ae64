"""ThreadSanitizer runs of the tool's host pipeline (test infrastructure, CPU only): build/tsan/fqtool
(`make tsan`: the host sources instrumented, oracle/cpu_engine.cpp standing in for the engine) runs a
golden case with host packs (FQ_TEXT_MODE=0), several engines and workers; the outputs must equal the
reference's and stderr must hold no ThreadSanitizer report."""
import os
import subprocess

import e2e_util as E
from fqtool_amd import abi

TSAN_BIN = os.path.join(abi.REPO_DIR, "build", "tsan", "fqtool")


def tsan_available():
    return os.path.exists("/usr/lib/gcc/x86_64-linux-gnu/11/libtsan.so") or os.path.exists(TSAN_BIN)


def build():
    if not os.path.exists(TSAN_BIN):
        subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "tsan"], check=True)


def run_case(case, outdir, workers, devices, inputs=None):
    """Runs one golden case under TSan (inputs: a directory holding replacements of the golden input
    files, e.g. recompressed); returns (stderr text, number of TSan reports)."""
    argv = E.argv_for(TSAN_BIN, case, outdir)
    if inputs:
        argv = [a.replace(E.INPUTS, inputs) for a in argv]
    if not E.is_split(case):  # with -s / -S, -w is the number of file sequences
        argv[2] = str(workers)
    m = E.manifest()[case]
    if " -d" not in m["args"]:  # (duplication tables do not merge across the stand-in's engines)
        argv += ["--devices", ",".join(["0"] * devices), "--pack_pairs", "777"]
    env = dict(os.environ, FQ_TEXT_MODE="0", TSAN_OPTIONS="halt_on_error=0 second_deadlock_stack=1 history_size=4")
    p = subprocess.run(argv, capture_output=True, env=env, cwd=outdir, timeout=600)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 0, err[-3000:]
    E.check_outputs(case, outdir)
    return err, err.count("WARNING: ThreadSanitizer")
