"""ThreadSanitizer runs of the tool's host pipeline (test infrastructure, CPU only): build/tsan/fqtool
(`make tsan`: the host sources instrumented, oracle/cpu_engine.cpp standing in for the engine) runs a
golden case in one of the tool's three pipelines -- host packs (FQ_TEXT_MODE=0), text packs, or the
raw stream (plain inputs: the window reader, one thread per engine, RawMulti's ordered hand-offs) --
on several engines and workers; the outputs must equal the reference's and stderr must hold no
ThreadSanitizer report."""
import os
import subprocess

import e2e_util as E
from fqtool_amd import abi

TSAN_BIN = os.path.join(abi.REPO_DIR, "build", "tsan", "fqtool")


def tsan_available():
    """The TSan runtime of the host compiler (the one `make tsan` links), wherever it lives."""
    if os.path.exists(TSAN_BIN):
        return True
    cxx = os.environ.get("CXX", "g++")
    try:
        lib = subprocess.run([cxx, "-print-file-name=libtsan.so"], capture_output=True, text=True, timeout=60).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return False
    return os.path.isabs(lib) and os.path.exists(lib)  # (an unknown name comes back bare)


def build():
    subprocess.run(["make", "-s", "-C", abi.REPO_DIR, "tsan"], check=True)  # (incremental: a stale build is remade)


def run_case(case, outdir, workers, devices, inputs=None, mode="host", env_extra=None, pack_pairs=777):
    """Runs one golden case under TSan (inputs: a directory holding replacements of the golden input
    files, e.g. recompressed; mode: "host" packs, "text" packs, or the "raw" stream, for which the
    gzip inputs are decompressed to plain files); returns (stderr text, number of TSan reports)."""
    argv = E.argv_for(TSAN_BIN, case, outdir)
    if inputs:
        argv = [a.replace(E.INPUTS, inputs) for a in argv]
    if mode == "raw":
        import gzip
        import shutil
        ind = os.path.normpath(outdir) + "_plain_in"  # (beside the outputs, which are checked file by file)
        os.makedirs(ind, exist_ok=True)
        for k, a in enumerate(argv):
            if a.endswith(".fq.gz") and os.path.exists(a):
                plain = os.path.join(ind, os.path.basename(a)[:-3])
                with gzip.open(a, "rb") as f, open(plain, "wb") as g:
                    shutil.copyfileobj(f, g)
                argv[k] = plain
    if not E.is_split(case):  # with -s / -S, -w is the number of file sequences
        argv[2] = str(workers)
    m = E.manifest()[case]
    if " -d" not in m["args"]:  # (duplication tables do not merge across the stand-in's engines)
        argv += ["--devices", ",".join(["0"] * devices), "--pack_pairs", str(pack_pairs)]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 second_deadlock_stack=1 history_size=4")
    if mode == "host":
        env["FQ_TEXT_MODE"] = "0"
    elif mode == "text":
        env["FQ_RAW_MODE"] = "0"
    env.update(env_extra or {})
    try:
        p = subprocess.run(argv, capture_output=True, env=env, cwd=outdir, timeout=600)
    finally:
        if mode == "raw":
            import shutil
            shutil.rmtree(os.path.normpath(outdir) + "_plain_in", ignore_errors=True)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 0, err[-3000:]
    E.check_outputs(case, outdir)
    return err, err.count("WARNING: ThreadSanitizer")
