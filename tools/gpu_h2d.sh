#!/bin/bash
# H2D paths for FASTQ bytes (tools/micro/h2d.hip) on a 3.5 GB synthetic file in the page cache
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
python3 - <<'PY'
import os
blk = (b"@SYN:1:1101:12345:0000001 1:N:0:ACGTACGT\n" + b"ACGT" * 37 + b"AC\n+\n" + b"F" * 150 + b"\n") * 65536
with open("/tmp/h2d.fq", "wb") as f:
    for _ in range(3500 * 1000 * 1000 // len(blk)):
        f.write(blk)
PY
timeout -k 10 120 ./tools/micro/h2d /tmp/h2d.fq 256 8 > gpurun_out/h2d.txt 2>&1
timeout -k 10 120 ./tools/micro/h2d /tmp/h2d.fq 64 16 >> gpurun_out/h2d.txt 2>&1
rm -f /tmp/h2d.fq
