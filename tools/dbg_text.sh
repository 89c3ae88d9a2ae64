set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/dbg; D=gpurun_out/dbg
T=tests/golden/inputs
./fqtool_amd/bin/fqtool -i $T/r1.fq.gz -I $T/r2.fq.gz -o $D/a1.fq -O $D/a2.fq -J $D/a.json -H $D/a.html > $D/a.log 2>&1
FQ_TEXT_MODE=0 ./fqtool_amd/bin/fqtool -i $T/r1.fq.gz -I $T/r2.fq.gz -o $D/b1.fq -O $D/b2.fq -J $D/b.json -H $D/b.html > $D/b.log 2>&1
wc -l $D/a1.fq $D/b1.fq $D/a2.fq $D/b2.fq; cmp $D/a1.fq $D/b1.fq | head; cmp $D/a2.fq $D/b2.fq | head; tail -2 $D/a.log
ls -l $D/a1.fq $D/b1.fq; tail -c 40 $D/a1.fq | od -c | tail -4; tail -c 40 $D/b1.fq | od -c | tail -4
