# PC sampling of the fast kernel (one ablation-free launch per VARIANTS entry of valu_probe.py)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
CONFIG=${CONFIG:-C3} VARIANTS=full timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCM:-host_trap} --pc-sampling-unit ${PCU:-time} --pc-sampling-interval ${PCI:-1} --output-format csv -d gpurun_out/pcs -o pcs -- python tools/valu_probe.py > gpurun_out/pcs.log 2>&1
rc=$?; tail -5 gpurun_out/pcs.log; ls -R gpurun_out/pcs | head; exit $rc
