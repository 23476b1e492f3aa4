# run-to-run determinism of the Fisher-product row kernels, default build and the
# explicit-wait-state diagnostic build (tools/build_ablate.sh nops -DMRL_SPLIT_NOPS=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python tools/determinism_probe.py > gpurun_out/det.log 2>&1 || { tail -5 gpurun_out/det.log; exit 1; }
cat gpurun_out/det.log
MRL_LIB_PATH=tools/ablate/libmrl_hip_nops.so timeout -k 10 240 python tools/determinism_probe.py > gpurun_out/det_nops.log 2>&1 || { tail -5 gpurun_out/det_nops.log; exit 1; }
cat gpurun_out/det_nops.log
