# split-operand Fisher product: GPU tests + probe (one MI355X)
set -o pipefail
tag=${1:-r04c}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/${tag}_probe.log; exit 1; }
cat gpurun_out/${tag}_probe.log
echo R04_C_OK
