# split Fisher product diagnosis + SQ counters; PPO golden GPU tests (one MI355X)
set -o pipefail
tag=${1:-r04d}
cd $GRAFT_REPO_ROOT
export MRL_FISHER=split MRL_VJP_SPLIT=1
timeout -k 10 200 python tools/split_diag.py > gpurun_out/${tag}_diag.log 2>&1 || { echo DIAG_FAILED; tail -20 gpurun_out/${tag}_diag.log; exit 1; }
cat gpurun_out/${tag}_diag.log
unset MRL_FISHER MRL_VJP_SPLIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ppo.py tests/test_gpu_rccl.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export MRL_FISHER=split MRL_VJP_SPLIT=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${tag}_sq -o run -- python3 tools/split_probe.py > gpurun_out/${tag}_sq.log 2>&1 || { echo SQ_FAILED; tail -5 gpurun_out/${tag}_sq.log; exit 1; }
python tools/sq_split.py gpurun_out/${tag}_sq split_kernel mlp_rows_kernel mlp_vjp16 > gpurun_out/${tag}_sq.txt
cat gpurun_out/${tag}_sq.txt
echo R04_D_OK
