# Round-4 C5 evidence (one MI355X): Humanoid bench lines, the layered rollout step's SQ
# issue floor (tools/step_issue.py), PMC traffic of the largest policy GEMM.
# Usage (on the box): bash tools/r04_b.sh TAG  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04b}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_humanoid.py tests/test_gpu_iteration.py tests/test_gpu_layered.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  cat gpurun_out/${tag}_bench_${n}.json
}
run humanoid_bf16 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for dt in bf16 fp32; do
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/${tag}_sq_hm_$dt -o run -- python3 tools/humanoid_collect.py 1024 32 $dt > gpurun_out/${tag}_sq_hm_$dt.log 2>&1 || { echo SQ_FAILED $dt; tail -5 gpurun_out/${tag}_sq_hm_$dt.log; exit 1; }
python tools/step_issue.py gpurun_out/${tag}_sq_hm_$dt Humanoid-v2/$dt --out gpurun_out/${tag}_rollout_issue.json > /dev/null || exit 1
done
L=gemm:bf16:NN_dual_dtanh:1048576x512x512
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_gemm_fetch -o run -- python3 tools/gemm_pmc_probe.py $L 5 > gpurun_out/${tag}_gemm_f.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/${tag}_gemm_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_gemm_write -o run -- python3 tools/gemm_pmc_probe.py $L 5 > gpurun_out/${tag}_gemm_w.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/${tag}_gemm_w.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${tag}_gemm_fetch gpurun_out/${tag}_gemm_write --gemm $L --key Humanoid-v2/bf16/1024 --out gpurun_out/${tag}_pmc_gemm.json || exit 1
cat gpurun_out/${tag}_rollout_issue.json | head -30
run humanoid 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1
# A/B: the VF fit after the rollout (the default co-schedules it on shared CUs)
export MRL_COSCHED_FIT=0; run humanoid_bf16_serial_fit 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16 --no-cpu-baseline
unset MRL_COSCHED_FIT
echo R04_B_OK
