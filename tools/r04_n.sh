# Tiled TN GEMM with four register stages in flight (one MI355X): bit-identity tests,
# a timing probe of depth 1 vs 4, C5 bf16 lines.  Usage: bash tools/r04_n.sh TAG
set -o pipefail
tag=${1:-r04n}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_layered.py tests/test_gpu_humanoid.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 120 python tools/tn_probe.py > gpurun_out/${tag}_probe.txt 2>&1 || { tail -5 gpurun_out/${tag}_probe.txt; exit 1; }
cat gpurun_out/${tag}_probe.txt
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_${n}.json'));print('$n', d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
}
C5="--env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --no-cpu-baseline --dtype bf16"
run c5_bf16 400 $C5
MRL_GEMM_TN_DEPTH=1 run c5_bf16_depth1 400 $C5
run c5_bf16_b 400 $C5
echo R04_N_OK
