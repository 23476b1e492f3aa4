# C5 per-iteration trims (one MI355X): batched colsum loads, the VF fit's pinned tape
# input, the rollout's bf16 obs rows written by mrl_rollout_obs; their tests, then C5
# lines.  Usage (on the box): bash tools/r04_l.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04l2}
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_humanoid.py tests/test_gpu_bf16.py tests/test_gpu_iteration.py tests/test_gpu_golden_r3.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_${n}.json'));print('$n', d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
}
C5="--env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --no-cpu-baseline"
run c5_bf16 400 $C5 --dtype bf16
run c5_bf16_b 400 $C5 --dtype bf16
run c5_fp32 500 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 --no-cpu-baseline
echo R04_L_OK
