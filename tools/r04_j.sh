# Round-4 C5 co-scheduling A/B (one MI355X): the fit's GEMMs capped in LDS
# (MRL_COSCHED_LDS), four-env Humanoid blocks (MRL_HM_WPB) and the rollout stream's
# priority (MRL_COSCHED_PRIO), bit-identity tests first.  Usage (on the box): bash tools/r04_j.sh TAG  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04j}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py::test_bf16_lds_limited_gemms_equal_default tests/test_gpu_humanoid.py "tests/test_gpu_iteration.py::test_cosched_fit_beside_wave_per_env_rollout_is_bit_identical" -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  cat gpurun_out/${tag}_bench_${n}.json
}
C5="--env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16 --no-cpu-baseline"
run c5_default 400 $C5
MRL_COSCHED_PRIO=1 run c5_prio 400 $C5
run c5_default2 400 $C5
MRL_COSCHED_PRIO=1 run c5_prio2 400 $C5
echo R04_J_OK
