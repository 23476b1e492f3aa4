# Round evidence, part A (one MI355X): full GPU suite + the Hopper / CartPole bench lines.
# Usage (on the box): bash tools/evidence_a.sh TAG   -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-ev}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  cat gpurun_out/${tag}_bench_${n}.json
}
run hopper 400
run cartpole_bf16 400 --env CartPole-v0 --steps 5 --dtype bf16
run cartpole 400 --env CartPole-v0 --steps 5
run hopper_bf16 400 --steps 10 --dtype bf16
echo EVIDENCE_A_OK
