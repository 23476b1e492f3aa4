# Remaining bench lines at the closing round-4 code (one MI355X): C3 bf16, C2 fp32.
# Usage: bash tools/r04_s.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04s}
cd $GRAFT_REPO_ROOT
run() {  # name, bench args...
  n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_${n}.json'));print('$n', d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
}
run hopper_bf16 --dtype bf16 --no-cpu-baseline
run cartpole --env CartPole-v0 --no-cpu-baseline
echo R04_S_OK
