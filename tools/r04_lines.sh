# Round-4 bench lines beside the default one (one MI355X): PMC traffic of the default
# line (tools/prof_pmc_run.sh), then C3 bf16, C2 bf16, C2 fp32.  Usage: bash tools/r04_lines.sh TAG
set -o pipefail
tag=${1:-r04l}
cd $GRAFT_REPO_ROOT
bash tools/prof_pmc_run.sh ${tag} || exit 1
run() {  # name, bench args...
  n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_${n}.json'));print('$n', d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
}
run hopper_bf16 --dtype bf16
run cartpole_bf16 --env CartPole-v0 --dtype bf16
run cartpole --env CartPole-v0
run humanoid_bf16 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16
echo R04_LINES_OK
