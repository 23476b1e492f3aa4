# Round-4 closing evidence (one MI355X): the whole GPU suite, the default bench line and
# its rocprofv3 kernel summary + host gaps, and the C2 / C5 bf16 lines.
# Usage (on the box): bash tools/r04_final.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04f}
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  cat gpurun_out/${tag}_bench_${n}.json
}
run hopper 400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_host_gap.txt && tail -4 gpurun_out/${tag}_host_gap.txt
run cartpole_bf16 300 --env CartPole-v0 --dtype bf16 --no-cpu-baseline
run humanoid_bf16 500 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16 --no-cpu-baseline
echo R04_FINAL_OK
