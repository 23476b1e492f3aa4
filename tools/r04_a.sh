# Round-4 check (one MI355X): GPU suite, default bench line, rocprofv3 kernel summary.
# Usage (on the box): bash tools/r04_a.sh TAG [quick]  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04}
cd $GRAFT_REPO_ROOT
if [ "$2" = "quick" ]; then
  sel="tests/test_gpu_pipeline.py tests/test_gpu_rccl.py tests/test_gpu_golden_r3.py tests/test_gpu_iteration.py"
else
  sel="tests"
fi
timeout -k 10 900 python -u -m pytest $sel -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_hopper.json 2> gpurun_out/${tag}_bench_hopper.err || { echo BENCH_FAILED; tail -5 gpurun_out/${tag}_bench_hopper.err; exit 1; }
cat gpurun_out/${tag}_bench_hopper.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
echo R04_A_OK
