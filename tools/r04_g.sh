# Quick round-4 check (one MI355X): split / iteration / PPO tests, split probe, default
# bench line, rocprofv3 kernel summary.  Usage: bash tools/r04_g.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04g}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_iteration.py tests/test_gpu_ppo.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
MRL_VJP_SPLIT_FORM=2 timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { tail -5 gpurun_out/${tag}_probe.log; exit 1; }
grep -E "fvp|fused" gpurun_out/${tag}_probe.log
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_hopper.json 2> gpurun_out/${tag}_bench_hopper.err || { echo BENCH_FAILED; tail -5 gpurun_out/${tag}_bench_hopper.err; exit 1; }
cat gpurun_out/${tag}_bench_hopper.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv | tail -4
echo R04_G_OK
