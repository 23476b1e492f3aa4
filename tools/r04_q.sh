# Host part of the snapshot capture moved under the prelaunched rollout (one MI355X):
# checkpoint / iteration tests, then the default line's kernel trace and host gaps.
# Usage: bash tools/r04_q.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04q}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_checkpoint.py tests/test_gpu_iteration.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_host_gap.txt && tail -4 gpurun_out/${tag}_host_gap.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${tag}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print(d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
echo R04_Q_OK
