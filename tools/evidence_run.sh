set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/ev_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/ev_tests.log; exit 1; }
tail -2 gpurun_out/ev_tests.log
timeout -k 10 400 python bench.py > gpurun_out/ev_bench_hopper.json 2> gpurun_out/ev_bench_hopper.err || exit 1
timeout -k 10 300 python tools/rollout_stamps.py > gpurun_out/ev_stamps.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 > gpurun_out/ev_bench_humanoid.json 2> gpurun_out/ev_bench_humanoid.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ev_prof.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ev_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ev_pmc_f.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ev_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ev_pmc_w.log 2>&1 || exit 1
echo EVIDENCE_OK
