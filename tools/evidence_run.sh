# Round evidence on one MI355X: GPU tests, bench lines (Hopper default, Humanoid), the
# rocprofv3 kernel summary of the default bench and the PMC HBM-traffic passes.
# Usage (on the box): bash tools/evidence_run.sh TAG    -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-ev}
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_hopper.json 2> gpurun_out/${tag}_bench_hopper.err || exit 1
cat gpurun_out/${tag}_bench_hopper.json
timeout -k 10 600 python bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 > gpurun_out/${tag}_bench_humanoid.json 2> gpurun_out/${tag}_bench_humanoid.err || exit 1
cat gpurun_out/${tag}_bench_humanoid.json
timeout -k 10 400 python bench.py --env CartPole-v0 --steps 5 > gpurun_out/${tag}_bench_cartpole.json 2> gpurun_out/${tag}_bench_cartpole.err || exit 1
cat gpurun_out/${tag}_bench_cartpole.json
for c in "Hopper-v2 --steps 10" "CartPole-v0 --steps 5" "Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1"; do
n=$(echo $c | cut -d' ' -f1 | cut -d- -f1 | tr A-Z a-z)
timeout -k 10 600 python bench.py --env $c --dtype bf16 --no-cpu-baseline > gpurun_out/${tag}_bench_${n}_bf16.json 2> gpurun_out/${tag}_bench_${n}_bf16.err || exit 1
cat gpurun_out/${tag}_bench_${n}_bf16.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || exit 1
if [ "$2" = "pmc" ]; then
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_f.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_w.log 2>&1 || exit 1
fi
echo EVIDENCE_OK
