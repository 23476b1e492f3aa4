# Round evidence, part B (one MI355X): the Humanoid bench lines, the rocprofv3 kernel
# summary of the default bench, PMC HBM-traffic passes and SQ passes.
# Usage (on the box): bash tools/evidence_b.sh TAG [pmc]   -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-ev}
cd $GRAFT_REPO_ROOT
run() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  cat gpurun_out/${tag}_bench_${n}.json
}
run humanoid 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1
run humanoid_bf16 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1 --dtype bf16
run humanoid8k_bf16 900 --env Humanoid-v2 --envs 8192 --hid 512,512,512 --steps 5 --warmup 1 --dtype bf16 --cpu-envs 64 --cpu-horizon 64
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || exit 1
if [ "$2" = "pmc" ]; then
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_f.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_w.log 2>&1 || exit 1
for c in "Hopper-v2 fp32" "Hopper-v2 bf16" "CartPole-v0 bf16" "CartPole-v0 fp32"; do
set -- $c
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${tag}_sq_$1_$2 -o run -- python3 bench.py --env $1 --dtype $2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_sq_$1_$2.log 2>&1 || exit 1
done
fi
echo EVIDENCE_B_OK
