# C5 bf16 kernel summary (one MI355X): rocprofv3 kernel trace + stats of a 3-iteration
# Humanoid bf16 bench.  Usage (on the box): bash tools/r04_k.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04k}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 --dtype bf16 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
head -25 gpurun_out/${tag}_prof/run_kernel_stats.csv | cut -c1-200
echo R04_K_OK
