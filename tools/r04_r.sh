# C2 bf16 (CartPole, 4096 x 1024) kernel trace + host gaps (one MI355X).  Usage: bash tools/r04_r.sh TAG
set -o pipefail
tag=${1:-r04r}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --env CartPole-v0 --dtype bf16 --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_host_gap.txt && tail -4 gpurun_out/${tag}_host_gap.txt
echo R04_R_OK
