# rocprofv3 kernel-trace summary + separate FETCH_SIZE / WRITE_SIZE passes of the default
# bench (or of `bench.py EXTRA...`), and the per-role HBM bytes per launch.
# Usage (on the box): bash tools/prof_pmc_run.sh TAG [bench args...]  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-prof}
shift
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
echo PROF_OK
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${tag}_pmc_f.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${tag}_pmc_w.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write --out gpurun_out/${tag}_pmc.json > /dev/null
echo PMC_OK
