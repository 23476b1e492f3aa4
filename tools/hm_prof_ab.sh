# rocprofv3 kernel durations of the C5 bf16 line for several builds on one box:
#   bash tools/hm_prof_ab.sh TAG NAME=SO_PATH ... (NAME=default: the in-tree build)
set -o pipefail
tag=${1:?tag}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}; so=${spec#*=}
  [ "$so" = default ] && so=""
  MRL_LIB_PATH=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_$name -o run --output-format csv \
    -- python3 bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 2 --warmup 1 --dtype bf16 --no-cpu-baseline \
    > gpurun_out/${tag}_$name.log 2>&1 || { echo PROF_FAILED $name; tail -5 gpurun_out/${tag}_$name.log; exit 1; }
  echo "== $name"
  python tools/step_timeline.py gpurun_out/${tag}_$name/run_kernel_trace.csv | tail -9
done
