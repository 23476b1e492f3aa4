# Humanoid step change on one MI355X against a baseline build:
#   bash tools/hm_ab.sh TAG BASE_SO [REPS]
# bit-identity of the step over 256 envs x 64 steps (tools/hm_twin_ab.py), the Humanoid
# GPU tests, the phase stamps, and a C5 bf16 A/B of REPS pairs (tools/ab_bench.sh)
set -o pipefail
tag=${1:?tag}; base=${2:?base so}; reps=${3:-2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MRL_LIB_PATH=$base timeout -k 10 200 python -u tools/hm_twin_ab.py run /tmp/twin_base.npz > gpurun_out/${tag}_twin.log 2>&1 &&
  timeout -k 10 200 python -u tools/hm_twin_ab.py run /tmp/twin_new.npz >> gpurun_out/${tag}_twin.log 2>&1 ||
  { tail -5 gpurun_out/${tag}_twin.log; exit 1; }
python tools/hm_twin_ab.py cmp /tmp/twin_base.npz /tmp/twin_new.npz >> gpurun_out/${tag}_twin.log 2>&1
twin=$?
grep -v amdgpu gpurun_out/${tag}_twin.log | grep -v saved
[ $twin = 0 ] || { echo NOT_BIT_IDENTICAL; exit 1; }
bash tools/hm_check.sh $tag || exit 1
BENCH_ARGS="--env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1 --dtype bf16" \
  bash tools/ab_bench.sh ${tag}_ab - $reps base=MRL_LIB_PATH=$base new
