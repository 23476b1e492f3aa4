# Humanoid step change check on one MI355X: bash tools/hm_check.sh TAG [bench]
#   the Humanoid GPU tests, the step's phase stamps (tools/humanoid_stamps.py) and,
#   with "bench", the C5 bf16 line
set -o pipefail
tag=${1:?tag}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_humanoid.py tests/test_humanoid_physics.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_hm_tests.log 2>&1 || { echo HM_TESTS_FAILED; tail -30 gpurun_out/${tag}_hm_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_hm_tests.log
timeout -k 10 300 python -u tools/humanoid_stamps.py > gpurun_out/${tag}_hm_stamps.txt 2>&1 ||
  { tail -5 gpurun_out/${tag}_hm_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_hm_stamps.txt
if [ "$2" = bench ]; then
  timeout -k 10 500 python bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1 --dtype bf16 \
    --no-cpu-baseline > gpurun_out/${tag}_bench_humanoid_bf16.json 2> gpurun_out/${tag}_bench_humanoid_bf16.err ||
    { tail -5 gpurun_out/${tag}_bench_humanoid_bf16.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_humanoid_bf16.json'));print(d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
fi
echo HM_CHECK_OK
