# Rollout A/B (one MI355X): the Hopper step with the branch-free row selections (default),
# without them (sel0), and with branch-free joint limits / health test too (lim1); rollout
# parity tests on the default build.  Usage: bash tools/r04_h.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04h}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_humanoid.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for v in default sel0 lim1 default; do
  if [ $v = default ]; then unset MRL_LIB_PATH; else export MRL_LIB_PATH=tools/ablate/libmrl_hip_$v.so; fi
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_bench_$v.json 2> gpurun_out/${tag}_bench_$v.err || { echo BENCH_FAILED $v; tail -5 gpurun_out/${tag}_bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_$v.json'));print('$v', d['ms_per_step'], d['phase_ms_per_iter'], d['roofline'].get('mean_launch_ms'))"
done
unset MRL_LIB_PATH
for fc in 128 96; do
  MRL_FIT_CUS=$fc timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_bench_fit$fc.json 2> gpurun_out/${tag}_bench_fit$fc.err || { echo BENCH_FAILED fit$fc; tail -5 gpurun_out/${tag}_bench_fit$fc.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_fit$fc.json'));print('fit$fc', d['ms_per_step'], d['phase_ms_per_iter'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q -m gpu -k vjp16_valu --timeout 120 --timeout-method thread > gpurun_out/${tag}_vg2_tests.log 2>&1 || { echo VG2_TESTS_FAILED; tail -30 gpurun_out/${tag}_vg2_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_vg2_tests.log
MRL_VJP16_VG2=1 timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe_vg2.log 2>&1 || { tail -5 gpurun_out/${tag}_probe_vg2.log; exit 1; }
echo "== probe vg2"; grep "fvp rows" gpurun_out/${tag}_probe_vg2.log
for v in default occ3; do
  if [ $v = default ]; then unset MRL_LIB_PATH; else export MRL_LIB_PATH=tools/ablate/libmrl_hip_$v.so; fi
  timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe_$v.log 2>&1 || { tail -5 gpurun_out/${tag}_probe_$v.log; exit 1; }
  echo "== probe $v"; grep "fvp rows" gpurun_out/${tag}_probe_$v.log
done
unset MRL_LIB_PATH
timeout -k 10 300 python tools/humanoid_stamps.py 1024 > gpurun_out/${tag}_hm_stamps.txt 2>&1 || { echo STAMPS_FAILED; tail -5 gpurun_out/${tag}_hm_stamps.txt; exit 1; }
cat gpurun_out/${tag}_hm_stamps.txt
echo R04_H_OK
