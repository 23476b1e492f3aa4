# One-call round-4 sweep (one MI355X, <= 20 min): the whole GPU suite, then the A/B
# measurements (Hopper quad-step variants, fit CU cap, VJP16 VALU head gradient, JVP rows
# at 3 waves per SIMD), the Humanoid step stamps, the C5 lines (bf16, co-scheduled fit)
# and the default line with its rocprofv3 summary.  Usage: bash tools/r04_all.sh TAG
set -o pipefail
tag=${1:-r04x}
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
hb() {  # name, env..., -- bench args
  n=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/${tag}_bench_$n.json 2> gpurun_out/${tag}_bench_$n.err || { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_$n.json'));print('$n', d['ms_per_step'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'], d['roofline'].get('mean_launch_ms'))"
}
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline"
hb default $B
hb sel1 MRL_LIB_PATH=tools/ablate/libmrl_hip_sel1.so $B
hb lim1 MRL_LIB_PATH=tools/ablate/libmrl_hip_lim1.so $B
timeout -k 10 300 env MRL_LIB_PATH=tools/ablate/libmrl_hip_sel1.so python -u -m pytest tests/test_gpu_pipeline.py -x -q -m gpu -k "rollout" --timeout 120 --timeout-method thread > gpurun_out/${tag}_sel1_tests.log 2>&1 || { echo SEL1_TESTS_FAILED; tail -30 gpurun_out/${tag}_sel1_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_sel1_tests.log
hb fit128 MRL_FIT_CUS=128 $B
hb vg2 MRL_VJP16_VG2=1 $B
hb occ3 MRL_LIB_PATH=tools/ablate/libmrl_hip_occ3.so $B
for v in default vg2; do
  if [ $v = vg2 ]; then export MRL_VJP16_VG2=1; fi
  timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe_$v.log 2>&1 || { tail -5 gpurun_out/${tag}_probe_$v.log; exit 1; }
  echo "== probe $v"; grep "fvp rows" gpurun_out/${tag}_probe_$v.log
done
unset MRL_VJP16_VG2
timeout -k 10 200 python tools/humanoid_stamps.py 1024 > gpurun_out/${tag}_hm_stamps.txt 2>&1 || { echo STAMPS_FAILED; tail -5 gpurun_out/${tag}_hm_stamps.txt; exit 1; }
cat gpurun_out/${tag}_hm_stamps.txt
H="python bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 --dtype bf16 --no-cpu-baseline"
hb humanoid_bf16 $H
hb humanoid_bf16_cosched MRL_COSCHED_FIT=1 $H
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv | tail -2
echo R04_ALL_OK
