# Round evidence on one MI355X, one parametrised recipe (replaces the per-round r0x_*.sh).
# Usage (on the box): bash tools/evidence.sh TAG STEP [STEP ...]  -> gpurun_out/TAG_*
#   tests        the whole GPU suite (pytest -m gpu)
#   hopper       the default bench line (C3 Hopper-v2 fp32, the driver's command)
#   prof         rocprofv3 --kernel-trace --stats of the default line + host gaps
#   pmc          separate FETCH_SIZE / WRITE_SIZE passes of the default line -> TAG_pmc.json
#   lines        C3 bf16, C2 bf16 / fp32, C5 bf16 / fp32 lines
#   sq           SQ wave-time split of the Fisher-product kernels (tools/fisher_probe.py, tools/sq_split.py)
#   issue        SQ issue floor of the persistent rollout per bench line (tools/rollout_issue.py)
#   stamps       per-phase stamps of the persistent Hopper rollout (tools/persistent_stamps.py)
#   det          run-to-run determinism of the Fisher-product kernels (tools/det_locate.py)
#   fisher       one Fisher product at 4.19 M rows: one-pass kernel vs the two-kernel pair
#   fisher_tests the Fisher-product GPU tests only (split / one-pass / full size)
#   gae          mrl_gae alone: exact-fit vs general kernel (MRL_GAE_GENERAL=1) + rocprof stats
#   pair         the default bench line with the two-kernel Fisher product (MRL_FISHER_ONEPASS=0)
#   layered_tests  the layered-path / Humanoid GPU tests only
#   c5prof       rocprofv3 kernel trace of the C5 bf16 line + the per-step timeline (tools/step_timeline.py)
#   c5 / c5_f32  C5 Humanoid fp32 line (split GEMMs / exact-f32 GEMMs: MRL_GEMM_SPLIT=0)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:?tag}
shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bench() {  # name, timeout, bench args...
  n=$1; t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/${tag}_bench_${n}.json 2> gpurun_out/${tag}_bench_${n}.err ||
    { echo BENCH_FAILED $n; tail -5 gpurun_out/${tag}_bench_${n}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_${n}.json'));print('$n', d['value'], d.get('trpo_iters_per_sec'), d.get('phase_ms_per_iter'), d['roofline']['frac'])"
}
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
      tail -1 gpurun_out/${tag}_tests.log ;;
    hopper) bench hopper 400 ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv \
        -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 ||
        { echo PROF_FAILED; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
      python tools/host_gap.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_host_gap.txt &&
        tail -4 gpurun_out/${tag}_host_gap.txt ;;
    pmc)  # counter passes serialise the dispatches: the rollout <-> iteration streams are ordered
          # by events there (MRL_XSTREAM_EVENT=1); a stream waiting on a memory value written by a
          # packet queued behind it would never run (r06i: the FETCH pass hung)
      export MRL_XSTREAM_EVENT=1
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o run \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_f.log 2>&1 || exit 1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o run \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_pmc_w.log 2>&1 || exit 1
      python tools/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write \
        --out gpurun_out/${tag}_pmc.json > /dev/null && echo PMC_OK
      unset MRL_XSTREAM_EVENT ;;
    lines)
      bench hopper_bf16 400 --dtype bf16 --no-cpu-baseline
      bench cartpole_bf16 400 --env CartPole-v0 --dtype bf16 --no-cpu-baseline
      bench cartpole 400 --env CartPole-v0 --no-cpu-baseline
      bench humanoid_bf16 500 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 10 --warmup 1 --dtype bf16 --no-cpu-baseline
      bench humanoid 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1 --no-cpu-baseline ;;
    sq)  # SQ wave-time split of the Fisher-product kernels (one 8-counter pass of the probe)
      timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
        -d gpurun_out/${tag}_sq -o run -- python3 tools/fisher_probe.py > gpurun_out/${tag}_sq.log 2>&1 ||
        { echo SQ_FAILED; tail -5 gpurun_out/${tag}_sq.log; exit 1; }
      python tools/sq_split.py gpurun_out/${tag}_sq mlp_fisher_hyb_kernel mlp_fvp_split_kernel mlp_vjp16_kernel \
        > gpurun_out/${tag}_sq.txt && cat gpurun_out/${tag}_sq.txt ;;
    issue)  # the persistent rollout's SQ issue floor per step -> profiles-style TAG_rollout_issue.json
      export MRL_XSTREAM_EVENT=1  # counter passes: event ordering (see pmc)
      for line in "Hopper-v2 fp32" "Hopper-v2 bf16" "CartPole-v0 bf16" "CartPole-v0 fp32"; do
        set -- $line
        timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY \
          SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${tag}_issue_$1_$2 -o run \
          -- python3 bench.py --env $1 --dtype $2 --steps 2 --warmup 1 --no-cpu-baseline \
          > gpurun_out/${tag}_issue_$1_$2.log 2>&1 || { echo ISSUE_FAILED $1 $2; tail -5 gpurun_out/${tag}_issue_$1_$2.log; exit 1; }
        python tools/rollout_issue.py gpurun_out/${tag}_issue_$1_$2 $1/$2 1024 --out gpurun_out/${tag}_rollout_issue.json
      done
      unset MRL_XSTREAM_EVENT ;;
    stamps)
      timeout -k 10 300 python -u tools/persistent_stamps.py Hopper-v2 > gpurun_out/${tag}_stamps.txt 2>&1 ||
        { tail -5 gpurun_out/${tag}_stamps.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/${tag}_stamps.txt | tail -20 ;;
    fisher)
      timeout -k 10 200 python -u tools/fisher_probe.py > gpurun_out/${tag}_fisher.log 2>&1 ||
        { tail -5 gpurun_out/${tag}_fisher.log; exit 1; }
      grep -v amdgpu.ids gpurun_out/${tag}_fisher.log ;;
    fisher_tests)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_fullsize.py -m gpu -x -q \
        --timeout 300 --timeout-method thread > gpurun_out/${tag}_fisher_tests.log 2>&1 ||
        { echo FISHER_TESTS_FAILED; tail -40 gpurun_out/${tag}_fisher_tests.log; exit 1; }
      tail -1 gpurun_out/${tag}_fisher_tests.log ;;
    gae)  # mrl_gae alone: the exact-fit kernel, the general one (MRL_GAE_GENERAL=1), and a rocprof pass
      timeout -k 10 120 python -u tools/gae_probe.py > gpurun_out/${tag}_gae.log 2>&1 &&
        MRL_GAE_GENERAL=1 timeout -k 10 120 python -u tools/gae_probe.py >> gpurun_out/${tag}_gae.log 2>&1 &&
        timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_gae_prof -o run --output-format csv \
          -- python3 tools/gae_probe.py >> gpurun_out/${tag}_gae.log 2>&1 || { tail -5 gpurun_out/${tag}_gae.log; exit 1; }
      grep -v amdgpu.ids gpurun_out/${tag}_gae.log | grep gae
      grep -h gae gpurun_out/${tag}_gae_prof/run_kernel_stats.csv ;;
    pair) MRL_FISHER_ONEPASS=0 bench pair 400 --no-cpu-baseline ;;
    layered_tests)
      timeout -k 10 900 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_humanoid.py -m gpu -x -q \
        --timeout 300 --timeout-method thread > gpurun_out/${tag}_layered_tests.log 2>&1 ||
        { echo LAYERED_TESTS_FAILED; tail -40 gpurun_out/${tag}_layered_tests.log; exit 1; }
      tail -1 gpurun_out/${tag}_layered_tests.log ;;
    c5prof)  # kernel trace of the C5 bf16 line: the layered rollout's per-step timeline
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_c5prof -o run --output-format csv \
        -- python3 bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 2 --warmup 1 --dtype ${C5DT:-bf16} \
        --no-cpu-baseline > gpurun_out/${tag}_c5prof.log 2>&1 || { echo C5PROF_FAILED; tail -5 gpurun_out/${tag}_c5prof.log; exit 1; }
      python tools/step_timeline.py gpurun_out/${tag}_c5prof/run_kernel_trace.csv > gpurun_out/${tag}_c5_timeline.txt &&
        cat gpurun_out/${tag}_c5_timeline.txt ;;
    c5) bench humanoid 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 --warmup 1 --no-cpu-baseline ;;
    c5_f32) MRL_GEMM_SPLIT=0 bench humanoid_f32gemm 600 --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 5 \
      --warmup 1 --no-cpu-baseline ;;
    det)
      REPS=8 timeout -k 10 200 python -u tools/det_locate.py > gpurun_out/${tag}_det.log 2>&1 ||
        { tail -5 gpurun_out/${tag}_det.log; exit 1; }
      grep -v amdgpu.ids gpurun_out/${tag}_det.log | head -4 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo EVIDENCE_OK $tag "$@"
