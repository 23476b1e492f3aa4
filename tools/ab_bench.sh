# A/B of bench lines on one box: bash tools/ab_bench.sh TAG TESTFILES REPS NAME=ENV[,ENV] ...
# (TESTFILES: "-" for none).  Each NAME runs `python bench.py` (C3 fp32 default) with its
# env assignments (MRL_LIB_PATH=tools/gvar/x.so selects a variant build), alternating;
# BENCH_ARGS (environment) adds bench.py arguments, e.g. another line.
set -o pipefail
tag=$1; tests=$2; reps=$3; shift 3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ "$tests" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    [ "$envs" = "$spec" ] && envs=""
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/${tag}_${name}$rep.json 2> gpurun_out/${tag}_${name}$rep.err || { tail -5 gpurun_out/${tag}_${name}$rep.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${tag}_${name}$rep.json'));print('${name}$rep', d['value'], d['trpo_iters_per_sec'], d['phase_ms_per_iter'])"
  done
done
