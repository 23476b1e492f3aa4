# FETCH_SIZE / WRITE_SIZE of the one-pass Fisher product, the default build and the role
# probes (tools/role_probe.sh: 1 = JVP role only, 2 = VJP role only), each counter its own
# rocprofv3 pass over tools/fisher_probe.py.  Usage (on the box): bash tools/fisher_pmc.sh TAG
set -o pipefail
tag=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in default role1 role2; do
  lib=""
  [ $v != default ] && lib=$GRAFT_REPO_ROOT/tools/gvar/libmrl_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    MRL_LIB_PATH=$lib MRL_PROBE_ROWS=4194304 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv \
      -d gpurun_out/${tag}_${v}_$c -o run -- python3 tools/fisher_probe.py > gpurun_out/${tag}_${v}_$c.log 2>&1 ||
      { echo PMC_FAILED $v $c; tail -5 gpurun_out/${tag}_${v}_$c.log; exit 1; }
    echo PMC_OK $v $c
  done
done
