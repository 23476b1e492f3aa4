# One Fisher product at 4.19 M rows (tools/fisher_probe.py: ms per product) and its FETCH_SIZE
# pass, for the default build and tools/gvar/libmrl_<v>.so variants.
# Usage (on the box): bash tools/fisher_var.sh TAG v1 v2 ...
set -o pipefail
tag=${1:?tag}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in default "$@"; do
  lib=""
  [ $v != default ] && lib=$GRAFT_REPO_ROOT/tools/gvar/libmrl_$v.so
  MRL_LIB_PATH=$lib timeout -k 10 150 python -u tools/fisher_probe.py > gpurun_out/${tag}_$v.log 2>&1 ||
    { echo PROBE_FAILED $v; tail -5 gpurun_out/${tag}_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${tag}_$v.log
  MRL_LIB_PATH=$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d gpurun_out/${tag}_${v}_FETCH -o run -- python3 tools/fisher_probe.py > gpurun_out/${tag}_${v}_pmc.log 2>&1 ||
    { echo PMC_FAILED $v; tail -5 gpurun_out/${tag}_${v}_pmc.log; exit 1; }
done
