# split VJP forms: timing + SQ counters (one MI355X)
set -o pipefail
tag=${1:-r04e}
cd $GRAFT_REPO_ROOT
for f in 1 2; do
  MRL_FISHER=split MRL_VJP_SPLIT_FORM=$f timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe$f.log 2>&1 || { tail -5 gpurun_out/${tag}_probe$f.log; exit 1; }
  echo "== VJP form $f"; grep -E "fvp|fused" gpurun_out/${tag}_probe$f.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MRL_FISHER=split MRL_VJP_SPLIT_FORM=2 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${tag}_sq -o run -- python3 tools/split_probe.py > gpurun_out/${tag}_sq.log 2>&1 || { echo SQ_FAILED; tail -5 gpurun_out/${tag}_sq.log; exit 1; }
python tools/sq_split.py gpurun_out/${tag}_sq split mlp_rows_kernel mlp_vjp16 > gpurun_out/${tag}_sq.txt
cat gpurun_out/${tag}_sq.txt
echo R04_E_OK
