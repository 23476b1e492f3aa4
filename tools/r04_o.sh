# The fp32 Fisher product's kernels at C3 size (4.19 M rows, Hopper's 11-64-64-3 net;
# one MI355X): SQ wave-time split and HBM bytes per launch (separate FETCH_SIZE /
# WRITE_SIZE passes) of the split JVP rows, the exact-f32 VJP and the one-pass fused
# product.  Usage: bash tools/r04_o.sh TAG -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04o}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export MRL_PROBE_NCASES=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${tag}_sq -o run -- python3 tools/split_probe.py > gpurun_out/${tag}_sq.log 2>&1 || { echo SQ_FAILED; tail -5 gpurun_out/${tag}_sq.log; exit 1; }
python tools/sq_split.py gpurun_out/${tag}_sq mlp_fvp_split_kernel mlp_vjp16_kernel mlp_fisher_split_kernel mlp_rows_kernel > gpurun_out/${tag}_sq.txt || exit 1
cat gpurun_out/${tag}_sq.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_fetch -o run -- python3 tools/split_probe.py > gpurun_out/${tag}_f.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/${tag}_f.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_write -o run -- python3 tools/split_probe.py > gpurun_out/${tag}_w.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/${tag}_w.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${tag}_fetch gpurun_out/${tag}_write --out gpurun_out/${tag}_pmc.json || exit 1
grep -E "fvp|fused" gpurun_out/${tag}_sq.log
echo R04_O_OK
