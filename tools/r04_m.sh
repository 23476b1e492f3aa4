# The Humanoid step's SQ issue floor at the four-env blocks (one MI355X): SQ passes of
# tools/humanoid_collect.py for bf16 / fp32 -> step_issue.py.  Usage: bash tools/r04_m.sh TAG
set -o pipefail
tag=${1:-r04m}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
cp profiles/rollout_issue_r04.json gpurun_out/${tag}_rollout_issue.json
for dt in bf16 fp32; do
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/${tag}_sq_hm_$dt -o run -- python3 tools/humanoid_collect.py 1024 32 $dt > gpurun_out/${tag}_sq_hm_$dt.log 2>&1 || { echo SQ_FAILED $dt; tail -5 gpurun_out/${tag}_sq_hm_$dt.log; exit 1; }
python tools/step_issue.py gpurun_out/${tag}_sq_hm_$dt Humanoid-v2/$dt --out gpurun_out/${tag}_rollout_issue.json > gpurun_out/${tag}_issue_$dt.txt || exit 1
done
python -c "import json;d=json.load(open('gpurun_out/${tag}_rollout_issue.json'));print(json.dumps({k:v for k,v in d.items() if k.startswith('Humanoid')})[:1500])"
echo R04_M_OK
