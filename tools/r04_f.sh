# Round-4 fused Fisher product check (one MI355X): split tests, probe timings, then the
# whole GPU suite, the default bench line and its rocprofv3 kernel summary.
# Usage (on the box): bash tools/r04_f.sh TAG  -> gpurun_out/TAG_*
set -o pipefail
tag=${1:-r04f}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${tag}_split_tests.log 2>&1 || { echo SPLIT_TESTS_FAILED; tail -40 gpurun_out/${tag}_split_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_split_tests.log
MRL_VJP_SPLIT_FORM=2 timeout -k 10 200 python tools/split_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { tail -5 gpurun_out/${tag}_probe.log; exit 1; }
grep -E "fvp|fused" gpurun_out/${tag}_probe.log
bash tools/r04_a.sh $tag
