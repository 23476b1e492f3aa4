# Rollout experiment loop (one MI355X): the rollout parity tests, then the persistent
# kernel's phase stamps (tools/persistent_stamps.py) and the production kernel's
# collect time (no stamps) for Hopper-v2 and CartPole-v0.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k "rollout or persistent" > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
timeout -k 10 300 python tools/persistent_stamps.py Hopper-v2 CartPole-v0 "$@" 2>&1 | grep -v amdgpu.ids
