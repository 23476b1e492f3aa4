# Persistent-rollout stamps of the in-tree library and of diagnostic builds
# (tools/ablate/libmrl_hip_<name>.so).  Usage: bash tools/exp_variants.sh ENV name...
set -o pipefail
cd $GRAFT_REPO_ROOT
env=$1; shift
timeout -k 10 120 python tools/persistent_stamps.py $env 2>&1 | grep -v amdgpu.ids | sed 's/^/base /'
for n in "$@"; do
  MRL_LIB_PATH=tools/ablate/libmrl_hip_$n.so timeout -k 10 120 python tools/persistent_stamps.py $env 2>&1 | grep -v amdgpu.ids | sed "s/^/$n /"
done
