# A/B: bf16 PROB / LOSSES / SURRGRAD row passes at 4 waves/SIMD (spilling) vs the default
set -o pipefail
cd $GRAFT_REPO_ROOT
for net in 4,2,softmax 11,3,gauss; do
  for lib in modular_rl_amd/libmrl_hip.so tools/ablate/libmrl_hip_occ4.so modular_rl_amd/libmrl_hip.so tools/ablate/libmrl_hip_occ4.so; do
    MRL_LIB_PATH=$lib MRL_PROBE_NET=$net MRL_PROBE_DTYPE=bf16 timeout -k 10 120 python tools/fvp_probe.py 2>&1 | grep "^\[" | grep -v uncached || exit 1
  done
done
