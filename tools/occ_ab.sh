# A/B of the bf16 row kernels' occupancy (3 vs 2 waves/SIMD) and the FVP rows grid cap
set -o pipefail
cd $GRAFT_REPO_ROOT
for net in 4,2,softmax 11,3,gauss; do
  for lib in modular_rl_amd/libmrl_hip.so tools/ablate/libmrl_hip_occ2.so; do
    for nb in 0 512 1024; do
      if [ $nb = 0 ]; then unset MRL_ROWS_BF16_BLOCKS; else export MRL_ROWS_BF16_BLOCKS=$nb; fi
      echo "== $net $lib blocks=$nb"
      MRL_LIB_PATH=$lib MRL_PROBE_NET=$net MRL_PROBE_DTYPE=bf16 timeout -k 10 120 python tools/fvp_probe.py 2>&1 | grep "^\[" || exit 1
    done
  done
done
