# determinism of the split JVP across diagnostic builds + timing of the variants
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in default noslp nofence w12; do
  lib=""; [ $v != default ] && lib=tools/ablate/libmrl_hip_$v.so
  MRL_LIB_PATH=$lib REPS=4 timeout -k 10 200 python tools/determinism_probe.py > gpurun_out/det2_$v.log 2>&1 || { tail -5 gpurun_out/det2_$v.log; exit 1; }
  echo "== $v"; grep split gpurun_out/det2_$v.log
  MRL_LIB_PATH=$lib MRL_FISHER=split timeout -k 10 200 python tools/split_probe.py > gpurun_out/probe2_$v.log 2>&1 || { tail -5 gpurun_out/probe2_$v.log; exit 1; }
  grep fvp gpurun_out/probe2_$v.log
done
