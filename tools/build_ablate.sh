#!/bin/bash
# Diagnostic builds of libmrl_hip.so with -D switches (tools/ablate/libmrl_hip_<name>.so);
# select one at run time with MRL_LIB_PATH.  Usage: tools/build_ablate.sh NAME -DFLAG ...
set -e
name=$1; shift
out=tools/ablate/$name; mkdir -p $out
for f in mlp_kernels mlp_bf16 mlp_split scan rollout gemm gemm_bf16 runtime; do
  extra=""; [ $f = mlp_split ] && extra="-fno-slp-vectorize"  # as the Makefile
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude $extra "$@" \
    -c modular_rl_amd/csrc/$f.hip -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ablate/libmrl_hip_$name.so $out/*.o
rm -rf $out
echo tools/ablate/libmrl_hip_$name.so
