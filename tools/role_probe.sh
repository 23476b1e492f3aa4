#!/bin/bash
# Diagnostic builds of the one-pass Fisher kernel with one role idle (MRL_FISHER_ROLE_PROBE
# 1: VJP tiles skipped, 2: JVP tiles skipped; barriers unchanged; 3: no round barrier) into tools/gvar/, for
# tools/fisher_probe.py under MRL_LIB_PATH.  CPU-side build only.
set -e
mkdir -p build/var tools/gvar
OBJS="build/mlp_bf16.o build/mlp_split.o build/scan.o build/rollout.o build/gemm.o build/gemm_bf16.o build/runtime.o"
for v in 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude \
    -DMRL_FISHER_ROLE_PROBE=$v -c modular_rl_amd/csrc/mlp_kernels.hip -o build/var/mlp_kernels_role$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/gvar/libmrl_role$v.so build/var/mlp_kernels_role$v.o $OBJS
done
