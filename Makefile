# Build libmrl_hip.so (gfx950 only) in-tree and the C oracle helpers.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := modular_rl_amd/csrc
SRCS := $(CSRC)/mlp_kernels.hip $(CSRC)/mlp_bf16.hip $(CSRC)/mlp_split.hip $(CSRC)/scan.hip $(CSRC)/rollout.hip $(CSRC)/gemm.hip $(CSRC)/gemm_bf16.hip $(CSRC)/runtime.hip
HDRS := $(wildcard $(CSRC)/*.h) include/mrl_hip.h
OBJS := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRCS))
LIB := modular_rl_amd/libmrl_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude

all: $(LIB)

# mlp_split.hip: no SLP vectorisation -- the packed-f32 (v_pk_fma_f32) head sums it formed
# gave run-to-run different results in a few 16-row groups per 4 M rows on gfx950
# (tools/determinism_probe.py); the explicit packed builtins stay
build/mlp_split.o: HIPFLAGS += -fno-slp-vectorize

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
