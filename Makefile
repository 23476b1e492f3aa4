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

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
