# Build libmrl_hip.so (gfx950 only) in-tree and the C oracle helpers.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := modular_rl_amd/csrc
SRCS := $(CSRC)/mlp_kernels.hip $(CSRC)/mlp_bf16.hip $(CSRC)/mlp_split.hip $(CSRC)/scan.hip $(CSRC)/rollout.hip $(CSRC)/gemm.hip $(CSRC)/gemm_bf16.hip $(CSRC)/runtime.hip
HDRS := $(wildcard $(CSRC)/*.h) include/mrl_hip.h
OBJS := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRCS))
LIB := modular_rl_amd/libmrl_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude

# C restatement of the TRPO graph's batch means (test infrastructure: tests only)
ORACLE_LIB := oracle/libmrl_oracle.so

# the product library only; the test-only C oracle (gcc -mavx2 -fopenmp) is `make oracle`
# (tests/conftest.py and __graft_entry__.build() run `make all oracle`)
all: $(LIB)


build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# Host-side UndefinedBehaviorSanitizer build of the same sources (the device code is
# unchanged: -fsanitize applies to the host compilation only, -Xarch_host before each
# flag).  tests/test_abi.py::test_host_code_under_ubsan runs the host queries and the
# argument checks of the C ABI against it in a child process.
CLANG_RT := $(firstword $(wildcard /opt/rocm/lib/llvm/lib/clang/*/lib/linux))
UBSAN_FLAGS := -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
UBSAN_OBJS := $(patsubst $(CSRC)/%.hip,build/ubsan/%.o,$(SRCS))
UBSAN_LIB := build/ubsan/libmrl_hip_ubsan.so

ubsan: $(UBSAN_LIB)

build/ubsan/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build/ubsan
	$(HIPCC) $(HIPFLAGS) -O1 $(UBSAN_FLAGS) -c $< -o $@

$(UBSAN_LIB): $(UBSAN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -shared-libsan -Xarch_host -fsanitize=undefined \
	  -Wl,-rpath,$(CLANG_RT) -o $@ $(UBSAN_OBJS)

oracle: $(ORACLE_LIB)
$(ORACLE_LIB): oracle/mlp_c.c
	gcc -O3 -mavx2 -ffp-contract=off -fopenmp -shared -fPIC -o $@ $<

clean:
	rm -rf build $(LIB) $(ORACLE_LIB)

.PHONY: all clean ubsan oracle
