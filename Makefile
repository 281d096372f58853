# mxk8s native build — gfx950 (MI355X) only.
#
#   make            build every native artefact in-tree
#   make kernels    HIP kernel library  mxk8s/_lib/libmxkernels.so
#   make gemm-exp   the same library with every A/B GEMM schedule and the
#                   attention forward A/B variants 5-9
#                   (-DMXK_GEMM_EXPERIMENTS) -> mxk8s/_lib/libmxkernels_exp.so,
#                   selected with MXK_KERNELS_LIB (python -m mxk8s.validate.gemm)
#   make node       C++ node library    mxk8s/_lib/libmxnode.so (+ CLIs in bin/)
#   make tools      validator binaries  bin/mx-vector-add bin/mx-gemm-bench bin/mx-allreduce-perf
#   make test-native  host unit tests of libmxnode (ASan+UBSan build)
#   make test-native-tsan  libmxnode re-entrancy test under ThreadSanitizer
#
# Everything lands inside the repo so `gpurun` snapshots carry it to the box.

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
OUT_LIB   := mxk8s/_lib
OUT_BIN   := bin
BUILD     := build

HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wshadow -Wno-unused-function \
             -Inative/kernels
CXXFLAGS  := -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Inative/libmxnode -I$(ROCM)/include
LDLIBS_NODE := -ldl -lpthread

KERNEL_SRCS := native/kernels/gemm_bf16.hip native/kernels/vector_add.hip \
               native/kernels/fused_ops.hip native/kernels/optim.hip native/kernels/attention.hip native/kernels/attention_bwd256.hip native/kernels/attention_fwd256.hip native/kernels/attention_dq256.hip \
               native/kernels/gemm_bf16_layouts.hip native/kernels/xent.hip native/kernels/contention.hip
KERNEL_OBJS := $(patsubst native/kernels/%.hip,$(BUILD)/kernels/%.o,$(KERNEL_SRCS))
EXP_SRCS    := $(KERNEL_SRCS) $(wildcard native/kernels/experiments/*.hip)
EXP_OBJS    := $(patsubst native/kernels/%.hip,$(BUILD)/exp/%.o,$(EXP_SRCS))
KERNEL_HDRS := $(wildcard native/kernels/*.h)

NODE_SRCS := $(wildcard native/libmxnode/*.cc)
NODE_OBJS := $(patsubst native/libmxnode/%.cc,$(BUILD)/node/%.o,$(NODE_SRCS))
NODE_HDRS := $(wildcard native/libmxnode/*.h)

.PHONY: all kernels gemm-exp node tools clean test-native test-native-tsan fake-amdsmi
all: kernels node tools fake-amdsmi

kernels: $(OUT_LIB)/libmxkernels.so

# the 256-row dQ kernel's softmax beside MFMAs: no SLP-packed v_pk_*_f32
# (an anti-lever beside MFMAs at one wave per SIMD; -1.5 % on the backward)
$(BUILD)/kernels/attention_dq256.o: HIPFLAGS += -fno-slp-vectorize
$(BUILD)/exp/attention_dq256.o: HIPFLAGS += -fno-slp-vectorize

$(BUILD)/kernels/%.o: native/kernels/%.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT_LIB)/libmxkernels.so: $(KERNEL_OBJS)
	@mkdir -p $(OUT_LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

gemm-exp: $(OUT_LIB)/libmxkernels_exp.so

$(BUILD)/exp/%.o: native/kernels/%.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DMXK_GEMM_EXPERIMENTS -c $< -o $@

$(OUT_LIB)/libmxkernels_exp.so: $(EXP_OBJS)
	@mkdir -p $(OUT_LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

# ---- node library + CLIs (plain C++17, no GPU needed to build or test) ----
node: $(OUT_LIB)/libmxnode.so $(OUT_BIN)/mx-gpu-enum $(OUT_BIN)/mx-cdi-gen

$(BUILD)/node/%.o: native/libmxnode/%.cc $(NODE_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT_LIB)/libmxnode.so: $(NODE_OBJS)
	@mkdir -p $(OUT_LIB)
	$(CXX) -shared -o $@ $^ $(LDLIBS_NODE)

$(OUT_BIN)/mx-gpu-enum: native/tools/mx_gpu_enum.cc $(NODE_OBJS)
	@mkdir -p $(OUT_BIN)
	$(CXX) $(CXXFLAGS) -o $@ $< $(NODE_OBJS) $(LDLIBS_NODE)

$(OUT_BIN)/mx-cdi-gen: native/tools/mx_cdi_gen.cc $(NODE_OBJS)
	@mkdir -p $(OUT_BIN)
	$(CXX) $(CXXFLAGS) -o $@ $< $(NODE_OBJS) $(LDLIBS_NODE)

# ---- validator binaries (HIP / RCCL / rocBLAS) ----
tools: $(OUT_BIN)/mx-vector-add $(OUT_BIN)/mx-gemm-bench $(OUT_BIN)/mx-allreduce-perf

$(BUILD)/tools/%.o: native/tools/%.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/tools/allreduce_perf.o: native/rccl_bench/allreduce_perf.cc native/rccl_bench/sweep_plan.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OUT_BIN)/mx-vector-add: $(BUILD)/tools/vector_add_main.o $(BUILD)/kernels/vector_add.o
	@mkdir -p $(OUT_BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^

$(OUT_BIN)/mx-gemm-bench: $(BUILD)/tools/gemm_bench_main.o $(BUILD)/kernels/gemm_bf16.o $(BUILD)/kernels/gemm_bf16_layouts.o
	@mkdir -p $(OUT_BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ -L$(ROCM)/lib -lrocblas -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib

$(OUT_BIN)/mx-allreduce-perf: $(BUILD)/tools/allreduce_perf.o
	@mkdir -p $(OUT_BIN)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ -L$(ROCM)/lib -lrccl -lrocprofiler-sdk-roctx -lpthread -Wl,-rpath,$(ROCM)/lib

# ---- scriptable fake libamd_smi.so (CPU test tier: MXK8S_AMDSMI_LIB) ----
fake-amdsmi: $(BUILD)/test/libfake_amdsmi.so

$(BUILD)/test/libfake_amdsmi.so: native/libmxnode/tests/fake_amdsmi.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -shared -o $@ $< -lpthread

# ---- host tests (sanitized) ----
test-native: $(BUILD)/asan/test_mxnode
	$(BUILD)/asan/test_mxnode tests/fixtures/sysfs

$(BUILD)/asan/test_mxnode: native/libmxnode/tests/test_mxnode.cc $(NODE_SRCS) $(NODE_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -g -fsanitize=address,undefined -fno-omit-frame-pointer -o $@ \
	    native/libmxnode/tests/test_mxnode.cc $(NODE_SRCS) $(LDLIBS_NODE)

test-native-tsan: $(BUILD)/tsan/test_mxnode_threads
	TSAN_OPTIONS=halt_on_error=1 $(BUILD)/tsan/test_mxnode_threads tests/fixtures/sysfs

$(BUILD)/tsan/test_mxnode_threads: native/libmxnode/tests/test_mxnode_threads.cc $(NODE_SRCS) $(NODE_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -g -fsanitize=thread -o $@ \
	    native/libmxnode/tests/test_mxnode_threads.cc $(NODE_SRCS) $(LDLIBS_NODE)

clean:
	rm -rf $(BUILD) $(OUT_LIB)/*.so $(OUT_BIN)
