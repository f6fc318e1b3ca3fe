# Builds the product library (HIP kernels + C ABI) for gfx950, in-tree, and the
# CPU oracle (test infrastructure).  `python -c "import __graft_entry__ as g; g.build()"`
# runs this.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS ?= -O3 -fPIC -std=c++17 -Wall -Wextra
PKG      := rustnetworkstack_amd
CSRC     := $(PKG)/csrc
BUILD    := $(PKG)/build
LIB      := $(PKG)/librns_checksum.so

CABI_TEST := tests/c/test_batch_abi

all: $(LIB) oracle $(CABI_TEST)

# A plain C caller of the C ABI (no torch): built here, run by tests/test_c_caller.py on a GPU.
$(CABI_TEST): tests/c/test_batch_abi.c oracle/csum_oracle.c include/rns_checksum.h $(LIB)
	gcc -std=gnu11 -O1 -Wall -Wextra -Werror -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include \
	    tests/c/test_batch_abi.c oracle/csum_oracle.c -L$(PKG) -lrns_checksum -Wl,-rpath,'$$ORIGIN/../../$(PKG)' \
	    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread -o $@

# One translation unit per kernel family (rns_launch.hpp), compiled in parallel (make -j).
HIP_SRCS := $(wildcard $(CSRC)/*.hip)
HIP_HDRS := $(wildcard $(CSRC)/*.hpp) include/rns_checksum.h
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIP_SRCS))

$(BUILD)/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@

$(BUILD)/host_checksum.o: $(CSRC)/host_checksum.cpp include/rns_checksum.h
	@mkdir -p $(BUILD)
	g++ $(CXXFLAGS) -Iinclude -c $< -o $@

$(BUILD)/host_io.o: $(CSRC)/host_io.cpp include/rns_checksum.h
	@mkdir -p $(BUILD)
	g++ $(CXXFLAGS) -Iinclude -c $< -o $@

$(LIB): $(HIP_OBJS) $(BUILD)/host_checksum.o $(BUILD)/host_io.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

oracle:
	$(MAKE) -C oracle

# A/B experiment build: `make -j8 ab ABDEF="-DRNS_ROWS_D=4" ABNAME=d4` -> tools/ab/librns_checksum_d4.so
# (load it with RNS_CHECKSUM_LIB=...).  Knobs: RNS_CLASS_LOG2G / RNS_CLASS_U (class-kernel shapes),
# RNS_MIXED_OCC / RNS_FILL_OCC / RNS_CHAIN_OCC (waves/SIMD bounds), RNS_ROWS_D, RNS_STREAM_MAXLEN, ...
ABDEF  ?= -DRNS_ROWS_D=4
ABNAME ?= d4
AB_BUILD := $(BUILD)/ab_$(ABNAME)
AB_OBJS  := $(patsubst $(CSRC)/%.hip,$(AB_BUILD)/%.o,$(HIP_SRCS))
AB_LIB   := tools/ab/librns_checksum_$(ABNAME).so
$(AB_BUILD)/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(AB_BUILD)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(ABDEF) -Iinclude -c $< -o $@
$(AB_LIB): $(AB_OBJS) $(BUILD)/host_checksum.o $(BUILD)/host_io.o
	@mkdir -p tools/ab
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

ab: $(AB_LIB)

# Register / occupancy report for every kernel instantiation.
resources: $(HIP_OBJS)
	for o in $(HIP_OBJS); do bash tools/scratch_report.sh $$o | tail -n +2; done | sort -k3 | \
	    awk 'BEGIN { print "scratch_B_per_lane\tvgprs\tkernel" } { print }'

asm: $(HIP_SRCS)
	@mkdir -p $(BUILD)/asm
	for f in $(HIP_SRCS); do (cd $(BUILD)/asm && $(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -I../../../include \
	    --cuda-device-only -S ../../../$$f -o $$(basename $$f .hip).s) || exit 1; done

clean:
	rm -rf $(BUILD) $(LIB) $(CABI_TEST)
	$(MAKE) -C oracle clean

.PHONY: all oracle resources asm clean ab
