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

$(BUILD)/rns_checksum.o: $(CSRC)/rns_checksum.hip include/rns_checksum.h
	@mkdir -p $(BUILD)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@

$(BUILD)/host_checksum.o: $(CSRC)/host_checksum.cpp include/rns_checksum.h
	@mkdir -p $(BUILD)
	g++ $(CXXFLAGS) -Iinclude -c $< -o $@

$(BUILD)/host_io.o: $(CSRC)/host_io.cpp include/rns_checksum.h
	@mkdir -p $(BUILD)
	g++ $(CXXFLAGS) -Iinclude -c $< -o $@

$(LIB): $(BUILD)/rns_checksum.o $(BUILD)/host_checksum.o $(BUILD)/host_io.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

oracle:
	$(MAKE) -C oracle

# A/B experiment build: `make ab ABDEF="-DRNS_CLASS_U=1,4,4,3,4" ABNAME=u3` -> tools/ab/librns_checksum_u3.so
# (load it with RNS_CHECKSUM_LIB=...).  Knobs: RNS_CLASS_LOG2G / RNS_CLASS_U (mixed-kernel class shapes),
# RNS_MIXED_OCC (waves/SIMD bound), RNS_FILL_BLOCK, RNS_FILL_NOSTORE, RNS_RX_PLAIN.
ABDEF  ?= -DRNS_CLASS_U=1,4,4,3,4
ABNAME ?= u3
AB_LIB := tools/ab/librns_checksum_$(ABNAME).so
$(AB_LIB): $(CSRC)/rns_checksum.hip $(BUILD)/host_checksum.o $(BUILD)/host_io.o include/rns_checksum.h
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(ABDEF) -Iinclude -c $< -o $(BUILD)/rns_checksum_$(ABNAME).o
	@mkdir -p tools/ab
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(BUILD)/rns_checksum_$(ABNAME).o $(BUILD)/host_checksum.o $(BUILD)/host_io.o

ab: $(AB_LIB)

# Register / occupancy report for every kernel instantiation.
resources: $(CSRC)/rns_checksum.hip
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o /dev/null -Rpass-analysis=kernel-resource-usage

asm: $(CSRC)/rns_checksum.hip
	@mkdir -p $(BUILD)/asm
	cd $(BUILD)/asm && $(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -I../../../include -c ../../../$< -o rns.o -save-temps

clean:
	rm -rf $(BUILD) $(LIB) $(CABI_TEST)
	$(MAKE) -C oracle clean

.PHONY: all oracle resources asm clean ab
