# Top-level build (no cmake needed): gcc for host C, hipcc for gfx950.
#
#   make            libhiphuff.so + HuffFramework CLI + oracle + test emulator
#   make lib        huffmandecoderongpus_amd/libhiphuff.so only
#
# Outputs stay in-tree (git-ignored) so they travel to the GPU box.

HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
CXX      ?= g++
ARCH     ?= gfx950
PKG      := huffmandecoderongpus_amd
CSRC     := $(PKG)/csrc
BUILD    := build
INC      := -Iinclude -I$(CSRC)
CFLAGS   := -O3 -fPIC -Wall -Wextra -std=gnu11 $(INC)
HIPFLAGS := $(HIPEXTRA) -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-result -Wno-unused-value \
            -Wno-comment $(INC)

LIB      := $(PKG)/libhiphuff.so
CLI      := $(BUILD)/HuffFramework
EMU      := tests/emu/libhh_emu.so

all: lib cli oracle emu ubench

lib: $(LIB)
cli: $(CLI)
emu: $(EMU)

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/hh_huff.o: $(CSRC)/hh_huff.c $(CSRC)/hh_internal.h $(CSRC)/hh_fsm.h include/hiphuff.h | $(BUILD)
	$(CC) $(CFLAGS) -c $< -o $@

$(BUILD)/hh_plugin.o: $(CSRC)/hh_plugin.c include/hiphuff.h include/hiphuff_plugin.h | $(BUILD)
	$(CC) $(CFLAGS) -c $< -o $@

$(BUILD)/hh_device.o: $(CSRC)/hh_device.hip $(CSRC)/hh_algo.h $(CSRC)/hh_internal.h $(CSRC)/hh_fsm_dev.h \
                      $(CSRC)/hh_fsm.h $(CSRC)/hh_fsm_algo.h include/hiphuff.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hh_one.o: $(CSRC)/hh_one.hip $(CSRC)/hh_fsm_kern.h $(CSRC)/hh_fsm_dev.h $(CSRC)/hh_fsm.h $(CSRC)/hh_fsm_algo.h \
                   $(CSRC)/hh_internal.h include/hiphuff.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hh_fsm.o: $(CSRC)/hh_fsm.hip $(CSRC)/hh_fsm_kern.h $(CSRC)/hh_fsm_dev.h $(CSRC)/hh_fsm.h $(CSRC)/hh_fsm_algo.h \
                   $(CSRC)/hh_internal.h include/hiphuff.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hh_encode.o: $(CSRC)/hh_encode.hip $(CSRC)/hh_internal.h include/hiphuff.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hh_probe.o: $(CSRC)/hh_probe.hip include/hiphuff.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(BUILD)/hh_device.o $(BUILD)/hh_fsm.o $(BUILD)/hh_one.o $(BUILD)/hh_encode.o $(BUILD)/hh_probe.o $(BUILD)/hh_huff.o $(BUILD)/hh_plugin.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

$(CLI): $(PKG)/host/hh_cli.c $(LIB) include/hiphuff.h include/hiphuff_plugin.h
	$(CC) -O2 -Wall -Wextra -std=gnu11 $(INC) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $@ $< -L$(PKG) -lhiphuff \
	    -Wl,-rpath,'$$ORIGIN/../$(PKG)' -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lm

oracle:
	$(MAKE) -C oracle

# microbenchmarks the profiling scripts run (tools/profile.sh: FETCH_SIZE
# calibration on known byte counts)
ubench: $(BUILD)/ub_fetch
$(BUILD)/ub_fetch: tools/ubench/ub_fetch.hip | $(BUILD)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

$(EMU): tests/emu/hh_emu.cpp tests/emu/hh_fsm_emu.cpp $(CSRC)/hh_algo.h $(CSRC)/hh_fsm_algo.h $(CSRC)/hh_fsm.h $(CSRC)/hh_internal.h $(BUILD)/hh_huff.o
	$(CXX) -O2 -fPIC -shared $(INC) -Wno-comment -o $@ tests/emu/hh_emu.cpp tests/emu/hh_fsm_emu.cpp $(BUILD)/hh_huff.o

clean:
	rm -rf $(BUILD) $(LIB) $(EMU)
	$(MAKE) -C oracle clean

.PHONY: all lib cli emu oracle ubench clean

# A/B variant of the library: make variant V=name HIPEXTRA="-DHH_X=1"
# -> build/libhiphuff_<name>.so (tools/ab.sh)
variant: $(BUILD)/hh_plugin.o $(BUILD)/hh_encode.o $(BUILD)/hh_probe.o
	$(HIPCC) $(HIPFLAGS) -c $(CSRC)/hh_device.hip -o $(BUILD)/hh_device_$(V).o
	$(HIPCC) $(HIPFLAGS) -c $(CSRC)/hh_fsm.hip -o $(BUILD)/hh_fsm_$(V).o
	$(HIPCC) $(HIPFLAGS) -c $(CSRC)/hh_one.hip -o $(BUILD)/hh_one_$(V).o
	$(CC) $(CFLAGS) $(HIPEXTRA) -c $(CSRC)/hh_huff.c -o $(BUILD)/hh_huff_$(V).o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(BUILD)/libhiphuff_$(V).so $(BUILD)/hh_device_$(V).o \
	    $(BUILD)/hh_fsm_$(V).o $(BUILD)/hh_one_$(V).o $(BUILD)/hh_huff_$(V).o $^
.PHONY: variant
