# Build of the MI355X-native simplex (gfx950 only) and its CPU oracle.
#   make            -> distributedlpsolver_amd/libdlp.so + oracle/liboracle.so
#   make ref        -> oracle/_ref/dlp_ref (reference built from its own sources; container only)
#   make asm        -> build/dlp_kernels-gfx950.s (ISA audit)
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PKG       := distributedlpsolver_amd
CSRC      := $(PKG)/csrc
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I$(CSRC) \
             -Wall -Wno-unused-function
LIBDLP    := $(PKG)/libdlp.so
OBJS      := build/dlp_kernels.o build/dlp_batched.o build/dlp_mw.o build/dlp_session.o build/dlp_adalloc.o \
             build/dlp_instance.o build/dlp_general.o build/dlp_defer.o build/dlp_cluster.o

all: $(LIBDLP) oracle tools

build:
	mkdir -p build

build/%.o: $(CSRC)/%.hip $(CSRC)/dlp_internal.h $(CSRC)/dlp_device.h include/dlp.h | build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/%.o: $(CSRC)/%.cpp $(CSRC)/dlp_internal.h $(CSRC)/dlp_host.h include/dlp.h include/distributed_solver/instance.h | build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDLP): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

asm: | build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $(CSRC)/dlp_kernels.hip -o build/dlp_kernels-gfx950.s

clean:
	rm -rf build $(LIBDLP)
	$(MAKE) -C oracle clean

.PHONY: all oracle ref asm clean

tools: build/hbm_ceiling build/fetch_calib build/chainlab

build/hbm_ceiling: tools/hbm_ceiling.hip | build
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

build/fetch_calib: tools/fetch_calib.hip | build
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

build/chainlab: tools/chainlab.hip | build
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -o $@ $<

.PHONY: tools
