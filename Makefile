# Top-level build: the product library (gfx950 HIP + host C++) and the test oracle.
#   make            -> ray-tracing-project_amd/lib/librtamd.so, oracle/build/liboracle.so, CLI
# Float semantics: -ffp-contract=off everywhere (no FMA contraction; the reference rounds every op),
# hipcc's default correctly rounded fp32 division / sqrt kept, no fast-math. -fno-slp-vectorize: the
# SLP packing into v_pk_*_f32 costs more in lane shuffles than it saves here (measured -6% trace time).
PKG      := ray-tracing-project_amd
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
HIPFLAGS := -O3 --offload-arch=$(ARCH) -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
            -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable
CXXFLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function
OBJ      := $(PKG)/build
LIB      := $(PKG)/lib/librtamd.so
HDRS     := include/rt/rt_api.h $(wildcard $(PKG)/csrc/*.h)
# source hash embedded in the library (rt_source_hash(); rtamd.source_hash() recomputes it from the tree)
SRCS     := $(sort $(wildcard $(PKG)/csrc/*.hip $(PKG)/csrc/*.cpp $(PKG)/csrc/*.h) include/rt/rt_api.h)
SRC_HASH := $(shell cat $(SRCS) | sha256sum | cut -c1-16)
VERSION_H := $(OBJ)/rt_version.h
# rewritten only when the hash changes, so unchanged sources do not relink
$(shell mkdir -p $(OBJ) && echo '#define RT_SOURCE_HASH "$(SRC_HASH)"' > $(VERSION_H).new && \
        (cmp -s $(VERSION_H).new $(VERSION_H) || cp $(VERSION_H).new $(VERSION_H)); rm -f $(VERSION_H).new)

all: $(LIB) variants oracle cli

$(OBJ)/rt_device.o: $(PKG)/csrc/rt_device.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/rt_host.o: $(PKG)/csrc/rt_host.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/rt_variants.o: $(PKG)/csrc/rt_variants.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/rt_build.o: $(PKG)/csrc/rt_build.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -Wno-unused-result -c $< -o $@

$(OBJ)/rt_boxes.o: $(PKG)/csrc/rt_boxes.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/rt_version.o: $(PKG)/csrc/rt_version.cpp $(VERSION_H) include/rt/rt_api.h
	$(CXX) $(CXXFLAGS) -I$(OBJ) -c $< -o $@

$(OBJ)/rt_cache.o: $(PKG)/csrc/rt_cache.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

PRODUCT_OBJS := $(OBJ)/rt_device.o $(OBJ)/rt_host.o $(OBJ)/rt_cache.o $(OBJ)/rt_build.o $(OBJ)/rt_boxes.o $(OBJ)/rt_version.o
$(LIB): $(PRODUCT_OBJS)
	@mkdir -p $(PKG)/lib
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread

# the A/B kernel variants (rt_variants.hip) linked beside the product objects: the same library plus the
# measured alternatives, for tests/test_gpu_parity.py's variant check and A/B timing (RTAMD_LIB)
VARLIB := $(PKG)/lib/librtamd_variants.so
variants: $(VARLIB)
$(VARLIB): $(PRODUCT_OBJS) $(OBJ)/rt_variants.o
	@mkdir -p $(PKG)/lib
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread

# A/B builds of the same sources with extra device flags (experiments only):
#   make ablib TAG=noslp EXTRA="-fno-slp-vectorize"  ->  lib/librtamd_noslp.so  (select with RTAMD_LIB)
ablib: $(PKG)/csrc/rt_device.hip $(HDRS) $(OBJ)/rt_host.o $(OBJ)/rt_cache.o $(OBJ)/rt_build.o $(OBJ)/rt_boxes.o $(OBJ)/rt_version.o
	@mkdir -p $(OBJ) $(PKG)/lib
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $< -o $(OBJ)/rt_device_$(TAG).o
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $(PKG)/csrc/rt_variants.hip -o $(OBJ)/rt_variants_$(TAG).o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(PKG)/lib/librtamd_$(TAG).so $(OBJ)/rt_device_$(TAG).o $(OBJ)/rt_variants_$(TAG).o $(OBJ)/rt_host.o $(OBJ)/rt_cache.o $(OBJ)/rt_build.o $(OBJ)/rt_boxes.o $(OBJ)/rt_version.o -lpthread

# debug build of the same sources with every scalar prefetch offset checked on the device (RT_CHECK_PREFETCH:
# an out-of-range offset is recorded and fails the next rt_synchronize) -> lib/librtamd_pfcheck.so,
# run the GPU suite against it with RTAMD_LIB
pfcheck:
	$(MAKE) ablib TAG=pfcheck EXTRA=-DRT_CHECK_PREFETCH=1

cli: $(PKG)/lib/rt_render_cli

$(PKG)/lib/rt_render_cli: $(PKG)/host/main.cpp $(PKG)/host/flyscene.cpp $(PKG)/host/flyscene.hpp $(LIB)
	$(CXX) $(CXXFLAGS) -Iinclude -o $@ $(PKG)/host/main.cpp $(PKG)/host/flyscene.cpp \
	    -L$(PKG)/lib -lrtamd -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

asm: $(PKG)/csrc/rt_device.hip $(HDRS)
	@mkdir -p $(OBJ)/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o $(OBJ)/asm/rt_device.s $<
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -c -Rpass-analysis=kernel-resource-usage -o /dev/null $< 2> $(OBJ)/asm/resource.txt || true

clean:
	rm -rf $(OBJ) $(PKG)/lib
	$(MAKE) -C oracle clean

.PHONY: ablib all variants oracle cli asm clean pfcheck
