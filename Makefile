# Builds the MI355X (gfx950) engine in-tree:
#   openr_amd/lib/libopenr_gpu.so      HIP kernels + C-ABI (include/openr_gpu.h)
#   openr_amd/_decision*.so            C++ drop-in (LinkState/SpfSolver/...) +
#                                      pybind11 binding, linked to the above
#   oracle/_refcpu*.so                 CPU oracle (test infrastructure only)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
PY_INC := $(shell python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC := $(shell python3 -c "import pybind11;print(pybind11.get_include())")
EXT := $(shell python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

LIB := openr_amd/lib/libopenr_gpu.so
MOD := openr_amd/_decision$(EXT)
KERNELS := $(wildcard openr_amd/csrc/kernels/*.hip)
KERNEL_H := $(wildcard openr_amd/csrc/kernels/*.h)
HOST := $(wildcard openr_amd/csrc/host/*.cpp)
HOST_H := $(wildcard openr_amd/csrc/host/*.h) include/openr_gpu.h openr_amd/csrc/gen/topogen.h

CCONS := tests/c_consumer/spf_square

all: $(LIB) $(MOD) oracle $(CCONS)

# plain-C consumer of the C-ABI (tests/test_capi.py runs it)
$(CCONS): tests/c_consumer/spf_square.c include/openr_gpu.h $(LIB)
	gcc -std=c11 -O2 -Wall -Iinclude $< -o $@ -Lopenr_amd/lib -lopenr_gpu \
	  -Wl,-rpath,'$$ORIGIN/../../openr_amd/lib'


# one object per kernel translation unit (parallel make), then one link
KOBJ := $(patsubst openr_amd/csrc/kernels/%.hip,build/kernels/%.o,$(KERNELS))

# each object leaves its kernels' resource report (VGPRs, scratch, occupancy)
# in build/kernels/<tu>.ru; tools/kernel_resources.py lists the spills
build/kernels/%.o: openr_amd/csrc/kernels/%.hip $(KERNEL_H) include/openr_gpu.h
	@mkdir -p build/kernels
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -c $< -o $@ \
	  -Rpass-analysis=kernel-resource-usage 2> $@.ru || { cat $@.ru; rm -f $@; false; }

$(LIB): $(KOBJ)
	@mkdir -p openr_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared $(KOBJ) -o $@.tmp && mv -f $@.tmp $@

$(MOD): $(HOST) $(HOST_H) openr_amd/csrc/py/bindings.cpp $(LIB)
	$(CXX) -O2 -std=c++17 -fPIC -shared -Wall -Wno-unused-function \
	  -Iinclude -Iopenr_amd/csrc/host -I$(PY_INC) -I$(PYBIND_INC) \
	  $(HOST) openr_amd/csrc/py/bindings.cpp -o $@.tmp \
	  -Lopenr_amd/lib -lopenr_gpu -Wl,-rpath,'$$ORIGIN/lib' && mv -f $@.tmp $@

oracle:
	$(MAKE) -C oracle

# diagnostic build: per-unit phase clocks written into ogs_spf_out.sel
# (tools/stamps.py); never loaded by the product
STAMPS := openr_amd/lib/libopenr_gpu_stamps.so
stamps: $(STAMPS)
SOBJ := $(patsubst openr_amd/csrc/kernels/%.hip,build/stamps/%.o,$(KERNELS))
build/stamps/%.o: openr_amd/csrc/kernels/%.hip $(KERNEL_H) include/openr_gpu.h
	@mkdir -p build/stamps
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -DOGS_STAMPS -Iinclude -c $< -o $@
$(STAMPS): $(SOBJ)
	@mkdir -p openr_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared $(SOBJ) -o $@

# CPU sanitizer build (AddressSanitizer + UBSan) of the drop-in's host code
# (tests/asan/host_asan.cpp over a host-only C-ABI stub, no device) and of
# the oracle (build/asan/_refcpu, driven by tools/asan_oracle.py with libasan
# preloaded); `make asan` runs both and keeps the log in profiles/
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
ASAN_BIN := build/asan/host_asan
ASAN_REF := build/asan/_refcpu$(EXT)
ASAN_LOG ?= profiles/r06_asan.log
$(ASAN_BIN): $(HOST) $(HOST_H) tests/asan/host_asan.cpp tests/asan/ogs_stub.cpp
	@mkdir -p build/asan
	$(CXX) -std=c++17 $(SAN) -Wall -Wno-unused-function -Iinclude -Iopenr_amd/csrc/host \
	  $(HOST) tests/asan/host_asan.cpp tests/asan/ogs_stub.cpp -o $@ -lpthread
$(ASAN_REF): oracle/refcpu/refcpu.cpp oracle/refcpu/refcpu.h oracle/refcpu/bindings.cpp openr_amd/csrc/gen/topogen.h
	@mkdir -p build/asan
	$(CXX) -std=c++17 $(SAN) -fPIC -shared -I$(PY_INC) -I$(PYBIND_INC) \
	  oracle/refcpu/refcpu.cpp oracle/refcpu/bindings.cpp -o $@ -lpthread
asan: $(ASAN_BIN) $(ASAN_REF)
	{ echo "== host_asan (drop-in host code, ASan+UBSan)"; \
	  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 ./$(ASAN_BIN) && \
	  echo "== oracle (refcpu, ASan+UBSan, KATs + generated RouteDbs)" && \
	  LD_PRELOAD=$$($(CXX) -print-file-name=libasan.so):$$($(CXX) -print-file-name=libubsan.so) \
	  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 python3 tools/asan_oracle.py; } 2>&1 | tee $(ASAN_LOG)

clean:
	rm -f $(LIB) $(MOD) $(STAMPS) $(CCONS) $(KOBJ) $(SOBJ)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean stamps asan
