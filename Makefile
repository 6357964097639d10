# Build of the MI355X (gfx950) SAR path.  No cmake: hipcc + g++ only.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
INC := -Iinclude -Ie2sar_amd/csrc
LIBDIR := e2sar_amd/lib

HIP_SRCS := e2sar_amd/csrc/sar_kernels.hip e2sar_amd/csrc/capi.cpp
HIP_HDRS := include/e2sar_hip.h e2sar_amd/csrc/sar_kernels.hpp e2sar_amd/csrc/wire.hpp

all: $(LIBDIR)/libe2sar_hip.so oracle

$(LIBDIR)/libe2sar_hip.so: $(HIP_SRCS) $(HIP_HDRS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(INC) -shared -o $@ $(HIP_SRCS)

oracle:
	$(MAKE) -C oracle

# A/B-only launch forms (include/e2sar_hip_experimental.h) in a library of their own;
# run with E2SAR_HIP_LIB=build/variants/lib_experimental.so
experimental: build/variants/lib_experimental.so

build/variants/lib_experimental.so: $(HIP_SRCS) $(HIP_HDRS) include/e2sar_hip_experimental.h
	@mkdir -p build/variants
	$(HIPCC) $(HIPFLAGS) -DE2SAR_HIP_EXPERIMENTAL=1 $(INC) -shared -o $@ $(HIP_SRCS)

clean:
	rm -rf $(LIBDIR) e2sar_amd/csrc/*.o
	$(MAKE) -C oracle clean

.PHONY: all oracle clean experimental

# ---- reference-shaped C++ facade (pure C++ over the C ABI) ----
CXX ?= g++
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HOST_SRCS := e2sar_amd/csrc/host/util.cpp e2sar_amd/csrc/host/segmenter.cpp e2sar_amd/csrc/host/reassembler.cpp
HOST_HDRS := include/e2sar_amd/e2sar.hpp e2sar_amd/csrc/host/host_common.hpp include/e2sar_hip.h

$(LIBDIR)/libe2sar_amd.so: $(HOST_SRCS) $(HOST_HDRS) $(LIBDIR)/libe2sar_hip.so
	$(CXX) $(CXXFLAGS) -Iinclude -Ie2sar_amd/csrc/host -shared -o $@ $(HOST_SRCS) \
		-L$(LIBDIR) -le2sar_hip -Wl,-rpath,'$$ORIGIN' -lpthread

all: $(LIBDIR)/libe2sar_amd.so

# ---- e2sar_py: the reference's Python module surface, over the C++ facade ----
PYEXT := $(shell python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC := $(shell python3 -c "import sysconfig,pybind11;print('-I'+sysconfig.get_paths()['include'],'-I'+pybind11.get_include())")

e2sar_amd/e2sar_py$(PYEXT): e2sar_amd/csrc/host/py_e2sar.cpp $(HOST_HDRS) include/e2sar_amd/e2sarHeaders.hpp $(LIBDIR)/libe2sar_amd.so
	$(CXX) $(CXXFLAGS) -fvisibility=hidden $(PYINC) -Iinclude -shared -o $@ e2sar_amd/csrc/host/py_e2sar.cpp \
		-L$(LIBDIR) -le2sar_amd -le2sar_hip -Wl,-rpath,'$$ORIGIN/lib'

all: e2sar_amd/e2sar_py$(PYEXT)

# ---- e2sar_perf-shaped tool over the C++ facade ----
build/e2sar_perf: tools/e2sar_perf.cpp $(HOST_HDRS) include/e2sar_amd/e2sarHeaders.hpp $(LIBDIR)/libe2sar_amd.so
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -Iinclude -o $@ tools/e2sar_perf.cpp -L$(LIBDIR) -le2sar_amd -le2sar_hip \
		-Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

all: build/e2sar_perf

# ---- e2sar_ft-shaped file transfer tool over the C++ facade ----
build/e2sar_ft: tools/e2sar_ft.cpp $(HOST_HDRS) $(LIBDIR)/libe2sar_amd.so
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -Iinclude -o $@ tools/e2sar_ft.cpp -L$(LIBDIR) -le2sar_amd -le2sar_hip \
		-Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

all: build/e2sar_ft
