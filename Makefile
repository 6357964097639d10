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

clean:
	rm -rf $(LIBDIR) e2sar_amd/csrc/*.o
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
