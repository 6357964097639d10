"""e2sar_amd -- MI355X-native (gfx950) implementation of E2SAR's data-plane SAR path.

Segmentation (reference src/e2sarDPSegmenter.cpp) and reassembly
(src/e2sarDPReassembler.cpp) run as hand-written HIP kernels behind the C ABI in
include/e2sar_hip.h.  Submodules:

  _capi      ctypes binding of the C ABI (loads e2sar_amd/lib/libe2sar_hip.so)
  sar        device-level batch API (DeviceSegmenter / DeviceReassembler)
  headers    wire-format classes mirroring the reference pybind header bindings
"""

__version__ = "0.1.0"
