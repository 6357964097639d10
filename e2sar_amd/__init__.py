"""e2sar_amd -- MI355X-native (gfx950) implementation of E2SAR's data-plane SAR path.

Segmentation (reference src/e2sarDPSegmenter.cpp) and reassembly
(src/e2sarDPReassembler.cpp) run as hand-written HIP kernels behind the C ABI in
include/e2sar_hip.h.  Submodules:

  _capi      ctypes binding of the C ABI (loads e2sar_amd/lib/libe2sar_hip.so)
  sar        device-level batch API (DeviceSegmenter / DeviceReassembler)
  dist       multi-GPU routing (PacketRouter) and the all-to-all-v exchange
  e2sar_py   pybind module with the reference's e2sar_py names (DataPlane.Segmenter /
             Reassembler, header classes REHdr / LBHdrV2 / LBHdrV3 / SyncHdr, EjfatURI),
             built from csrc/host/py_e2sar.cpp over the C++ facade
"""

__version__ = "0.1.0"
