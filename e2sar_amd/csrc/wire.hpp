// wire.hpp -- LB+RE header words as the gfx950 kernels emit and parse them.
//
// The 36-byte LB+RE header (include/e2sarHeaders.hpp:302-315 in the reference) is
// handled as nine little-endian dwords so a lane can build or test any 16-byte chunk
// of a datagram in registers.  Field placement, big-endian encoding and the version
// dispatch follow:
//   LBHdrV2  e2sarHeaders.hpp:111-127   'L','B', version 2, nextProto 1, rsvd, entropy, tick
//   LBHdrV3  e2sarHeaders.hpp:191-208   'L','B', version 3, nextProto 1, slotSelect, portSelect, tick
//   LBHdrU   e2sarHeaders.hpp:287-297   any version other than 3 builds a v2 header
//   REHdr    e2sarHeaders.hpp:21-38     0x10, 0, dataId, bufferOffset, bufferLength, eventNum
//   _send    e2sarDPSegmenter.cpp:743-755 (v3 slotSelect = tick & 0xFFFF, portSelect = entropy)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace e2sar_amd {

constexpr uint32_t kLBHdrLen = 16;
constexpr uint32_t kREHdrLen = 20;
constexpr uint32_t kLBREHdrLen = 36;
constexpr uint32_t kREVersionNibble = 1u << 4;   // rehdrVersionNibble (e2sarHeaders.hpp:15)

__host__ __device__ inline uint32_t bswap32(uint32_t x)
{
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
__host__ __device__ inline uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// The nine header dwords.  w[0..3] = LB header, w[4..8] = RE header.
struct HdrWords {
    uint32_t w[9];
};

__host__ __device__ inline void lbre_words(HdrWords &h, int lbVersion, uint16_t entropy,
                                           uint64_t tick, uint16_t dataId, uint32_t off,
                                           uint32_t len, uint64_t eventNum)
{
    const bool v3 = (lbVersion == 3);
    h.w[0] = 0x4Cu | (0x42u << 8) | ((v3 ? 3u : 2u) << 16) | (1u << 24);
    h.w[1] = (v3 ? bswap16((uint32_t)(tick & 0xFFFFu)) : 0u) | (bswap16(entropy) << 16);
    h.w[2] = bswap32((uint32_t)(tick >> 32));
    h.w[3] = bswap32((uint32_t)tick);
    h.w[4] = kREVersionNibble | (bswap16(dataId) << 16);
    h.w[5] = bswap32(off);
    h.w[6] = bswap32(len);
    h.w[7] = bswap32((uint32_t)(eventNum >> 32));
    h.w[8] = bswap32((uint32_t)eventNum);
}

// REHdr::validate() (e2sarHeaders.hpp:98-101) on the first RE dword.
__host__ __device__ inline bool re_valid(uint32_t re0) { return (re0 & 0xFFFFu) == kREVersionNibble; }

}  // namespace e2sar_amd
