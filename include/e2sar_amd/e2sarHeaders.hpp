// e2sarHeaders.hpp -- host-side wire-format structs of the SAR path.
//
// Same byte layout, field semantics and method names as the reference's
// include/e2sarHeaders.hpp:21-421 (REHdr, LBHdrV2, LBHdrV3, LBHdrU, LBREHdr, SyncHdr and
// the header-length helpers), written here without Boost: get_Fields() returns a
// std::tuple.  The gfx950 kernels build and parse the same 36-byte LB+RE header as nine
// little-endian dwords (e2sar_amd/csrc/wire.hpp); tests check both against the oracle.
#pragma once

#include <cstddef>
#include <cstdint>
#include <new>
#include <tuple>

namespace e2sar {

using EventNum_t = uint64_t;
using UnixTimeNano_t = uint64_t;
using EventRate_t = uint32_t;

namespace be {
inline uint16_t h16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }
inline uint32_t h32(uint32_t v) { return __builtin_bswap32(v); }
inline uint64_t h64(uint64_t v) { return __builtin_bswap64(v); }
}  // namespace be

constexpr uint8_t rehdrVersion = 1;
constexpr uint8_t rehdrVersionNibble = rehdrVersion << 4;

struct REHdr {
    const uint8_t preamble[2]{rehdrVersionNibble, 0};
    uint16_t dataId{0};
    uint32_t bufferOffset{0};
    uint32_t bufferLength{0};   // event length, not the length of this segment
    EventNum_t eventNum{0};

    void set(uint16_t data_id, uint32_t buff_off, uint32_t buff_len, EventNum_t event_num)
    {
        dataId = be::h16(data_id);
        bufferOffset = be::h32(buff_off);
        bufferLength = be::h32(buff_len);
        eventNum = be::h64(event_num);
    }
    EventNum_t get_eventNum() const { return be::h64(eventNum); }
    uint32_t get_bufferLength() const { return be::h32(bufferLength); }
    uint32_t get_bufferOffset() const { return be::h32(bufferOffset); }
    uint16_t get_dataId() const { return be::h16(dataId); }
    std::tuple<uint16_t, uint32_t, uint32_t, EventNum_t> get_Fields() const
    {
        return {get_dataId(), get_bufferOffset(), get_bufferLength(), get_eventNum()};
    }
    uint8_t get_HeaderVersion() const { return preamble[0] >> 4; }
    bool validate() const { return preamble[0] == rehdrVersionNibble && preamble[1] == 0; }
} __attribute__((__packed__));

constexpr uint8_t lbhdrVersion2 = 2;
constexpr uint8_t lbhdrVersion3 = 3;

struct LBHdrV2 {
    const char preamble[2]{'L', 'B'};
    uint8_t version{lbhdrVersion2};
    uint8_t nextProto{rehdrVersion};
    uint16_t rsvd{0};
    uint16_t entropy{0};
    EventNum_t eventNum{0};

    void set(uint16_t ent, EventNum_t event_num)
    {
        entropy = be::h16(ent);
        eventNum = be::h64(event_num);
    }
    uint8_t get_version() const { return version; }
    bool check_version() const { return version == lbhdrVersion2; }
    uint8_t get_nextProto() const { return nextProto; }
    uint16_t get_entropy() const { return be::h16(entropy); }
    EventNum_t get_eventNum() const { return be::h64(eventNum); }
    std::tuple<uint8_t, uint8_t, uint16_t, EventNum_t> get_Fields() const
    {
        return {version, nextProto, get_entropy(), get_eventNum()};
    }
} __attribute__((__packed__));

struct LBHdrV3 {
    const char preamble[2]{'L', 'B'};
    uint8_t version{lbhdrVersion3};
    uint8_t nextProto{rehdrVersion};
    uint16_t slotSelect{0};
    uint16_t portSelect{0};
    EventNum_t tick{0};

    void set(uint16_t slt, uint16_t prt, EventNum_t tk)
    {
        slotSelect = be::h16(slt);
        portSelect = be::h16(prt);
        tick = be::h64(tk);
    }
    uint8_t get_version() const { return version; }
    bool check_version() const { return version == lbhdrVersion3; }
    uint8_t get_nextProto() const { return nextProto; }
    uint16_t get_slotSelect() const { return be::h16(slotSelect); }
    uint16_t get_portSelect() const { return be::h16(portSelect); }
    EventNum_t get_tick() const { return be::h64(tick); }
    std::tuple<uint8_t, uint8_t, uint16_t, uint16_t, EventNum_t> get_Fields() const
    {
        return {version, nextProto, get_slotSelect(), get_portSelect(), get_tick()};
    }
} __attribute__((__packed__));

union LBHdrU {
    LBHdrV2 lb2;
    LBHdrV3 lb3;
    LBHdrU() {}
    explicit LBHdrU(uint8_t ver)
    {
        if (ver == 3) new (this) LBHdrV3();
        else new (this) LBHdrV2();   // any other version builds v2 (reference :289-293)
    }
} __attribute__((__packed__));

struct LBREHdr {
    LBHdrU lbu;
    REHdr re;
    LBREHdr() : lbu(lbhdrVersion2), re() {}
    explicit LBREHdr(uint8_t ver) : lbu(ver), re() {}
} __attribute__((__packed__));

constexpr uint8_t synchdrVersion2 = 2;

struct SyncHdr {
    const char preamble[2]{'L', 'C'};
    uint8_t version{synchdrVersion2};
    uint8_t rsvd{0};
    uint32_t eventSrcId{0};
    EventNum_t eventNumber{0};
    EventRate_t avgEventRateHz{0};
    UnixTimeNano_t unixTimeNano{0};

    void set(uint32_t esid, EventNum_t event_num, EventRate_t avg_rate, UnixTimeNano_t ut)
    {
        eventSrcId = be::h32(esid);
        eventNumber = be::h64(event_num);
        avgEventRateHz = be::h32(avg_rate);
        unixTimeNano = be::h64(ut);
    }
    uint8_t get_version() const { return version; }
    bool check_version() const { return version == synchdrVersion2; }
    uint32_t get_eventSrcId() const { return be::h32(eventSrcId); }
    EventNum_t get_eventNumber() const { return be::h64(eventNumber); }
    uint32_t get_avgEventRateHz() const { return be::h32(avgEventRateHz); }
    UnixTimeNano_t get_unixTimeNano() const { return be::h64(unixTimeNano); }
    std::tuple<uint32_t, EventNum_t, uint32_t, UnixTimeNano_t> get_Fields() const
    {
        return {get_eventSrcId(), get_eventNumber(), get_avgEventRateHz(), get_unixTimeNano()};
    }
} __attribute__((__packed__));

static_assert(sizeof(REHdr) == 20, "REHdr is 20 bytes");
static_assert(sizeof(LBHdrV2) == 16 && sizeof(LBHdrV3) == 16, "LB headers are 16 bytes");
static_assert(sizeof(LBREHdr) == 36, "LB+RE is 36 bytes");
static_assert(sizeof(SyncHdr) == 28, "SyncHdr is 28 bytes");

constexpr size_t IPV4_HDRLEN = 20;
constexpr size_t IPV6_HDRLEN = 40;
constexpr size_t UDP_HDRLEN = 8;
constexpr size_t IP_HDRLEN = IPV4_HDRLEN;
constexpr size_t TOTAL_HDR_LEN{IP_HDRLEN + UDP_HDRLEN + sizeof(LBHdrV2) + sizeof(REHdr)};

inline constexpr size_t getIPHeaderLength(bool useIPv6) { return useIPv6 ? IPV6_HDRLEN : IPV4_HDRLEN; }
inline constexpr size_t getTotalHeaderLength(bool useIPv6)
{
    return getIPHeaderLength(useIPv6) + UDP_HDRLEN + sizeof(LBHdrV2) + sizeof(REHdr);
}

}  // namespace e2sar
