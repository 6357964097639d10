// host_common.hpp -- internal helpers shared by the Segmenter/Reassembler façade.
#pragma once

#include <atomic>
#include <chrono>
#include <map>
#include <string>

#include "e2sar_amd/e2sar.hpp"
#include "e2sar_hip.h"

namespace e2sar {
namespace detail {

bool read_ini(const std::string &path, std::map<std::string, std::string> &out, std::string &err);
bool ini_bool(const std::map<std::string, std::string> &m, const std::string &k, bool def);
double ini_num(const std::map<std::string, std::string> &m, const std::string &k, double def);

// C-ABI status -> E2SARErrorInfo (status = -(E2SARErrorc))
inline E2SARErrorInfo hip_error(int rc, const std::string &what)
{
    return E2SARErrorInfo{static_cast<E2SARErrorc>(-rc), what + ": " + e2sar_hip_last_error()};
}

inline uint64_t now_us()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

// clockEntropyTest (e2sarUtil.hpp:549-574): Shannon entropy, in bits, of the low 8 bits of
// the microsecond wall clock sampled every sleepMs; measured once per process (the clock
// does not change under it) -- the reference measures it in every Segmenter constructor
float clock_entropy_bits();

// Segmenter MTU rules (segmenter.cpp): interface/override resolution and the 9000-byte limit
uint32_t resolve_mtu(uint16_t flagsMtu, uint32_t ifMtu, const std::string &iface);
void check_mtu_limit(uint32_t mtu);
EventNum_t take_send_number(std::atomic<EventNum_t> &userEventNum, EventNum_t eventNum, size_t depth, size_t cap,
                            bool *accepted);

inline uint64_t steady_ms()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace detail
}  // namespace e2sar
