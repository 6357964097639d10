// ro_sort.hip -- the key sort of the reference-order reassembly mode (rocPRIM radix sort),
// in a translation unit of its own so the rocPRIM templates do not slow the main build.
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include "sar_kernels.hpp"

namespace e2sar_amd {

hipError_t ro_sort_keys(void *temp, size_t &tempBytes, const unsigned long long *in, unsigned long long *out,
                        uint32_t n, unsigned endBit, hipStream_t stream)
{
    // keys are slot << 32 | position and arrive in position order; the radix sort is stable,
    // so sorting the slot bits alone (32 .. endBit) keeps each slot's positions in order.
    // rocPRIM sorts inputs of up to 1M items by block sorts and merge passes (9 launches,
    // ~56 us per 150K-datagram batch); its onesweep form is a histogram and two passes over
    // 14 bits, but on gfx950 it resets an ordered-block-id counter with a 4-byte
    // hipMemsetAsync before each pass, and a HIP graph holding it faulted on replay
    // (DESIGN 4.4).  So onesweep outside graph capture (162.4 instead of 179.5 us per
    // 205-event batch, bit-exact over the reference-order suite and 100 random seeds) and
    // the merge-sort form inside it.  E2SAR_RO_ONESWEEP: 0 never, 1 outside capture
    // (default), 2 always (A/B only).
    using Merge = rocprim::radix_sort_config<>;
    using Onesweep = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;
    static const int onesweep = [] {      // 0 never, 1 outside capture, 2 always (A/B only)
        const char *v = getenv("E2SAR_RO_ONESWEEP");
        return v ? atoi(v) : 1;
    }();
    if (!temp) {            // size query: room for either form
        size_t a = 0, b = 0;
        hipError_t e = rocprim::radix_sort_keys<Merge>(nullptr, a, in, out, (size_t)n, 32u, endBit, stream);
        if (e == hipSuccess) e = rocprim::radix_sort_keys<Onesweep>(nullptr, b, in, out, (size_t)n, 32u, endBit, stream);
        tempBytes = a > b ? a : b;
        return e;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (onesweep == 2 ||
        (onesweep == 1 && hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone))
        return rocprim::radix_sort_keys<Onesweep>(temp, tempBytes, in, out, (size_t)n, 32u, endBit, stream);
    return rocprim::radix_sort_keys<Merge>(temp, tempBytes, in, out, (size_t)n, 32u, endBit, stream);
}

size_t ro_scratch_bytes(uint32_t n, uint32_t tableSlots)
{
    size_t tb = 0;
    if (ro_sort_keys(nullptr, tb, nullptr, nullptr, n, ro_sort_end_bit(tableSlots), nullptr) != hipSuccess) return 0;
    return ro_fixed_bytes(n) + ro_align(tb);
}

}  // namespace e2sar_amd
