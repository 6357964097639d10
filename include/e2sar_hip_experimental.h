/*
 * e2sar_hip_experimental.h -- launch forms of the device-local round trip that measured no
 * gain on any BASELINE configuration, kept for A/B runs only.  They are
 * compiled into the library only with -DE2SAR_HIP_EXPERIMENTAL=1
 * (`make experimental` -> build/variants/lib_experimental.so, loaded with
 * E2SAR_HIP_LIB=...); the product library does not export them.
 *
 *  - XCD-matched groups (e2sar_hip_seg_groups / e2sar_hip_reassemble_groups): reading each
 *    datagram on the XCD that wrote it -- at parity with e2sar_hip_reassemble_batch
 *    (reas_kernel 74.8-75.3 vs 75.0-75.3 us per 205-event batch);
 *  - the chained form (e2sar_hip_segment_reassemble_batch(es)): segmentation and
 *    reassembly in one launch -- at parity or slower than the two launches (146.9 vs 145.0
 *    us per batch).
 */
#ifndef E2SAR_HIP_EXPERIMENTAL_H
#define E2SAR_HIP_EXPERIMENTAL_H

#include "e2sar_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device-local round trips (a batch this library segmented is reassembled on the same GPU:
 * loopback, relay, the device-resident benchmark).  e2sar_hip_segment_batch writes its
 * datagrams in XCD stripes (runs of about one reassembly group of consecutive datagrams,
 * all written on one of the eight XCDs); e2sar_hip_seg_groups returns, for the same planned
 * host event table (pktBase filled by e2sar_hip_seg_plan), maxPacketsPerEvent, maxPldLen and
 * stride, the reassembly groups that match them: group g = datagrams [starts[g],
 * starts[g+1]) of the batch (at most 64), starts[0..*nGroups], *nGroups + 1 <= cap.
 * *nGroups = 0 when the batch has no stripes (a group would exceed 64 datagrams).
 * e2sar_hip_reassemble_groups is e2sar_hip_reassemble_batch with those groups (d_starts:
 * the table copied to the device): workgroup g reassembles group g on the XCD that wrote
 * it.  Results are those of e2sar_hip_reassemble_batch for any group table that covers
 * [0, nPackets) in order; only the fused form takes groups (a batch above 320 MiB of slots,
 * or reference-order mode, is reassembled as e2sar_hip_reassemble_batch does).  The
 * datagrams' receive body is the same: e2sarDPReassembler.cpp:335-427. */
int e2sar_hip_seg_groups(const e2sar_hip_seg_event *events, uint32_t nEvents, uint32_t maxPacketsPerEvent,
                         uint32_t maxPldLen, uint32_t stride, uint32_t *starts, uint32_t cap, uint32_t *nGroups);
int e2sar_hip_reassemble_groups(e2sar_hip_reas *r, const uint8_t *d_packets, uint32_t stride,
                                const uint32_t *d_lens, uint32_t nPackets, const uint32_t *d_starts,
                                uint32_t nGroups, uint64_t now_ms, void *stream);

/* Chained round trip (BASELINE config 2's device-resident step) in ONE launch: segment
 * the batch (as e2sar_hip_segment_batch, d_lens required) and reassemble the same
 * nPackets datagrams into r (as e2sar_hip_reassemble_batch).  Reassembly workgroups start
 * as soon as the segmentation workgroups that write their datagrams have published them
 * (write-through stores + per-group agent-scope counters held by r), so the two stages
 * overlap at their seam instead of meeting at a kernel boundary.  Results are those of
 * the two calls in sequence.  nPackets = seg_plan's total; r created withLBHeader, not
 * REFERENCE_ORDER.  The first call for a larger nPackets allocates r's counters
 * (synchronous; outside graph capture).  A group whose datagrams never all arrive (a bad
 * descriptor table) stops waiting after 2 s and sets errorFlags bit 4.  Asynchronous.
 * Replaces _send (e2sarDPSegmenter.cpp:660-871) followed by the receive body
 * (e2sarDPReassembler.cpp:335-427) on the same events. */
int e2sar_hip_segment_reassemble_batch(e2sar_hip_ctx *ctx, const e2sar_hip_seg_event *d_events, uint32_t nEvents,
                                       uint32_t maxPacketsPerEvent, uint32_t nPackets, int lbHdrVersion,
                                       uint32_t maxPldLen, uint8_t *d_packets, uint32_t stride, uint32_t *d_lens,
                                       e2sar_hip_reas *r, uint64_t now_ms, void *stream);

/* Several batches (at most 8) chained in one launch: batch b's reassembly groups wait on
 * batch b's segmentation only, and batch b+1's segmentation starts while batch b's
 * reassembly finishes.  Each batch needs its own packet and length buffers.  Results are
 * those of the batches' segment_batch + reassemble_batch calls in order. */
typedef struct e2sar_hip_segreas_batch {
    const e2sar_hip_seg_event *d_events;   /* descriptors on the device, pktBase from seg_plan */
    uint8_t *d_packets;
    uint32_t *d_lens;
    uint32_t nEvents;
    uint32_t maxPacketsPerEvent;
    uint32_t nPackets;
    uint32_t reserved;
} e2sar_hip_segreas_batch;
int e2sar_hip_segment_reassemble_batches(e2sar_hip_ctx *ctx, const e2sar_hip_segreas_batch *batches,
                                         uint32_t nBatches, int lbHdrVersion, uint32_t maxPldLen, uint32_t stride,
                                         e2sar_hip_reas *r, uint64_t now_ms, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* E2SAR_HIP_EXPERIMENTAL_H */
