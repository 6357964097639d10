/*
 * e2sar_oracle.h -- CPU restatement of the E2SAR segmentation/reassembly (SAR) path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (e2sar_amd/csrc).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product never links or calls it.
 *
 * It restates, in plain C, the reference algorithm at JeffersonLab/E2SAR v0.3.2:
 *   - wire headers            include/e2sarHeaders.hpp:21-102 (REHdr), :111-184 (LBHdrV2),
 *                              :191-274 (LBHdrV3), :278-315 (LBHdrU/LBREHdr), :406-421 (lengths)
 *   - segmentation loop       src/e2sarDPSegmenter.cpp:660-871 (SendThreadState::_send)
 *   - reassembly body         src/e2sarDPReassembler.cpp:310-428 (RecvThreadState::_threadBody)
 *   - event queue / getEvent  include/e2sarDPReassembler.hpp:132-161, src/e2sarDPReassembler.cpp:626-641
 *   - lost-event log / GC     include/e2sarDPReassembler.hpp:262-279, src/e2sarDPReassembler.cpp:236-291
 *
 * Parity pinning: the reference's C++ engines need Boost >= 1.89 and gRPC (absent in
 * this image) and its header needs <boost/tuple/tuple.hpp> (absent), so the reference
 * is unbuildable here.  This restatement is pinned by the reference's own known answers
 * (packet counts in test/e2sar_seg_test.cpp / test/e2sar_reas_test.cpp, header sizes in
 * test/boost_test.cpp:171-179, field round trips in test/mem_tests.cpp:93-127, content
 * equality in test/py_test/test_b2b_DP.py, the frame-count KAT in
 * scripts/bash-helpers/README.md:95-101) and the header hex KATs in SURVEY.md §8(a);
 * see tests/test_oracle_golden.py.
 */
#ifndef E2SAR_ORACLE_H
#define E2SAR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- header geometry (e2sarHeaders.hpp:406-421) ---- */
size_t e2o_total_hdr_len(int useIPv6);
size_t e2o_max_pld_len(unsigned mtu, int useIPv6);
size_t e2o_num_packets(size_t bytes, size_t maxPldLen);

/* ---- header pack / parse ---- */
/* 36-byte LB+RE header exactly as _send fills it (e2sarDPSegmenter.cpp:736-755). */
void e2o_lbre_hdr(uint8_t out[36], int lbHdrVersion, uint16_t entropy, uint64_t lbTick,
                  uint16_t dataId, uint32_t bufferOffset, uint32_t bufferLength,
                  uint64_t eventNum);
/* REHdr getters + validate() (e2sarHeaders.hpp:43-101).  Returns validate(). */
int e2o_re_parse(const uint8_t re[20], uint16_t *dataId, uint32_t *bufferOffset,
                 uint32_t *bufferLength, uint64_t *eventNum, uint8_t *version);

/* ---- segmentation (e2sarDPSegmenter.cpp:660-871 minus the socket) ----
 * Writes ceil(bytes/maxPldLen) datagrams [36-byte hdr][payload] into out at
 * packet stride `stride` (bytes past each datagram, up to the stride, are zeroed)
 * and their lengths into lens.  Returns the packet count. */
size_t e2o_segment_event(const uint8_t *event, size_t bytes, uint64_t eventNum,
                         uint16_t dataId, uint16_t entropy, uint64_t lbTick,
                         int lbHdrVersion, size_t maxPldLen,
                         uint8_t *out, size_t stride, uint32_t *lens);

/* ---- reassembly (e2sarDPReassembler.cpp:310-428) ---- */
typedef struct e2o_reas e2o_reas;

typedef struct e2o_reas_stats {
    uint64_t enqueueLoss;        /* hpp:103 */
    uint64_t reassemblyLoss;     /* hpp:104 */
    uint64_t eventSuccess;       /* hpp:105 */
    uint64_t totalBytes;         /* hpp:106 */
    uint64_t totalPackets;       /* hpp:107 */
    uint64_t badHeaderDiscards;  /* hpp:108 */
    uint64_t dataErrCnt;         /* hpp:115 (also: bounds violations, see .c) */
    uint64_t inProgress;         /* size of eventsInProgress */
} e2o_reas_stats;

/* queueCapacity 0 = the reference's unbounded eventQueue (hpp:126-127); nonzero models the
 * device's completed-record ring (a build parameter, not reference behaviour) */
e2o_reas *e2o_reas_new(int withLBHeader, size_t queueCapacity);
void e2o_reas_free(e2o_reas *r);
/* logical clock (ms) used for firstSegment / GC (stands in for steady_clock) */
void e2o_reas_set_time(e2o_reas *r, uint64_t now_ms);
/* one received datagram */
void e2o_reas_push(e2o_reas *r, const uint8_t *dgram, size_t nbytes);
/* n datagrams at a fixed stride, in array order (a recv loop over a packet ring) */
void e2o_reas_push_batch(e2o_reas *r, const uint8_t *pkts, size_t n, size_t stride,
                         const uint32_t *lens);
/* getEvent into a caller buffer: returns bytes (>=0), -1 empty, -2 buffer too small */
long long e2o_reas_pop_into(e2o_reas *r, uint8_t *buf, size_t cap, uint64_t *eventNum,
                            uint16_t *dataId);
/* getEvent: 0 on success (caller frees *event with e2o_free), -1 if queue empty */
int e2o_reas_pop(e2o_reas *r, uint8_t **event, size_t *bytes, uint64_t *eventNum,
                 uint16_t *dataId);
/* GC pass: drop in-progress events older than timeout_ms (cpp:236-291) */
size_t e2o_reas_gc(e2o_reas *r, uint64_t timeout_ms);
/* get_LostEvent: 0 on success, -1 if empty (hpp:593-604) */
int e2o_reas_lost_pop(e2o_reas *r, uint64_t *eventNum, uint16_t *dataId, uint64_t *numFragments);
void e2o_reas_get_stats(const e2o_reas *r, e2o_reas_stats *out);
void e2o_free(void *p);

/* ---- batch helpers used by the CPU baseline (same byte formula as the GPU) ---- */
/* segment n equal-size events laid out contiguously (event i at events + i*bytes). */
size_t e2o_segment_batch(const uint8_t *events, size_t n, size_t bytes,
                         const uint64_t *eventNums, uint16_t dataId,
                         const uint16_t *entropies, const uint64_t *ticks,
                         int lbHdrVersion, size_t maxPldLen,
                         uint8_t *pkts, size_t stride, uint32_t *lens);

/* ---- CPU baseline timing (cpu_bench.c; bench.py's cpu_baseline leg only) ----
 * `threads` POSIX threads each segment + reassemble the nEvents-event sample until
 * `seconds` have passed; returns 0 with the payload bytes done and the wall time.
 * ringBytes: 0 = each thread reuses one datagram buffer and one event block (cache-resident);
 * > 0 = per-thread rings of at least ringBytes of datagrams and of live events (DRAM). */
int e2o_cpu_bench(const uint8_t *events, size_t nEvents, size_t bytes, int lbHdrVersion, size_t maxPldLen,
                  uint16_t dataId, int threads, double seconds, size_t ringBytes, uint64_t *bytesDone,
                  double *elapsed);

#ifdef __cplusplus
}
#endif
#endif
