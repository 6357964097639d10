/*
 * cpu_bench.c -- timing driver for bench.py's cpu_baseline leg.  TEST INFRASTRUCTURE /
 * BASELINE ONLY: never linked by the product.
 *
 * T POSIX threads each run the oracle's SAR path (e2sar_oracle.c: _send's fragment loop,
 * then the receive body into a fresh event handed out as getEvent does and freed, as
 * bin/e2sar_perf.cpp:299 frees it) over a shared sample of events until a deadline, so a
 * run on every host core is not bounded by Python's interpreter lock.  The reference's own
 * parallelism is the same shape: a pool of send threads (e2sarDPSegmenter.cpp:380) and
 * one receive thread per port (e2sarDPReassembler.cpp:415), each on its own events.
 *
 * Working set.  ringBytes == 0 is the cache-resident form: each thread reuses one datagram
 * buffer, and each reassembled event is freed before the next is allocated, so malloc
 * hands the same 1 MiB block back every time -- only the shared event sample streams from
 * DRAM.  ringBytes > 0 streams everything: each thread segments into a ring of datagram
 * buffers of at least ringBytes and keeps its last ringBytes of reassembled events alive
 * (freed first-in first-out, as a consumer that holds events a while frees them), so no
 * datagram or event byte is still in a cache when it is touched again.
 */
#define _POSIX_C_SOURCE 200809L
#include "e2sar_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <time.h>

typedef struct {
    const uint8_t *events;
    size_t nEvents, bytes, maxPld, stride, npk;
    int lbVer;
    uint16_t dataId;
    double deadline;
    size_t ringBytes;           /* 0: cache-resident form; else per-thread datagram / event rings */
    uint64_t done;              /* payload bytes segmented + reassembled */
    int bad;
} job;

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void *worker(void *arg)
{
    job *j = (job *)arg;
    const size_t pkBytes = j->npk * j->stride;
    /* datagram ring slots and events kept alive: enough of each to cover ringBytes */
    const size_t nPk = j->ringBytes ? (j->ringBytes + pkBytes - 1) / pkBytes : 1;
    const size_t nKeep = j->ringBytes ? (j->ringBytes + j->bytes - 1) / j->bytes : 0;
    uint8_t *pk = (uint8_t *)malloc(nPk * pkBytes);
    uint32_t *ln = (uint32_t *)malloc(j->npk * sizeof(uint32_t));
    uint8_t **keep = (uint8_t **)calloc(nKeep ? nKeep : 1, sizeof(uint8_t *));
    if (!pk || !ln || !keep) {
        j->bad = 1;
        free(pk);
        free(ln);
        free(keep);
        return NULL;
    }
    size_t slot = 0, kept = 0;
    do {
        e2o_reas *r = e2o_reas_new(1, 1u << 20);
        for (size_t i = 0; i < j->nEvents; i++) {
            uint8_t *out = pk + (slot % nPk) * pkBytes;
            slot++;
            /* the same event metadata as tests/sar_inputs.py (entropy, tick) */
            const size_t n = e2o_segment_event(j->events + i * j->bytes, j->bytes, i, j->dataId,
                                               (uint16_t)(1 + (i * 0x9E37u) % 65535u),
                                               0x0001000000000000ull + i, j->lbVer, j->maxPld, out,
                                               j->stride, ln);
            e2o_reas_push_batch(r, out, n, j->stride, ln);
            uint8_t *ev = NULL;
            size_t nb = 0;
            uint64_t en = 0;
            uint16_t di = 0;
            if (e2o_reas_pop(r, &ev, &nb, &en, &di) != 0 || nb != j->bytes) j->bad = 1;
            if (nKeep) {                   /* hold the last nKeep events, free the oldest */
                e2o_free(keep[kept % nKeep]);
                keep[kept % nKeep] = ev;
                kept++;
            } else {
                e2o_free(ev);
            }
        }
        j->done += (uint64_t)j->nEvents * j->bytes;
        e2o_reas_free(r);
    } while (now_s() < j->deadline && !j->bad);
    for (size_t k = 0; k < nKeep; k++) e2o_free(keep[k]);
    free(keep);
    free(pk);
    free(ln);
    return NULL;
}

/* Run `threads` workers for `seconds` over nEvents events of `bytes` each (contiguous at
 * `events`), each thread with the working set ringBytes chooses (above).  Returns 0 and the
 * payload bytes done and the wall time, or -1 on a failed thread start / allocation /
 * round trip. */
int e2o_cpu_bench(const uint8_t *events, size_t nEvents, size_t bytes, int lbHdrVersion, size_t maxPldLen,
                  uint16_t dataId, int threads, double seconds, size_t ringBytes, uint64_t *bytesDone,
                  double *elapsed)
{
    if (threads < 1 || nEvents == 0 || maxPldLen == 0) return -1;
    job *jobs = (job *)calloc((size_t)threads, sizeof(job));
    pthread_t *ts = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !ts) {
        free(jobs);
        free(ts);
        return -1;
    }
    const size_t stride = (36 + maxPldLen + 15) / 16 * 16;
    const double t0 = now_s();
    int started = 0, rc = 0;
    for (int k = 0; k < threads; k++) {
        job *j = &jobs[k];
        j->events = events;
        j->nEvents = nEvents;
        j->bytes = bytes;
        j->maxPld = maxPldLen;
        j->stride = stride;
        j->npk = e2o_num_packets(bytes, maxPldLen);
        j->lbVer = lbHdrVersion;
        j->dataId = dataId;
        j->deadline = t0 + seconds;
        j->ringBytes = ringBytes;
        if (pthread_create(&ts[k], NULL, worker, j) != 0) {
            rc = -1;
            break;
        }
        started++;
    }
    uint64_t done = 0;
    for (int k = 0; k < started; k++) {
        pthread_join(ts[k], NULL);
        done += jobs[k].done;
        if (jobs[k].bad) rc = -1;
    }
    *elapsed = now_s() - t0;
    *bytesDone = done;
    free(jobs);
    free(ts);
    return rc;
}
