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
    uint8_t *pk = (uint8_t *)malloc(j->npk * j->stride);
    uint32_t *ln = (uint32_t *)malloc(j->npk * sizeof(uint32_t));
    if (!pk || !ln) {
        j->bad = 1;
        free(pk);
        free(ln);
        return NULL;
    }
    do {
        e2o_reas *r = e2o_reas_new(1, 1u << 20);
        for (size_t i = 0; i < j->nEvents; i++) {
            /* the same event metadata as tests/sar_inputs.py (entropy, tick) */
            const size_t n = e2o_segment_event(j->events + i * j->bytes, j->bytes, i, j->dataId,
                                               (uint16_t)(1 + (i * 0x9E37u) % 65535u),
                                               0x0001000000000000ull + i, j->lbVer, j->maxPld, pk,
                                               j->stride, ln);
            e2o_reas_push_batch(r, pk, n, j->stride, ln);
            uint8_t *ev = NULL;
            size_t nb = 0;
            uint64_t en = 0;
            uint16_t di = 0;
            if (e2o_reas_pop(r, &ev, &nb, &en, &di) != 0 || nb != j->bytes) j->bad = 1;
            e2o_free(ev);
        }
        j->done += (uint64_t)j->nEvents * j->bytes;
        e2o_reas_free(r);
    } while (now_s() < j->deadline && !j->bad);
    free(pk);
    free(ln);
    return NULL;
}

/* Run `threads` workers for `seconds` over nEvents events of `bytes` each (contiguous at
 * `events`).  Returns 0 and the payload bytes done and the wall time, or -1 on a failed
 * thread start / allocation / round trip. */
int e2o_cpu_bench(const uint8_t *events, size_t nEvents, size_t bytes, int lbHdrVersion, size_t maxPldLen,
                  uint16_t dataId, int threads, double seconds, uint64_t *bytesDone, double *elapsed)
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
