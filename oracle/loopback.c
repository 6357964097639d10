/* TEST INFRASTRUCTURE, NOT PRODUCT: BASELINE config 1 on the host CPU -- the reference's
 * SAR path with one Segmenter thread and one Reassembler thread over UDP loopback, as
 * bin/e2sar_perf.cpp's send / receive pair runs it (cpp:124-304), built from the oracle's
 * plain-C restatement (e2sar_oracle.c), never from the GPU product.  bench.py's
 * cpu_baseline leg runs it; nothing else does.
 *
 * Sender thread: for each event, e2o_segment_event (the _send fragment loop,
 * e2sarDPSegmenter.cpp:660-871) into a datagram buffer, then one sendto per datagram (the
 * reference's sendmsg per fragment, cpp:831-852).  Receiver thread: one recvfrom per
 * datagram (cpp:321) into the oracle's receive body (e2o_reas_push, cpp:335-427), then
 * getEvent and free (e2sarDPReassembler.cpp:626-641; delete[] in bin/e2sar_perf.cpp:299).
 * The reference paces its sender (--rate); here the sender instead keeps at most a window
 * of datagrams in flight (half of what the receive socket buffer holds), which measures the
 * fastest lossless rate of the pair.
 *
 * Usage: e2o_loopback BYTES MTU SECONDS   -> one JSON line on stdout. */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include "e2sar_oracle.h"

static size_t B, MTU, WINDOW;
static double SECONDS;
static int rxfd = -1, txfd = -1;
static struct sockaddr_in dst;
static atomic_ullong sentEvents, gotEvents, badEvents, rcvdPk;
static atomic_int stopFlag;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *sender(void *arg)
{
    (void)arg;
    const size_t mp = e2o_max_pld_len((unsigned)MTU, 0);
    const size_t npk = e2o_num_packets(B, mp);
    const size_t stride = (36 + mp + 15) & ~(size_t)15;
    uint8_t *ev = malloc(B), *pk = malloc(npk * stride);
    uint32_t *ln = malloc(npk * sizeof(uint32_t));
    for (size_t i = 0; i < B; i++) ev[i] = (uint8_t)(i * 131u + 7u);
    uint64_t sentPk = 0;
    for (uint64_t e = 0; !atomic_load(&stopFlag); e++) {
        ev[0] = (uint8_t)e;                                   /* each event differs */
        const size_t n = e2o_segment_event(ev, B, e, 1, (uint16_t)e, e, 2, mp, pk, stride, ln);
        for (size_t k = 0; k < n && !atomic_load(&stopFlag); k++) {
            while (sentPk >= atomic_load(&rcvdPk) + WINDOW && !atomic_load(&stopFlag)) sched_yield();
            if (sendto(txfd, pk + k * stride, ln[k], 0, (struct sockaddr *)&dst, sizeof dst) < 0) {
                k--;
                continue;
            }
            sentPk++;
        }
        atomic_store(&sentEvents, e + 1);
    }
    free(ev);
    free(pk);
    free(ln);
    return NULL;
}

static void *receiver(void *arg)
{
    (void)arg;
    e2o_reas *r = e2o_reas_new(1, 1024);
    uint8_t buf[9216];
    while (!atomic_load(&stopFlag)) {
        const ssize_t got = recvfrom(rxfd, buf, sizeof buf, 0, NULL, NULL);
        if (got <= 0) continue;                                /* 100 ms timeout */
        atomic_fetch_add(&rcvdPk, 1);
        e2o_reas_push(r, buf, (size_t)got);
        uint8_t *event;
        size_t nb;
        uint64_t en;
        uint16_t di;
        while (e2o_reas_pop(r, &event, &nb, &en, &di) == 0) {
            if (nb != B || event[0] != (uint8_t)en) atomic_fetch_add(&badEvents, 1);
            e2o_free(event);
            atomic_fetch_add(&gotEvents, 1);
        }
    }
    e2o_reas_free(r);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s BYTES MTU SECONDS\n", argv[0]);
        return 2;
    }
    B = strtoull(argv[1], NULL, 10);
    MTU = strtoull(argv[2], NULL, 10);
    SECONDS = atof(argv[3]);
    rxfd = socket(AF_INET, SOCK_DGRAM, 0);
    txfd = socket(AF_INET, SOCK_DGRAM, 0);
    int big = 64 << 20, have = 0;
    setsockopt(rxfd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(txfd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    socklen_t hl = sizeof have;
    getsockopt(rxfd, SOL_SOCKET, SO_RCVBUF, &have, &hl);       /* capped by net.core.rmem_max */
    /* a datagram costs about its size rounded to pages plus an skb in the buffer */
    WINDOW = (size_t)have / 2 / (((MTU + 4095) & ~(size_t)4095) + 1024);
    if (WINDOW < 4) WINDOW = 4;
    struct timeval tv = {0, 100000};
    setsockopt(rxfd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    memset(&dst, 0, sizeof dst);
    dst.sin_family = AF_INET;
    dst.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(rxfd, (struct sockaddr *)&dst, sizeof dst) != 0) return perror("bind"), 1;
    socklen_t sl = sizeof dst;
    getsockname(rxfd, (struct sockaddr *)&dst, &sl);
    pthread_t ts, tr;
    pthread_create(&tr, NULL, receiver, NULL);
    const double t0 = now_s();
    pthread_create(&ts, NULL, sender, NULL);
    double t1;
    while ((t1 = now_s()) - t0 < SECONDS) usleep(10000);
    const unsigned long long got = atomic_load(&gotEvents);
    atomic_store(&stopFlag, 1);
    pthread_join(ts, NULL);
    pthread_join(tr, NULL);
    const double dt = t1 - t0;
    printf("{\"events\": %llu, \"event_bytes\": %zu, \"mtu\": %zu, \"seconds\": %.3f, \"GiBps\": %.4f, "
           "\"Gbps\": %.3f, \"bad_events\": %llu, \"window_datagrams\": %zu, \"rcvbuf\": %d, "
           "\"sent_events\": %llu}\n",
           got, B, MTU, dt, got * (double)B / dt / (1u << 30), got * (double)B * 8 / dt / 1e9,
           (unsigned long long)atomic_load(&badEvents), WINDOW, have, (unsigned long long)atomic_load(&sentEvents));
    return 0;
}
