/*
 * e2sar_oracle.c -- plain-C restatement of the reference SAR path.
 * TEST INFRASTRUCTURE ONLY (see e2sar_oracle.h): the checker, never the product.
 *
 * Every function cites the reference line range it restates
 * (paths relative to JeffersonLab/E2SAR v0.3.2).
 */
#include "e2sar_oracle.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* big-endian helpers: glibc htobeNN / beNNtoh (include/portable_endian.h:23-25) */
static void put_be16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static void put_be64(uint8_t *p, uint64_t v) { put_be32(p, (uint32_t)(v >> 32)); put_be32(p + 4, (uint32_t)v); }
static uint16_t get_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static uint32_t get_be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static uint64_t get_be64(const uint8_t *p) { return ((uint64_t)get_be32(p) << 32) | get_be32(p + 4); }

/* ------------------------------------------------------------------ */
/* e2sarHeaders.hpp:406-421: IPv4 20 / IPv6 40 + UDP 8 + LB 16 + RE 20 */
size_t e2o_total_hdr_len(int useIPv6) { return (useIPv6 ? 40u : 20u) + 8u + 16u + 20u; }

/* e2sarDPSegmenter.hpp:241 (maxPldLen{mtu - getTotalHeaderLength(v6)}) */
size_t e2o_max_pld_len(unsigned mtu, int useIPv6)
{
    size_t h = e2o_total_hdr_len(useIPv6);
    return mtu > h ? mtu - h : 0;   /* ctor throws when mtu <= h (hpp:315-316) */
}

/* e2sarDPSegmenter.cpp:670: numBuffers = (bytes + maxPldLen - 1) / maxPldLen */
size_t e2o_num_packets(size_t bytes, size_t maxPldLen)
{
    return maxPldLen ? (bytes + maxPldLen - 1) / maxPldLen : 0;
}

/*
 * LBREHdr(ver) + re.set + lb2.set / lb3.set exactly as _send does
 * (e2sarDPSegmenter.cpp:736-755; struct layouts e2sarHeaders.hpp:21-38, 111-127, 191-208;
 *  version dispatch LBHdrU(ver) :287-297 -- anything but 3 builds a v2 header).
 */
void e2o_lbre_hdr(uint8_t out[36], int lbHdrVersion, uint16_t entropy, uint64_t lbTick,
                  uint16_t dataId, uint32_t bufferOffset, uint32_t bufferLength,
                  uint64_t eventNum)
{
    memset(out, 0, 36);
    out[0] = 'L';
    out[1] = 'B';
    if (lbHdrVersion == 3) {
        out[2] = 3;                               /* version{lbhdrVersion3} */
        out[3] = 1;                               /* nextProto{rehdrVersion} */
        put_be16(out + 4, (uint16_t)(lbTick & 0xFFFF)); /* slotSelect = lbEventNum & 0xFFFF (cpp:753) */
        put_be16(out + 6, entropy);               /* portSelect = entropy */
        put_be64(out + 8, lbTick);                /* tick */
    } else {
        out[2] = 2;                               /* version{lbhdrVersion2} */
        out[3] = 1;
        put_be16(out + 4, 0);                     /* rsvd */
        put_be16(out + 6, entropy);
        put_be64(out + 8, lbTick);                /* eventNum (tick) */
    }
    /* REHdr at +16 (sizeof(LBHdrU) == 16) */
    out[16] = 1u << 4;                            /* rehdrVersionNibble */
    out[17] = 0;
    put_be16(out + 18, dataId);
    put_be32(out + 20, bufferOffset);
    put_be32(out + 24, bufferLength);
    put_be64(out + 28, eventNum);
}

/* REHdr::get_* and validate() (e2sarHeaders.hpp:43-101) */
int e2o_re_parse(const uint8_t re[20], uint16_t *dataId, uint32_t *bufferOffset,
                 uint32_t *bufferLength, uint64_t *eventNum, uint8_t *version)
{
    if (dataId) *dataId = get_be16(re + 2);
    if (bufferOffset) *bufferOffset = get_be32(re + 4);
    if (bufferLength) *bufferLength = get_be32(re + 8);
    if (eventNum) *eventNum = get_be64(re + 12);
    if (version) *version = (uint8_t)(re[0] >> 4);
    return re[0] == (1u << 4) && re[1] == 0;
}

/*
 * The _send fragment loop (e2sarDPSegmenter.cpp:702-770) with the socket replaced by
 * "materialise the datagram at out + k*stride": iov[0] = 36-byte header, iov[1] =
 * event[curOffset : curOffset+curLen].  bufferOffset = curOffset - event, bufferLength
 * = bytes (the EVENT length, :742-743).
 */
size_t e2o_segment_event(const uint8_t *event, size_t bytes, uint64_t eventNum,
                         uint16_t dataId, uint16_t entropy, uint64_t lbTick,
                         int lbHdrVersion, size_t maxPldLen,
                         uint8_t *out, size_t stride, uint32_t *lens)
{
    size_t k = 0;
    size_t cur = 0;
    size_t curLen = bytes <= maxPldLen ? bytes : maxPldLen;     /* :704 */
    while (cur < bytes) {                                        /* :731 */
        uint8_t *pkt = out + k * stride;
        e2o_lbre_hdr(pkt, lbHdrVersion, entropy, lbTick, dataId, (uint32_t)cur,
                     (uint32_t)bytes, eventNum);
        memcpy(pkt + 36, event + cur, curLen);
        if (stride > 36 + curLen)
            memset(pkt + 36 + curLen, 0, stride - 36 - curLen);
        if (lens) lens[k] = (uint32_t)(36 + curLen);
        cur += curLen;                                           /* :769-770 */
        curLen = (bytes > cur + maxPldLen) ? maxPldLen : bytes - cur;
        k++;
    }
    return k;
}

size_t e2o_segment_batch(const uint8_t *events, size_t n, size_t bytes,
                         const uint64_t *eventNums, uint16_t dataId,
                         const uint16_t *entropies, const uint64_t *ticks,
                         int lbHdrVersion, size_t maxPldLen,
                         uint8_t *pkts, size_t stride, uint32_t *lens)
{
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        total += e2o_segment_event(events + i * bytes, bytes, eventNums[i], dataId,
                                   entropies[i], ticks[i], lbHdrVersion, maxPldLen,
                                   pkts + total * stride, stride, lens + total);
    }
    return total;
}

/* ------------------------------------------------------------------ */
/* Reassembler state: eventsInProgress (hpp:224-233), event queue (hpp:126-161),
 * lostEvents set + lostEventsQueue (hpp:262-279). */

typedef struct item {
    uint64_t eventNum;
    uint16_t dataId;
    size_t bytes, curBytes, numFragments;
    uint64_t firstSegment;       /* logical ms */
    uint8_t *event;
    struct item *next;           /* hash chain / queue link */
} item;

typedef struct lost {
    uint64_t eventNum;
    uint16_t dataId;
    uint64_t numFragments;
    struct lost *next;
} lost;

#define NBUCKET 4096u

struct e2o_reas {
    int withLB;
    size_t qcap, qlen;
    item *qhead, *qtail;              /* event queue (FIFO) */
    item *bucket[NBUCKET];            /* eventsInProgress */
    size_t inProgress;
    lost *lostSeen;                   /* lostEvents (thread-local set) */
    lost *lqHead, *lqTail;            /* lostEventsQueue */
    uint64_t now;
    e2o_reas_stats st;
    uint64_t lastPopFrags;            /* numFragments of the event last handed out (test access) */
};

/* pair_hash (e2sarUtil.hpp:526-533) */
static unsigned bucket_of(uint64_t ev, uint16_t d)
{
    uint64_t t = d;
    uint64_t h = ev ^ (t | t << 16 | t << 32 | t << 48);
    return (unsigned)(h % NBUCKET);
}

e2o_reas *e2o_reas_new(int withLBHeader, size_t queueCapacity)
{
    e2o_reas *r = (e2o_reas *)calloc(1, sizeof(e2o_reas));
    r->withLB = withLBHeader;
    /* The reference's eventQueue{QSIZE} (hpp:126-127) is a boost::lockfree::queue WITHOUT
     * fixed_sized: QSIZE pre-sizes its node pool, push() allocates beyond it, so an enqueue
     * fails only on allocation failure -- the queue is unbounded.  queueCapacity 0 restates
     * that; a nonzero capacity models the device's completed-record ring
     * (e2sar_hip_reas_config.queueCapacity), a parameter of this build, not of the reference. */
    r->qcap = queueCapacity ? queueCapacity : SIZE_MAX;
    return r;
}

static void free_item(item *it) { if (it) { free(it->event); free(it); } }

void e2o_reas_free(e2o_reas *r)
{
    if (!r) return;
    for (unsigned b = 0; b < NBUCKET; b++) {
        item *it = r->bucket[b];
        while (it) { item *n = it->next; free_item(it); it = n; }
    }
    item *q = r->qhead;
    while (q) { item *n = q->next; free_item(q); q = n; }
    lost *l = r->lostSeen;
    while (l) { lost *n = l->next; free(l); l = n; }
    l = r->lqHead;
    while (l) { lost *n = l->next; free(l); l = n; }
    free(r);
}

void e2o_reas_set_time(e2o_reas *r, uint64_t now_ms) { r->now = now_ms; }

static item **find_slot(e2o_reas *r, uint64_t ev, uint16_t d)
{
    item **pp = &r->bucket[bucket_of(ev, d)];
    while (*pp && !((*pp)->eventNum == ev && (*pp)->dataId == d)) pp = &(*pp)->next;
    return pp;
}

/* EventQueueItem(REHdr*) / initFromHeader (hpp:89-98) */
static item *new_item(e2o_reas *r, uint64_t ev, uint16_t d, uint32_t len)
{
    item *it = (item *)calloc(1, sizeof(item));
    it->eventNum = ev;
    it->dataId = d;
    it->bytes = len;
    it->event = (uint8_t *)malloc(len ? len : 1);
    it->firstSegment = r->now;
    return it;
}

/* logLostEvent (hpp:262-279): dedupe on (eventNum, dataId), push to lost queue */
static void log_lost(e2o_reas *r, const item *it, int enqueLoss)
{
    for (lost *l = r->lostSeen; l; l = l->next)
        if (l->eventNum == it->eventNum && l->dataId == it->dataId) return;
    lost *s = (lost *)calloc(1, sizeof(lost));
    s->eventNum = it->eventNum; s->dataId = it->dataId;
    s->next = r->lostSeen; r->lostSeen = s;
    lost *q = (lost *)calloc(1, sizeof(lost));
    q->eventNum = it->eventNum; q->dataId = it->dataId; q->numFragments = it->numFragments;
    if (r->lqTail) r->lqTail->next = q; else r->lqHead = q;
    r->lqTail = q;
    if (enqueLoss) r->st.enqueueLoss++; else r->st.reassemblyLoss++;
}

/*
 * One datagram through the recv body (e2sarDPReassembler.cpp:331-427).
 * Deliberate, documented guards where the reference has undefined behaviour:
 *   - nbytes shorter than the headers: counted as badHeaderDiscards (reference reads
 *     past the datagram and memcpy's a negative length);
 *   - bufferOffset + payload > bufferLength: counted in dataErrCnt and dropped
 *     (reference overflows the heap buffer at :391).
 * Every other behaviour -- including the offset-0 "always new item" rule (:361-369),
 * duplicate double counting (:400) and eventSuccess on enqueue loss (:426) -- is kept.
 */
void e2o_reas_push(e2o_reas *r, const uint8_t *dgram, size_t nbytes)
{
    r->st.totalPackets++;                        /* :332 */
    r->st.totalBytes += nbytes;                  /* :333 */
    size_t hl = r->withLB ? 36 : 20;             /* :340-349 */
    if (nbytes < hl) { r->st.badHeaderDiscards++; return; }
    const uint8_t *re = dgram + (r->withLB ? 16 : 0);
    size_t pl = nbytes - hl;
    uint16_t d; uint32_t off, len; uint64_t ev;
    if (!e2o_re_parse(re, &d, &off, &len, &ev, NULL)) {     /* :351-357 */
        r->st.badHeaderDiscards++;
        return;
    }
    if ((uint64_t)off + pl > len) { r->st.dataErrCnt++; return; }

    item **slot = find_slot(r, ev, d);
    item *it;
    if (off == 0) {                              /* :361-369: always a new item */
        it = new_item(r, ev, d, len);
        if (*slot) {                             /* replaced entry is orphaned */
            item *old = *slot;
            it->next = old->next;
            free_item(old);
            r->inProgress--;
        } else {
            it->next = NULL;
        }
        *slot = it;
        r->inProgress++;
    } else if (*slot) {                          /* :372-375 */
        it = *slot;
    } else {                                     /* :376-384 out-of-order first fragment */
        it = new_item(r, ev, d, len);
        it->next = NULL;
        *slot = it;
        r->inProgress++;
    }

    memcpy(it->event + off, re + 20, pl);        /* :391-392 */
    it->numFragments++;                          /* :398 */
    it->curBytes += pl;                          /* :400 */

    if (it->curBytes == it->bytes) {             /* :403 */
        *slot = it->next;                        /* erase (:409) */
        it->next = NULL;
        r->inProgress--;
        if (r->qlen >= r->qcap) {                /* device ring full (hpp:140-145's failure path) */
            log_lost(r, it, 1);
            free_item(it);
        } else {
            if (r->qtail) r->qtail->next = it; else r->qhead = it;
            r->qtail = it;
            r->qlen++;
        }
        r->st.eventSuccess++;                    /* :426 (even on enqueue loss) */
    }
}

/* getEvent (cpp:626-641) */
int e2o_reas_pop(e2o_reas *r, uint8_t **event, size_t *bytes, uint64_t *eventNum,
                 uint16_t *dataId)
{
    item *it = r->qhead;
    if (!it) return -1;
    r->qhead = it->next;
    if (!r->qhead) r->qtail = NULL;
    r->qlen--;
    *event = it->event;
    *bytes = it->bytes;
    *eventNum = it->eventNum;
    *dataId = it->dataId;
    r->lastPopFrags = it->numFragments;
    free(it);
    return 0;
}

/* numFragments (cpp:398) of the event the last pop handed out: the reference keeps it in
 * the EventQueueItem; getEvent does not return it, the tests compare the device's count */
uint64_t e2o_reas_last_pop_frags(const e2o_reas *r) { return r->lastPopFrags; }

void e2o_reas_push_batch(e2o_reas *r, const uint8_t *pkts, size_t n, size_t stride,
                         const uint32_t *lens)
{
    for (size_t i = 0; i < n; i++) e2o_reas_push(r, pkts + i * stride, lens[i]);
}

long long e2o_reas_pop_into(e2o_reas *r, uint8_t *buf, size_t cap, uint64_t *eventNum,
                            uint16_t *dataId)
{
    item *it = r->qhead;
    if (!it) return -1;
    if (it->bytes > cap) return -2;
    uint8_t *ev; size_t b;
    e2o_reas_pop(r, &ev, &b, eventNum, dataId);
    memcpy(buf, ev, b);
    free(ev);
    return (long long)b;
}

/* GCThreadState::_threadBody one pass (cpp:252-274): inWaiting > timeout => lost */
size_t e2o_reas_gc(e2o_reas *r, uint64_t timeout_ms)
{
    size_t n = 0;
    for (unsigned b = 0; b < NBUCKET; b++) {
        item **pp = &r->bucket[b];
        while (*pp) {
            item *it = *pp;
            if (r->now - it->firstSegment > timeout_ms) {
                log_lost(r, it, 0);
                *pp = it->next;
                free_item(it);
                r->inProgress--;
                n++;
            } else {
                pp = &it->next;
            }
        }
    }
    return n;
}

/* get_LostEvent (hpp:593-604) */
int e2o_reas_lost_pop(e2o_reas *r, uint64_t *eventNum, uint16_t *dataId, uint64_t *numFragments)
{
    lost *l = r->lqHead;
    if (!l) return -1;
    r->lqHead = l->next;
    if (!r->lqHead) r->lqTail = NULL;
    *eventNum = l->eventNum; *dataId = l->dataId; *numFragments = l->numFragments;
    free(l);
    return 0;
}

void e2o_reas_get_stats(const e2o_reas *r, e2o_reas_stats *out)
{
    *out = r->st;
    out->inProgress = r->inProgress;
}

void e2o_free(void *p) { free(p); }
