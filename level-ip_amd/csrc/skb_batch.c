/*
 * skb_batch.c — f1/f2 of SURVEY.md §8f: batch-and-dispatch over level-ip frames.
 * See include/lvlip_skb.h for the contract; every decision cites the reference
 * line it mirrors.  Host logic only: the exported plan/apply steps, f4 on the
 * host and the skb-queue walkers.  The host frame calls themselves parse on
 * the device (frames_host.cpp); round 4's path, which planned every frame
 * here and batched the planned pieces, was retired in round 5 once the device
 * parse measured faster from every source.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lvlip_skb.h"

#define ETH_HDR_LEN 14u   /* include/ethernet.h: struct eth_hdr, 14 B packed */
#define ETH_P_IP 0x0800u
#define PROTO_ICMP 1u     /* include/ip.h: ICMPV4 */
#define PROTO_TCP 6u      /* include/ip.h: IP_TCP */
#define PENDING 0x80u     /* rx_plan: verdict decided once the header checksum is known */

static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t le32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

/* Frames sit hundreds of bytes apart, too far for the hardware prefetchers: each
 * header would be a DRAM round trip (~56 ns per frame measured).  Touch the
 * header PF_AHEAD frames early instead (a prefetch never faults). */
#define PF_AHEAD 32u
static inline void pf_header(const lvlip_frame *frames, uint32_t i, uint32_t n)
{
    if (i + PF_AHEAD < n) {
        const uint8_t *h = frames[i + PF_AHEAD].head;
        __builtin_prefetch(h + ETH_HDR_LEN);
        __builtin_prefetch(h + ETH_HDR_LEN + 63u);
    }
}
static inline uint32_t le16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

uint32_t lvlip_pseudo_sum_rfc(uint32_t saddr, uint32_t daddr, uint8_t proto, uint16_t len)
{
    /* the same words the reference adds (src/tcp.c:92-95), but as 16-bit halves so
     * no carry is lost: sum < 6 * 0xffff, folded by the checksum's final fold */
    return (saddr & 0xffffu) + (saddr >> 16) + (daddr & 0xffffu) + (daddr >> 16) +
           bswap16((uint16_t)proto) + bswap16(len);
}

/* ----------------------------------------------------------------- f1: RX */

/* frames [lo, hi) -> entries iov[0..m), tags with global frame indices */
static uint32_t rx_plan_range(const lvlip_frame *frames, uint32_t lo, uint32_t hi, uint32_t flags,
                              uint8_t *verdict, lvlip_csum_iov *iov, uint32_t *tag)
{
    uint32_t m = 0;
    for (uint32_t i = lo; i < hi; i++) {
        pf_header(frames, i, hi);
        const uint8_t *h = frames[i].head;
        const uint32_t flen = frames[i].len;
        verdict[i] = 0;
        if (!h || flen < ETH_HDR_LEN + 20u) {
            verdict[i] = LVLIP_RX_SHORT;
            continue;
        }
        if (be16(h + 12) != ETH_P_IP) { /* netdev_receive dispatch, src/netdev.c:67-80 */
            verdict[i] = LVLIP_RX_NOT_IP;
            continue;
        }
        const uint8_t *ih = h + ETH_HDR_LEN;
        const uint32_t version = ih[0] >> 4, ihl = ih[0] & 0x0fu; /* ihl:4 low nibble, include/ip.h:33-34 */
        if (version != 4u) { /* src/ip_input.c:22 */
            verdict[i] = LVLIP_RX_BAD_VERSION;
            continue;
        }
        if (ihl < 5u) { /* src/ip_input.c:27 */
            verdict[i] = LVLIP_RX_BAD_IHL;
            continue;
        }
        if (ih[8] == 0u) { /* ttl, src/ip_input.c:32 */
            verdict[i] = LVLIP_RX_TTL0;
            continue;
        }
        if (flen < ETH_HDR_LEN + ihl * 4u) {
            verdict[i] = LVLIP_RX_SHORT;
            continue;
        }
        /* checksum(ih, ihl*4, 0) must be 0, src/ip_input.c:38-43 */
        iov[m].ptr = ih;
        iov[m].len = (int32_t)(ihl * 4u);
        iov[m].start_sum = 0;
        tag[m++] = i << 1;
        /* decided after the checksum (ip_rcv checks it first): a pending
         * verdict PENDING|X becomes X if the header checksum passes */
        const uint32_t proto = ih[9];
        if (proto != PROTO_TCP && proto != PROTO_ICMP) { /* src/ip_input.c:51-60 */
            verdict[i] = PENDING | LVLIP_RX_UNKNOWN_PROTO;
            continue;
        }
        if (flags & LVLIP_RX_VERIFY_L4) {
            const uint32_t iplen = be16(ih + 2);
            if (iplen < ihl * 4u || flen < ETH_HDR_LEN + iplen) {
                verdict[i] = PENDING | LVLIP_RX_SHORT;
                continue;
            }
            const uint32_t l4len = iplen - ihl * 4u;
            iov[m].ptr = ih + ihl * 4u;
            iov[m].len = (int32_t)l4len;
            iov[m].start_sum = proto == PROTO_TCP
                                   ? lvlip_pseudo_sum_rfc(le32(ih + 12), le32(ih + 16), PROTO_TCP,
                                                          (uint16_t)l4len)
                                   : 0u;
            tag[m++] = (i << 1) | 1u;
        }
    }
    return m;
}

uint32_t lvlip_rx_plan(const lvlip_frame *frames, uint32_t n, uint32_t flags,
                       uint8_t *verdict, lvlip_csum_iov *iov, uint32_t *tag)
{
    return rx_plan_range(frames, 0, n, flags, verdict, iov, tag);
}

static inline int pending(uint8_t v) { return v == 0 || (v & PENDING); }

void lvlip_rx_apply(uint32_t n, uint8_t *verdict, uint32_t m, const uint32_t *tag,
                    const uint16_t *csum)
{
    (void)n;
    /* every pending frame has its header entry, so walking the entries reaches
     * all of them: header checksum first, then L4, then the deferred verdict */
    for (uint32_t k = 0; k < m; k++)
        if (!(tag[k] & 1u) && csum[k] != 0 && pending(verdict[tag[k] >> 1]))
            verdict[tag[k] >> 1] = LVLIP_RX_BAD_CSUM;
    for (uint32_t k = 0; k < m; k++)
        if ((tag[k] & 1u) && csum[k] != 0 && verdict[tag[k] >> 1] == 0)
            verdict[tag[k] >> 1] = LVLIP_RX_BAD_L4;
    for (uint32_t k = 0; k < m; k++) {
        uint8_t *v = &verdict[tag[k] >> 1];
        if (pending(*v)) *v = *v ? (uint8_t)(*v & ~PENDING) : (uint8_t)LVLIP_RX_OK;
    }
}

/* ----------------------------------------------------------------- f2: TX */

static uint32_t tx_plan_range(lvlip_frame *frames, uint32_t lo, uint32_t hi, lvlip_csum_iov *iov,
                              uint8_t **field)
{
    uint32_t m = 0;
    for (uint32_t i = lo; i < hi; i++) {
        pf_header(frames, i, hi);
        uint8_t *h = frames[i].head;
        if (!h || frames[i].len < ETH_HDR_LEN + 20u) return 0xFFFFFFFFu;
        uint8_t *ih = h + ETH_HDR_LEN;
        const uint32_t ihl = ih[0] & 0x0fu, iplen = be16(ih + 2), proto = ih[9];
        if ((ih[0] >> 4) != 4u || ihl < 5u || iplen < ihl * 4u ||
            frames[i].len < ETH_HDR_LEN + iplen)
            return 0xFFFFFFFFu;
        uint8_t *l4 = ih + ihl * 4u;
        const uint32_t l4len = iplen - ihl * 4u;
        /* The reference zeroes each checksum field before summing
         * (src/tcp_output.c:110, src/icmpv4.c:46, src/ip_output.c:42).  Instead
         * of writing the frame now, the field's current u16 (an even offset, so
         * it is exactly one summed word) is subtracted from the seed: mod 2^32
         * that is the same T, and a failed batch leaves the frame untouched. */
        if (proto == PROTO_TCP && l4len >= 20u) {
            iov[m].ptr = l4;
            iov[m].len = (int32_t)l4len;
            iov[m].start_sum = lvlip_pseudo_sum(le32(ih + 12), le32(ih + 16), PROTO_TCP,
                                                (uint16_t)l4len) - le16(l4 + 16);
            field[m++] = l4 + 16;
        } else if (proto == PROTO_ICMP && l4len >= 4u) {
            iov[m].ptr = l4;
            iov[m].len = (int32_t)l4len;
            iov[m].start_sum = 0u - le16(l4 + 2);
            field[m++] = l4 + 2;
        }
        iov[m].ptr = ih;
        iov[m].len = (int32_t)(ihl * 4u);
        iov[m].start_sum = 0u - le16(ih + 10);
        field[m++] = ih + 10;
    }
    return m;
}

uint32_t lvlip_tx_plan(lvlip_frame *frames, uint32_t n, lvlip_csum_iov *iov, uint8_t **field)
{
    return tx_plan_range(frames, 0, n, iov, field);
}

void lvlip_tx_apply(uint32_t m, uint8_t *const *field, const uint16_t *csum)
{
    for (uint32_t k = 0; k < m; k++) memcpy(field[k], &csum[k], 2); /* raw store */
}

/* ------------------------------------------- f1/f2 on the calling thread (CPU) */

/* One frame's RX verdict, the decisions of rx_plan_range in ip_rcv's order
 * (src/ip_input.c:17-60) with the checksums computed at once: a failing header
 * checksum (src/ip_input.c:38-43) outranks every verdict decided after it
 * (unknown protocol, short L4), as lvlip_rx_apply resolves the pending ones. */
static uint8_t rx_verdict_one(const uint8_t *h, uint32_t flen, uint32_t flags)
{
    if (!h || flen < ETH_HDR_LEN + 20u) return LVLIP_RX_SHORT;
    if (be16(h + 12) != ETH_P_IP) return LVLIP_RX_NOT_IP; /* src/netdev.c:67-80 */
    const uint8_t *ih = h + ETH_HDR_LEN;
    const uint32_t ihl = ih[0] & 0x0fu;
    if ((ih[0] >> 4) != 4u) return LVLIP_RX_BAD_VERSION; /* src/ip_input.c:22 */
    if (ihl < 5u) return LVLIP_RX_BAD_IHL;                /* src/ip_input.c:27 */
    if (ih[8] == 0u) return LVLIP_RX_TTL0;                /* src/ip_input.c:32 */
    if (flen < ETH_HDR_LEN + ihl * 4u) return LVLIP_RX_SHORT;
    if (checksum((void *)ih, (int)(ihl * 4u), 0) != 0) return LVLIP_RX_BAD_CSUM; /* :38-43 */
    const uint32_t proto = ih[9];
    if (proto != PROTO_TCP && proto != PROTO_ICMP) return LVLIP_RX_UNKNOWN_PROTO; /* :51-60 */
    if (flags & LVLIP_RX_VERIFY_L4) {
        const uint32_t iplen = be16(ih + 2);
        if (iplen < ihl * 4u || flen < ETH_HDR_LEN + iplen) return LVLIP_RX_SHORT;
        const uint32_t l4len = iplen - ihl * 4u;
        const uint32_t seed = proto == PROTO_TCP ? lvlip_pseudo_sum_rfc(le32(ih + 12), le32(ih + 16), PROTO_TCP,
                                                                         (uint16_t)l4len)
                                                 : 0u;
        if (checksum((void *)(ih + ihl * 4u), (int)l4len, (int)seed) != 0) return LVLIP_RX_BAD_L4;
    }
    return LVLIP_RX_OK;
}

int lvlip_rx_verify_cpu(const lvlip_frame *frames, uint32_t n, uint32_t flags, uint8_t *verdict)
{
    if ((n && (!frames || !verdict)) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    for (uint32_t i = 0; i < n; i++) {
        pf_header(frames, i, n);
        verdict[i] = rx_verdict_one(frames[i].head, frames[i].len, flags);
    }
    return LVLIP_OK;
}

/* tx_plan_range's refusal, for one frame (0 = well formed) */
static int tx_malformed(const lvlip_frame *f)
{
    const uint8_t *h = f->head;
    if (!h || f->len < ETH_HDR_LEN + 20u) return 1;
    const uint8_t *ih = h + ETH_HDR_LEN;
    const uint32_t ihl = ih[0] & 0x0fu, iplen = be16(ih + 2);
    return (ih[0] >> 4) != 4u || ihl < 5u || iplen < ihl * 4u || f->len < ETH_HDR_LEN + iplen;
}

int lvlip_tx_checksum_cpu(lvlip_frame *frames, uint32_t n)
{
    if ((n && !frames) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    /* every frame checked before the first store: a malformed one leaves the
     * batch untouched, as the GPU call does */
    for (uint32_t i = 0; i < n; i++) {
        pf_header(frames, i, n);
        if (tx_malformed(&frames[i])) return LVLIP_EINVAL;
    }
    for (uint32_t i = 0; i < n; i++) {
        pf_header(frames, i, n);
        uint8_t *ih = frames[i].head + ETH_HDR_LEN;
        const uint32_t ihl = ih[0] & 0x0fu, l4len = be16(ih + 2) - ihl * 4u, proto = ih[9];
        uint8_t *l4 = ih + ihl * 4u;
        /* each field's current u16 taken out of the seed (tx_plan_range): the
         * reference's zero-then-sum, src/tcp_output.c:110,126, src/icmpv4.c:46-47 */
        if (proto == PROTO_TCP && l4len >= 20u) {
            const uint32_t seed = lvlip_pseudo_sum(le32(ih + 12), le32(ih + 16), PROTO_TCP, (uint16_t)l4len) -
                                  le16(l4 + 16);
            const uint16_t c = checksum(l4, (int)l4len, (int)seed);
            memcpy(l4 + 16, &c, 2);
        } else if (proto == PROTO_ICMP && l4len >= 4u) {
            const uint16_t c = checksum(l4, (int)l4len, (int)(0u - le16(l4 + 2)));
            memcpy(l4 + 2, &c, 2);
        }
        /* src/ip_output.c:42,53 (the header sum does not cover the L4 bytes) */
        const uint16_t hc = checksum(ih, (int)(ihl * 4u), (int)(0u - le16(ih + 10)));
        memcpy(ih + 10, &hc, 2);
    }
    return LVLIP_OK;
}

/* ----------------------------------------------------------------- f4: RFC 1624 */

/* One's-complement add of two 16-bit values (end-around carry). */
static inline uint32_t oc_add(uint32_t a, uint32_t b)
{
    const uint32_t t = a + b;
    return (t & 0xffffu) + (t >> 16);
}

uint32_t lvlip_icmp_echo_reply_csum(uint16_t req_csum)
{
    /* The request verified: S + HC == 0xffff (one's complement), S the sum of the
     * message with the field zeroed, S in [1, 0xffff] (its type byte is 8).  So
     * S = ~HC, except HC = 0xffff (the other representation of zero), S = 0xffff.
     * Reply: the word {type, code} = 0x0008 becomes 0x0000 (RFC 1624 eqn. 3:
     * S' = S + ~m + m').  The reference's double fold of the full sum yields the
     * same value in [1, 0xffff] for any non-zero message, and 0 only for an
     * all-zero one; S' = 0xffff cannot tell those apart, hence RECOMPUTE. */
    const uint32_t S = req_csum == 0xffffu ? 0xffffu : (uint32_t)(uint16_t)~req_csum;
    const uint32_t S1 = oc_add(S, 0xffffu - 0x0008u);
    if (S1 == 0xffffu) return LVLIP_CSUM_RECOMPUTE;
    return (uint16_t)~S1;
}

uint32_t lvlip_icmp_echo_reply_fill(lvlip_frame *frames, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *h = frames[i].head;
        if (!h || frames[i].len < ETH_HDR_LEN + 20u) return 0xFFFFFFFFu;
        const uint8_t *ih = h + ETH_HDR_LEN;
        const uint32_t ihl = ih[0] & 0x0fu, iplen = be16(ih + 2);
        if ((ih[0] >> 4) != 4u || ihl < 5u || ih[9] != PROTO_ICMP || iplen < ihl * 4u + 4u ||
            frames[i].len < ETH_HDR_LEN + iplen || ih[ihl * 4u] != 8u || ih[ihl * 4u + 1u] != 0u)
            return 0xFFFFFFFFu;
    }
    uint32_t recomputed = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *ih = frames[i].head + ETH_HDR_LEN;
        const uint32_t ihl = ih[0] & 0x0fu, icmp_len = be16(ih + 2) - ihl * 4u;
        uint8_t *icmp = ih + ihl * 4u;
        const uint32_t c = lvlip_icmp_echo_reply_csum((uint16_t)le16(icmp + 2));
        icmp[0] = 0; /* ICMP_V4_REPLY, src/icmpv4.c:45 */
        uint16_t v;
        if (c == LVLIP_CSUM_RECOMPUTE) {
            memset(icmp + 2, 0, 2);
            v = checksum(icmp, (int)icmp_len, 0); /* src/icmpv4.c:46-47 */
            recomputed++;
        } else {
            v = (uint16_t)c;
        }
        memcpy(icmp + 2, &v, 2);
    }
    return recomputed;
}

/* --------------------------------------------- f1/f2 over level-ip's skb queues */

/* struct sk_buff (include/skbuff.h:9-23) and struct sk_buff_head (:25-29) on
 * LP64: the intrusive list_head (include/list.h) first, then the fields these
 * walkers read.  csum_cpu.c pins len and data of the same layout. */
struct lvlip_skb_layout {
    struct lvlip_skb_layout *next, *prev; /* struct list_head list */
    void *rt;
    void *dev;
    int refcnt;
    uint16_t protocol;
    uint32_t len;
    uint32_t dlen;
    uint32_t seq;
    uint32_t end_seq;
    uint8_t *end;
    uint8_t *head;
    uint8_t *data;
    uint8_t *payload;
};
_Static_assert(offsetof(struct lvlip_skb_layout, len) == 40, "sk_buff.len offset");
_Static_assert(offsetof(struct lvlip_skb_layout, end) == 56, "sk_buff.end offset");
_Static_assert(offsetof(struct lvlip_skb_layout, head) == 64, "sk_buff.head offset");
_Static_assert(offsetof(struct lvlip_skb_layout, data) == 72, "sk_buff.data offset");

struct lvlip_skb_queue_layout {
    struct lvlip_skb_layout *next, *prev; /* struct list_head head */
    uint32_t qlen;
};

/* The queue's skbs in list order as frames (list_for_each, include/list.h).
 * rx: skb->data .. skb->end; tx: skb->data - ETH_HDR_LEN, skb->len + 14.
 * Returns the count, or -1 on a malformed entry / allocation failure. */
static int64_t skb_list_frames(struct sk_buff_head *q, int rx, lvlip_frame **out)
{
    struct lvlip_skb_queue_layout *h = (struct lvlip_skb_queue_layout *)(void *)q;
    const void *stop = h;
    uint64_t n = 0;
    for (struct lvlip_skb_layout *s = h->next; (const void *)s != stop; s = s->next) {
        if (!s || n >= LVLIP_MAX_BATCH / 2u) return -1;
        n++;
    }
    *out = NULL;
    if (n == 0) return 0;
    lvlip_frame *f = (lvlip_frame *)malloc(sizeof(lvlip_frame) * (size_t)n);
    if (!f) return -1;
    uint64_t k = 0;
    for (struct lvlip_skb_layout *s = h->next; (const void *)s != stop; s = s->next, k++) {
        if (rx) {
            if (!s->data || s->end < s->data) {
                free(f);
                return -1;
            }
            f[k].head = s->data; /* tun_read's buffer, src/netdev.c:91 */
            f[k].len = (uint32_t)(s->end - s->data);
        } else {
            if (!s->data || s->data - s->head < (ptrdiff_t)ETH_HDR_LEN) {
                free(f);
                return -1;
            }
            f[k].head = s->data - ETH_HDR_LEN; /* netdev_transmit's push, src/netdev.c:40-61 */
            f[k].len = s->len + ETH_HDR_LEN;
        }
    }
    *out = f;
    return (int64_t)n;
}

int lvlip_rx_verify_skb_list(lvlip_csum_ctx *ctx, struct sk_buff_head *q, uint32_t flags,
                             uint8_t *verdict, uint32_t cap)
{
    if (!ctx || !q) return LVLIP_EINVAL;
    lvlip_frame *f = NULL;
    const int64_t n = skb_list_frames(q, 1, &f);
    if (n < 0) return LVLIP_EINVAL;
    if ((uint64_t)n > cap) {
        free(f);
        return LVLIP_ERANGE;
    }
    if (n && !verdict) {
        free(f);
        return LVLIP_EINVAL;
    }
    const int rc = n ? lvlip_rx_verify(ctx, f, (uint32_t)n, flags, verdict) : LVLIP_OK;
    free(f);
    return rc == LVLIP_OK ? (int)n : rc;
}

int lvlip_tx_checksum_skb_list(lvlip_csum_ctx *ctx, struct sk_buff_head *q)
{
    if (!ctx || !q) return LVLIP_EINVAL;
    lvlip_frame *f = NULL;
    const int64_t n = skb_list_frames(q, 0, &f);
    if (n < 0) return LVLIP_EINVAL;
    const int rc = n ? lvlip_tx_checksum(ctx, f, (uint32_t)n) : LVLIP_OK;
    free(f);
    return rc == LVLIP_OK ? (int)n : rc;
}

int lvlip_rx_verify_skb_list_cpu(struct sk_buff_head *q, uint32_t flags, uint8_t *verdict, uint32_t cap)
{
    if (!q) return LVLIP_EINVAL;
    lvlip_frame *f = NULL;
    const int64_t n = skb_list_frames(q, 1, &f);
    if (n < 0) return LVLIP_EINVAL;
    if ((uint64_t)n > cap) {
        free(f);
        return LVLIP_ERANGE;
    }
    const int rc = n ? lvlip_rx_verify_cpu(f, (uint32_t)n, flags, verdict) : LVLIP_OK;
    free(f);
    return rc == LVLIP_OK ? (int)n : rc;
}

int lvlip_tx_checksum_skb_list_cpu(struct sk_buff_head *q)
{
    if (!q) return LVLIP_EINVAL;
    lvlip_frame *f = NULL;
    const int64_t n = skb_list_frames(q, 0, &f);
    if (n < 0) return LVLIP_EINVAL;
    const int rc = n ? lvlip_tx_checksum_cpu(f, (uint32_t)n) : LVLIP_OK;
    free(f);
    return rc == LVLIP_OK ? (int)n : rc;
}
