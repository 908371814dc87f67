/*
 * oracle/ref_txq.c — level-ip's TX path with an optional batch-and-dispatch
 * step, built from the reference's own compiled objects.  TEST INFRASTRUCTURE
 * ONLY (north_star: "src/ip_output.c and src/tcp.c ... gain an optional
 * batch-and-dispatch path over skbuff lists"; VERDICT r04 Next #2).
 *
 * oracle/Makefile links _ref/libref_txq.so from the reference objects, with
 * three of them rewritten by objcopy (our copies; no reference source is
 * changed or copied):
 *   tcp.o       tcp_v4_checksum weakened: tcp_transmit_skb's checksum
 *               (src/tcp_output.c:126) resolves to the deferring one below
 *   ip_output.o ip_send_check weakened (its call at src/ip_output.c:53 resolves
 *               below), and its call of dst_neigh_output (src/ip_output.c:55)
 *               renamed to lvlip_txq_output, the queueing hook below
 *   icmpv4.o    its checksum() call (src/icmpv4.c:47) renamed to
 *               lvlip_txq_deferred_checksum
 * So every frame the stack transmits reaches lvlip_txq_output with its TCP /
 * ICMP and IPv4 checksum fields zero, exactly as tcp_transmit_skb, icmpv4_reply
 * and ip_output leave them before summing (src/tcp_output.c:110,
 * src/icmpv4.c:46, src/ip_output.c:42).
 *
 * The hook copies the skb (callers free it when ip_output returns,
 * src/tcp_output.c:177,264,495, src/icmpv4.c:53; a retransmit queue keeps it)
 * and links the copy into one sk_buff_head, as skb_queue_tail links skbs
 * (include/skbuff.h:55-59).  A flush then fills every queued frame's fields in
 * ONE call (lvlip_txq_fill: lvlip_tx_checksum_skb_list through a context,
 * which runs a small queue on this thread and a large one on the GPU,
 * include/lvlip_skb.h; with the CPU fill when the GPU call cannot run or
 * fails), or lets the caller fill them (the CPU variant of the test: the
 * oracle's tx_fill on lvlip_txq_frames' frames), and hands each skb in queue
 * order to the real dst_neigh_output (src/dst.c:6-30 -> netdev_transmit ->
 * tun_write).
 *
 * Holding instead of copying (lvlip_txq_set_hold(1), round 6): the hook keeps a
 * reference to the skb itself, no copy.  It raises skb->refcnt by HOLD, so the
 * caller's free_skb when ip_output returns is a no-op (src/skbuff.c:22-28
 * frees only below 1), and records the skb in an array (a retransmit queue's
 * skb is already linked into sk->write_queue through skb->list, so the held
 * skbs cannot share one sk_buff_head).  The flush fills the held frames with
 * ONE lvlip_tx_checksum over {data - 14, len + 14} each, sends them, and drops
 * the hold: an skb that is on no list afterwards (tcp_alloc_skb's control
 * segments, the RX skb icmpv4_reply answered in) is freed, as its caller
 * would have; a write-queue skb stays where it is.  A held frame must leave
 * before its headers are rewritten: every retransmit path of level-ip starts
 * with skb_reset_header (src/tcp_output.c:213,343,379), which oracle/Makefile
 * weakens in a copy of skbuff.o so that the one below first flushes the queue
 * when the skb is held.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dst.h"
#include "skbuff.h"
#include "list.h"

#include "lvlip_skb.h"
#include "ref_batch.h"

#define ETH_LEN 14 /* include/ethernet.h: struct eth_hdr */

static struct sk_buff_head g_txq = {{&g_txq.head, &g_txq.head}, 0};
static unsigned long g_deferred_sums;

/* holding (see above): the held skbs in transmit order */
#define HOLD (1 << 24)
static int g_hold;
static lvlip_csum_ctx *g_hold_ctx;
static struct sk_buff **g_held;
static lvlip_frame *g_held_frames;
static int g_nheld, g_capheld;
static unsigned long g_early_frames, g_reheld;

static int is_held(const struct sk_buff *skb) { return skb->refcnt >= HOLD / 2; }

/* Copy (0, the default) or hold (1) the frames ip_output hands over.  Only
 * while nothing is queued.  Returns 0, or -1. */
int lvlip_txq_set_hold(int on)
{
    if (g_txq.qlen || g_nheld) return -1;
    g_hold = on != 0;
    return 0;
}

/* The context the flush before a retransmit uses (NULL: the CPU fill).  Set
 * it back to NULL before destroying that context. */
void lvlip_txq_set_ctx(lvlip_csum_ctx *ctx) { g_hold_ctx = ctx; }

/* frames sent by the flushes skb_reset_header made before rewriting a held skb */
unsigned long lvlip_txq_early_frames(void) { return g_early_frames; }

/* held skbs transmitted again without skb_reset_header (their first frame
 * lost; level-ip has no such path, the tests check 0) */
unsigned long lvlip_txq_reheld(void) { return g_reheld; }

static int hold(struct sk_buff *skb)
{
    if (g_nheld == g_capheld) {
        const int cap = g_capheld ? 2 * g_capheld : 1024;
        struct sk_buff **h = realloc(g_held, (size_t)cap * sizeof *h);
        if (!h) return -1;
        g_held = h;
        lvlip_frame *f = realloc(g_held_frames, (size_t)cap * sizeof *f);
        if (!f) return -1;
        g_held_frames = f;
        g_capheld = cap;
    }
    skb->refcnt += HOLD;
    g_held[g_nheld++] = skb;
    return 0;
}

/* Drop the hold: free the skb when no one else keeps it (on no list, as
 * tcp_alloc_skb's and the RX path's skbs are; or its owner released it while
 * held, as tcp_clean_rto_queue's refcnt-- does, src/tcp_input.c:75-77). */
static void release(struct sk_buff *skb)
{
    skb->refcnt -= HOLD;
    if (skb->refcnt < 0 || (skb->refcnt == 0 && list_empty(&skb->list))) free_skb(skb);
}

/* src/tcp_output.c:126: the field stays 0 until the flush */
int tcp_v4_checksum(struct sk_buff *skb, uint32_t saddr, uint32_t daddr)
{
    (void)skb, (void)saddr, (void)daddr;
    g_deferred_sums++;
    return 0;
}

/* src/ip_output.c:53: ip_output zeroed the field (:42); it stays 0 */
void ip_send_check(struct iphdr *ihdr)
{
    (void)ihdr;
    g_deferred_sums++;
}

/* src/icmpv4.c:47: icmpv4_reply zeroed the field (:46); it stays 0 */
uint16_t lvlip_txq_deferred_checksum(void *addr, int count, int start_sum)
{
    (void)addr, (void)count, (void)start_sum;
    g_deferred_sums++;
    return 0;
}

/* In place of dst_neigh_output (src/ip_output.c:55): queue a copy of the
 * frame, compact: the 14 bytes netdev_transmit will push (src/netdev.c:46)
 * and skb->data .. skb->end, the IPv4 packet.  Returns what tun_write returns
 * for it (netdev_transmit, the frame's length with its Ethernet header), or
 * -1 when out of memory. */
int lvlip_txq_output(struct sk_buff *skb)
{
    if (g_hold && skb->data - skb->head >= ETH_LEN) {
        if (is_held(skb)) {
            g_reheld++;
            return -1;
        }
        return hold(skb) == 0 ? (int)(skb->len + ETH_LEN) : -1;
    }
    const unsigned int size = (unsigned int)(skb->end - skb->data) + ETH_LEN;
    struct sk_buff *c = alloc_skb(size);
    if (!c) return -1;
    memcpy(c->head + ETH_LEN, skb->data, size - ETH_LEN);
    c->data = c->head + ETH_LEN;
    c->len = skb->len;
    c->dlen = skb->dlen;
    c->dev = skb->dev;
    c->rt = skb->rt;
    c->protocol = skb->protocol;
    c->seq = skb->seq;
    c->end_seq = skb->end_seq;
    if (g_hold) { /* no room for the Ethernet header in front: hold the copy */
        if (hold(c) != 0) return -1;
    } else {
        skb_queue_tail(&g_txq, c);
    }
    return (int)(skb->len + ETH_LEN);
}

int lvlip_txq_len(void) { return g_hold ? g_nheld : (int)g_txq.qlen; }

/* the queue itself (an sk_buff_head), for a caller that makes the batch call directly */
struct sk_buff_head *lvlip_txq_queue(void) { return (struct sk_buff_head *)&g_txq; }

/* checksum computations the TX path deferred since the last call */
unsigned long lvlip_txq_deferred(void)
{
    const unsigned long d = g_deferred_sums;
    g_deferred_sums = 0;
    return d;
}

/* The queued frames in queue order (the skb's data - 14 .. data + len), for a
 * caller that fills the fields itself.  Returns the count. */
int lvlip_txq_frames(lvlip_frame *out, int cap)
{
    if (g_hold) {
        for (int k = 0; k < g_nheld && k < cap; k++) {
            out[k].head = g_held[k]->data - ETH_LEN;
            out[k].len = g_held[k]->len + ETH_LEN;
        }
        return g_nheld;
    }
    int k = 0;
    struct list_head *p;
    list_for_each(p, &g_txq.head) {
        struct sk_buff *s = list_entry(p, struct sk_buff, list);
        if (k < cap) {
            out[k].head = s->data - ETH_LEN;
            out[k].len = s->len + ETH_LEN;
        }
        k++;
    }
    return k;
}

/* A frame queued as if ip_output had queued it (the tests' malformed frame):
 * len bytes from its Ethernet header, route and device taken from the last
 * queued skb.  Returns 0, or -1 (out of memory, or nothing queued yet). */
int lvlip_txq_inject(const uint8_t *frame, unsigned int len)
{
    if (!lvlip_txq_len() || len < ETH_LEN) return -1;
    struct sk_buff *last = g_hold ? g_held[g_nheld - 1] : list_entry(g_txq.head.prev, struct sk_buff, list);
    struct sk_buff *c = alloc_skb(len);
    if (!c) return -1;
    memcpy(c->head, frame, len);
    c->data = c->head + ETH_LEN;
    c->len = len - ETH_LEN;
    c->dev = last->dev;
    c->rt = last->rt;
    if (g_hold) return hold(c);
    skb_queue_tail(&g_txq, c);
    return 0;
}

/* The flush's fill, as INTEGRATION.md §2a gives it to a maintainer: every
 * queued frame's checksums in ONE call through the context (a queue of at
 * most the context's cpu_max frames is summed on this thread by the library,
 * a longer one on the GPU).  No frame may leave with a deferred (zero) field
 * (src/ip_output.c:53-55 sends whatever the fields hold), so:
 *   - no context (it could not be made), or the call failed without touching
 *     the frames for a device / HIP / memory / arena reason: the same fill on
 *     this thread (lvlip_tx_checksum_skb_list_cpu);
 *   - LVLIP_EINVAL (a malformed frame: the call left EVERY frame untouched):
 *     each frame filled on its own on this thread; a frame the fill refuses
 *     (and one whose skb has no room for the Ethernet header) is unlinked,
 *     freed and counted, never sent.
 * Returns the number of frames filled, or a negative LVLIP_E* if even the
 * CPU fill could not run. */
static int fill_held(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r);

int lvlip_txq_fill(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r)
{
    struct sk_buff_head *q = (struct sk_buff_head *)&g_txq;
    memset(r, 0, sizeof *r);
    if (g_hold) return fill_held(ctx, r);
    int rc = ctx ? lvlip_tx_checksum_skb_list(ctx, q) : LVLIP_ENODEV;
    r->rc = rc;
    if (rc >= 0) return r->frames = rc;
    r->cpu = 1;
    if (rc != LVLIP_EINVAL) {
        rc = lvlip_tx_checksum_skb_list_cpu(q);
        if (rc >= 0) return r->frames = rc;
        if (rc != LVLIP_EINVAL) return rc;
    }
    struct list_head *p, *t;
    list_for_each_safe(p, t, &g_txq.head) {
        struct sk_buff *s = list_entry(p, struct sk_buff, list);
        lvlip_frame f = {s->data - ETH_LEN, s->len + ETH_LEN};
        if (!s->data || s->data - s->head < ETH_LEN || lvlip_tx_checksum_cpu(&f, 1) != LVLIP_OK) {
            list_del(&s->list);
            g_txq.qlen--;
            free_skb(s);
            r->dropped++;
        } else {
            r->frames++;
        }
    }
    return r->frames;
}

/* The dispatch step: each queued skb in order to the real dst_neigh_output,
 * then freed.  Returns the number of frames handed over. */
int lvlip_txq_send(void)
{
    int k = 0;
    if (g_hold) {
        /* g_nheld is read each time round: a send never holds (dst_neigh_output
         * writes to the tap), but keep the loop honest */
        for (; k < g_nheld; k++) {
            struct sk_buff *s = g_held[k];
            dst_neigh_output(s);
            release(s);
        }
        g_nheld = 0;
        return k;
    }
    while (g_txq.qlen) {
        struct sk_buff *s = list_first_entry(&g_txq.head, struct sk_buff, list);
        list_del(&s->list);
        g_txq.qlen--;
        dst_neigh_output(s);
        free_skb(s);
        k++;
    }
    return k;
}

/* lvlip_txq_fill for held frames: the same decisions over the frame array
 * (lvlip_tx_checksum, include/lvlip_skb.h), a refused frame's hold dropped
 * without sending it. */
static int fill_held(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r)
{
    const int n = g_nheld;
    if (!n) return 0;
    lvlip_txq_frames(g_held_frames, n);
    int rc = ctx ? lvlip_tx_checksum(ctx, g_held_frames, (uint32_t)n) : LVLIP_ENODEV;
    r->rc = rc;
    if (rc >= 0) return r->frames = n;
    r->cpu = 1;
    if (rc != LVLIP_EINVAL) {
        rc = lvlip_tx_checksum_cpu(g_held_frames, (uint32_t)n);
        if (rc >= 0) return r->frames = n;
        if (rc != LVLIP_EINVAL) return rc;
    }
    int k = 0;
    for (int i = 0; i < n; i++) {
        if (lvlip_tx_checksum_cpu(&g_held_frames[i], 1) != LVLIP_OK) {
            release(g_held[i]);
            r->dropped++;
        } else {
            g_held[k++] = g_held[i];
        }
    }
    g_nheld = k;
    return r->frames = k;
}

/* The whole flush in one call: lvlip_txq_fill, then lvlip_txq_send.  Returns
 * the frames sent, or the fill's negative LVLIP_E* (nothing sent). */
int lvlip_txq_flush(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r)
{
    const int rc = lvlip_txq_fill(ctx, r);
    return rc < 0 ? rc : lvlip_txq_send();
}

/* skb_reset_header (src/skbuff.c:50-54; weak in oracle/Makefile's copy of
 * skbuff.o): a held frame is flushed, with everything queued before it, before
 * the retransmit rewrites its headers. */
void skb_reset_header(struct sk_buff *skb)
{
    if (g_hold && is_held(skb)) {
        struct lvlip_txq_report r;
        const int sent = lvlip_txq_flush(g_hold_ctx, &r);
        if (sent > 0) g_early_frames += (unsigned long)sent;
    }
    skb->data = skb->end - skb->dlen;
    skb->len = skb->dlen;
}
