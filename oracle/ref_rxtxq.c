/*
 * oracle/ref_rxtxq.c — one RX burst through the batched stack in a single
 * call, so that a timed run measures level-ip and the library and not its
 * caller (scripts/compose_timing.py drives it from Python; level-ip as it is
 * runs the same burst as one lvlip_rxq_receive_all).  TEST INFRASTRUCTURE
 * ONLY; linked into _ref/libref_rxtxq*.so beside ref_rxq.c and ref_txq.c.
 */
#include <string.h>

#include "skbuff.h"

#include "ref_batch.h"

/* The RX verify over the queue (lvlip_rxq_verify: the context's call, the
 * CPU fallback), the dispatch with ip_rcv's header sum gated on the verdicts,
 * then the flush of everything the dispatch queued for TX (lvlip_txq_flush).
 * verdict holds cap bytes.  Returns the burst's frame count, or a negative
 * LVLIP_E* (the RX verify or the TX fill refused), or -100 when the dispatch
 * did not take every frame. */
int lvlip_rxtxq_burst(lvlip_csum_ctx *ctx, struct sk_buff_head *q, uint32_t flags, uint8_t *verdict,
                      uint32_t cap, struct lvlip_rxtxq_report *r)
{
    memset(r, 0, sizeof *r);
    const int n = (int)q->qlen;
    int rc = lvlip_rxq_verify(ctx, q, flags, verdict, cap, &r->rx_cpu);
    if (rc < 0) return rc;
    if (lvlip_rxq_dispatch(q, verdict, 1) != n) return -100;
    r->queued = lvlip_txq_len();
    rc = lvlip_txq_flush(ctx, &r->tx);
    if (rc < 0) return rc;
    r->sent = rc;
    return n;
}
