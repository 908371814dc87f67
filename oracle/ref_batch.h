/*
 * oracle/ref_batch.h — what the batch-and-dispatch harness (oracle/ref_txq.c,
 * ref_rxq.c, ref_rxtxq.c) exports to its callers.  TEST INFRASTRUCTURE ONLY.
 */
#ifndef LVLIP_REF_BATCH_H
#define LVLIP_REF_BATCH_H

#include <stdint.h>

#include "lvlip_skb.h"

struct sk_buff_head;

/* What a flush did (lvlip_txq_fill). */
struct lvlip_txq_report {
    int frames;  /* frames filled */
    int rc;      /* the batch call's return: >= 0, or LVLIP_E* (LVLIP_ENODEV: no context) */
    int cpu;     /* 1 if the fill fell back to this thread's CPU code after a failure */
    int dropped; /* malformed frames unlinked and freed, never sent */
};

int lvlip_txq_len(void);
int lvlip_txq_fill(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r);
int lvlip_txq_send(void);
int lvlip_txq_flush(lvlip_csum_ctx *ctx, struct lvlip_txq_report *r);

int lvlip_rxq_verify(lvlip_csum_ctx *ctx, struct sk_buff_head *q, uint32_t flags, uint8_t *verdict,
                     uint32_t cap, int *cpu);
int lvlip_rxq_dispatch(struct sk_buff_head *q, const uint8_t *verdict, int gate);

/* One RX burst through the batched stack (lvlip_rxtxq_burst). */
struct lvlip_rxtxq_report {
    int rx_cpu;                  /* the RX verify fell back to the CPU */
    int queued;                  /* replies queued by the dispatch */
    int sent;                    /* frames the flush handed to dst_neigh_output */
    struct lvlip_txq_report tx;  /* the flush's fill */
};

#endif
