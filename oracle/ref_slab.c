/*
 * oracle/ref_slab.c — level-ip's alloc_skb / free_skb (src/skbuff.c:5-28) with
 * the data buffers carved from one slab, which the batch context registers
 * (lvlip_csum_register, LVLIP_REG_DMA).  TEST INFRASTRUCTURE ONLY: the
 * allocator INTEGRATION.md §2b'' recommends to a maintainer whose stack batches
 * large bursts, run under the reference's own RX and TX code
 * (_ref/libref_rxtxq_slab.so, tests/ref_scale_child.py option "slab").
 *
 * oracle/Makefile weakens alloc_skb and free_skb in a copy of skbuff.o, so the
 * stack's every allocation (netdev_rx_loop's, tcp_alloc_skb's, arp's, the TX
 * queue's copies in ref_txq.c) lands here.  Buffers are bump-allocated in
 * 256-B granules in allocation order, so a burst's skbs lie densely and in
 * order in the slab; when every buffer is free again the bump pointer goes
 * back to the start.  A request that does not fit falls back to malloc.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "list.h"
#include "skbuff.h"

static uint8_t *g_slab;
static size_t g_bytes, g_next, g_live;

/* One slab of `bytes` (2 MiB aligned).  Returns 0, or -1. */
int lvlip_slab_init(size_t bytes)
{
    if (g_slab) return -1;
    if (posix_memalign((void **)&g_slab, 2u << 20, bytes) != 0) return -1;
    memset(g_slab, 0, bytes); /* fault the pages in before anyone times anything */
    g_bytes = bytes;
    return 0;
}

void *lvlip_slab_base(void) { return g_slab; }
size_t lvlip_slab_bytes(void) { return g_bytes; }

static int in_slab(const uint8_t *p) { return g_slab && p >= g_slab && p < g_slab + g_bytes; }

/* src/skbuff.c:5-20, the buffer from the slab */
struct sk_buff *alloc_skb(unsigned int size)
{
    struct sk_buff *skb = malloc(sizeof(struct sk_buff));
    memset(skb, 0, sizeof(struct sk_buff));
    const size_t sz = ((size_t)size + 255u) & ~(size_t)255u;
    if (g_slab && g_next + sz <= g_bytes) {
        skb->data = g_slab + g_next;
        g_next += sz;
        g_live++;
    } else {
        skb->data = malloc(size);
    }
    memset(skb->data, 0, size);
    skb->refcnt = 0;
    skb->head = skb->data;
    skb->end = skb->data + size;
    list_init(&skb->list);
    return skb;
}

/* src/skbuff.c:22-28 */
void free_skb(struct sk_buff *skb)
{
    if (skb->refcnt < 1) {
        if (in_slab(skb->head)) {
            if (--g_live == 0) g_next = 0;
        } else {
            free(skb->head);
        }
        free(skb);
    }
}
