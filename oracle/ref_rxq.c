/*
 * oracle/ref_rxq.c — ip_rcv's header checksum gated on a batch verdict, the
 * one-line change INTEGRATION.md §2b asks of a maintainer, made at link level
 * on the reference's own compiled ip_rcv.  TEST INFRASTRUCTURE ONLY (VERDICT
 * r04 Weak #5: show what the RX batch removes from the CPU, not only that its
 * decisions equal ip_rcv's).
 *
 * oracle/Makefile links _ref/libref_rxq.so from the reference objects with
 * ip_input.o's one checksum() call (src/ip_input.c:38) renamed by objcopy to
 * lvlip_rxq_checksum below.  A frame the GPU batch accepted (LVLIP_RX_OK) has
 * its IPv4 header marked by the driver (lvlip_rxq_accept); for it the check
 * at :38-43 takes the batch's result (the header summed to 0) instead of
 * summing the header again on the CPU.  Any other header is summed by the
 * reference's checksum() as before.  The counters say how many header sums
 * ran on the CPU and how many the batch answered.
 */
#include <stdint.h>

uint16_t checksum(void *addr, int count, int start_sum); /* src/utils.c:40 */

#define MAX_MARKS 65536
static const void *g_mark[MAX_MARKS];
static int g_nmark;
static unsigned long g_computed, g_skipped;

/* The batch verified this skb's IPv4 header (ip_hdr(skb), include/ip.h:47). */
int lvlip_rxq_accept(const void *ih)
{
    if (g_nmark >= MAX_MARKS) return -1;
    g_mark[g_nmark++] = ih;
    return 0;
}

uint16_t lvlip_rxq_checksum(void *addr, int count, int start_sum)
{
    for (int i = g_nmark - 1; i >= 0; i--)
        if (g_mark[i] == addr) {
            g_mark[i] = g_mark[--g_nmark]; /* one use per mark */
            g_skipped++;
            return 0; /* the batch's verdict: checksum(ih, ihl * 4, 0) == 0 */
        }
    g_computed++;
    return checksum(addr, count, start_sum);
}

unsigned long lvlip_rxq_computed(void) { return g_computed; }
unsigned long lvlip_rxq_skipped(void) { return g_skipped; }
