/*
 * tx_rx_batch.c — the INTEGRATION.md §2 sketches as a plain C program against
 * the C ABI only (include/lvlip_csum.h, include/lvlip_skb.h).
 *
 * What level-ip's tcp_send loop would hold just before netdev_transmit
 * (src/tcp_output.c:445-478 -> tcp_transmit_skb -> ip_output): N malloc'd
 * frames, Ethernet at head, IPv4 at head + 14, TCP at head + 34, checksum
 * fields holding garbage.  The program
 *   1. fills every TCP and IPv4 checksum of all N frames in one call
 *      (lvlip_tx_checksum), and checks each field against the per-call drop-in
 *      the reference's own call sites use: tcp_v4_checksum's arithmetic
 *      (lvlip_pseudo_sum + checksum, src/tcp.c:87-103) and ip_send_check
 *      (src/ip_output.c:8-12);
 *   2. hands the same frames to the RX side (lvlip_rx_verify, ip_rcv's
 *      decisions, src/ip_input.c:17-60) after corrupting one IPv4 header byte in
 *      every 97th frame, and checks the verdicts.
 * Prints "tx_rx_batch ok ..." and exits 0 when everything matches.
 *
 * SOURCE picks where the frames live (INTEGRATION.md §2b''):
 *   malloc    every frame its own malloc'd buffer, as level-ip allocates skbs
 *             (src/skbuff.c:5-20): the library gathers them into its pinned arena
 *   dma       every frame carved from one slab (64-B aligned, back to back)
 *             registered once with LVLIP_REG_DMA: the copy engine reads the slab
 *   zerocopy  the same slab registered LVLIP_REG_ZEROCOPY: the kernel reads it
 *             in place over PCIe
 * Each call's wall time and the process's CPU time per frame (every thread:
 * the caller and the library's workers) are printed beside it, after one
 * untimed call of each.
 *
 *   make -C examples && examples/build/tx_rx_batch [frames] [malloc|dma|zerocopy]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

static uint64_t rng_state = 0x1E7E1C5ull;
static uint64_t rnd(void) /* splitmix64 */
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

static double cpu_ms(void) /* the whole process: every thread */
{
    struct timespec t;
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

static void put16be(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* one frame as ip_output leaves it (include/ip.h, include/tcp.h layouts), in
 * its own malloc'd buffer, or at *slab_at (advanced past it, 64-B aligned) */
static uint8_t *make_frame(uint32_t payload, uint32_t saddr, uint32_t daddr, uint32_t *flen, uint8_t **slab_at)
{
    const uint32_t iplen = 20 + 20 + payload;
    uint8_t *h = slab_at ? *slab_at : malloc(14 + iplen);
    if (!h) return NULL;
    if (slab_at) *slab_at += (14 + iplen + 63u) & ~63u;
    for (uint32_t i = 0; i < 14 + iplen; i++) h[i] = (uint8_t)rnd();
    put16be(h + 12, 0x0800);                 /* ethertype IPv4 */
    uint8_t *ih = h + 14;
    ih[0] = 0x45;                            /* version 4, ihl 5 */
    ih[1] = 0;
    put16be(ih + 2, (uint16_t)iplen);
    ih[8] = 64;                              /* ttl */
    ih[9] = 6;                               /* IP_TCP */
    memcpy(ih + 12, &saddr, 4);              /* network order, as ip_output stores them */
    memcpy(ih + 16, &daddr, 4);
    ih[20 + 12] = 5 << 4;                    /* TCP data offset 5 */
    *flen = 14 + iplen;
    return h;                                /* both checksum fields left random */
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 0) : 65536u;
    const char *source = argc > 2 ? argv[2] : "malloc";
    const int use_slab = strcmp(source, "malloc") != 0;
    const uint32_t reg_flags = !strcmp(source, "zerocopy") ? LVLIP_REG_ZEROCOPY : LVLIP_REG_DMA;
    if (use_slab && strcmp(source, "dma") && strcmp(source, "zerocopy")) {
        fprintf(stderr, "usage: %s [frames] [malloc|dma|zerocopy]\n", argv[0]);
        return 2;
    }
    lvlip_frame *fr = calloc(n, sizeof *fr);
    uint8_t *verdict = malloc(n);
    /* the slab: every frame's 64-B rounded size at most 14 + 40 + 1460 + 63 */
    const size_t slab_bytes = use_slab ? (size_t)n * 1600u : 0;
    uint8_t *slab_mem = use_slab ? malloc(slab_bytes + 64) : NULL;
    uint8_t *slab = slab_mem ? (uint8_t *)(((uintptr_t)slab_mem + 63) & ~(uintptr_t)63) : NULL, *slab_at = slab;
    if (!fr || !verdict || (use_slab && !slab)) return 2;
    for (uint32_t i = 0; i < n; i++) {
        /* 10.0.0.x <-> 10.0.0.y, and every 8th pair large enough that the
         * reference's u32 pseudo-header sum loses its carry (src/tcp.c:92-95) */
        const uint32_t a = (i % 8 == 0) ? 0xC8FFFFFFu : 0x0400000Au + (uint32_t)(rnd() % 200u) * 0x01000000u;
        const uint32_t b = (i % 8 == 0) ? 0x64FFFFFFu : 0x0500000Au;
        fr[i].head = make_frame((uint32_t)(rnd() % 1461u), a, b, &fr[i].len, slab ? &slab_at : NULL);
        if (!fr[i].head) return 2;
    }

    lvlip_csum_ctx *ctx = NULL;
    int rc = lvlip_csum_ctx_create(&ctx, 0, 0);
    if (rc != LVLIP_OK) {
        fprintf(stderr, "lvlip_csum_ctx_create: %s\n", lvlip_strerror(rc));
        return 1;
    }
    if (slab && (rc = lvlip_csum_register(ctx, slab, slab_bytes, reg_flags)) != LVLIP_OK) {
        fprintf(stderr, "lvlip_csum_register: %s\n", lvlip_strerror(rc));
        return 1;
    }

    /* 1. TX: every checksum of every frame in one batch.  A first call starts
     * the context's workers and loads the kernels; the fill is idempotent (each
     * field's current value is taken out of its sum), so the timed call below
     * writes the same fields again. */
    if ((rc = lvlip_tx_checksum(ctx, fr, n)) != LVLIP_OK) {
        fprintf(stderr, "lvlip_tx_checksum: %s\n", lvlip_strerror(rc));
        return 1;
    }
    double t0 = now_ms(), c0 = cpu_ms();
    rc = lvlip_tx_checksum(ctx, fr, n);
    const double tx_ms = now_ms() - t0, tx_cpu = cpu_ms() - c0;
    if (rc != LVLIP_OK) {
        fprintf(stderr, "lvlip_tx_checksum: %s\n", lvlip_strerror(rc));
        return 1;
    }
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *ih = fr[i].head + 14, *th = ih + 20;
        const uint16_t iplen = (uint16_t)((ih[2] << 8) | ih[3]);
        const uint16_t tcplen = (uint16_t)(iplen - 20);
        uint16_t got_tcp, got_ip, want;
        memcpy(&got_tcp, th + 16, 2);
        memcpy(&got_ip, ih + 10, 2);
        uint32_t sa, da;
        memcpy(&sa, ih + 12, 4);
        memcpy(&da, ih + 16, 4);
        /* tcp_v4_checksum with the field zeroed, as tcp_transmit_skb calls it */
        memset(th + 16, 0, 2);
        want = checksum(th, tcplen, (int)lvlip_pseudo_sum(sa, da, 6, tcplen));
        bad += want != got_tcp;
        memcpy(th + 16, &got_tcp, 2);
        /* ip_send_check: zero the field, then checksum the header */
        memset(ih + 10, 0, 2);
        want = checksum(ih, 20, 0);
        bad += want != got_ip;
        memcpy(ih + 10, &got_ip, 2);
    }
    if (bad) {
        fprintf(stderr, "TX: %u checksum fields differ from the per-call path\n", bad);
        return 1;
    }

    /* 2. RX: ip_rcv's decisions for the same frames, a few corrupted */
    uint32_t corrupted = 0;
    for (uint32_t i = 0; i < n; i += 97) {
        fr[i].head[14 + 4] ^= 0x20; /* identification byte: header checksum now wrong */
        corrupted++;
    }
    (void)lvlip_rx_verify(ctx, fr, n, 0, verdict); /* warm-up, as for TX */
    t0 = now_ms();
    c0 = cpu_ms();
    rc = lvlip_rx_verify(ctx, fr, n, 0, verdict);
    const double rx_ms = now_ms() - t0, rx_cpu = cpu_ms() - c0;
    if (rc != LVLIP_OK) {
        fprintf(stderr, "lvlip_rx_verify: %s\n", lvlip_strerror(rc));
        return 1;
    }
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t want = (i % 97 == 0) ? LVLIP_RX_BAD_CSUM : LVLIP_RX_OK;
        if (verdict[i] != want) bad++;
    }
    if (bad) {
        fprintf(stderr, "RX: %u verdicts differ from ip_rcv's\n", bad);
        return 1;
    }
    if (slab) (void)lvlip_csum_unregister(ctx, slab);
    lvlip_csum_ctx_destroy(ctx);
    printf("tx_rx_batch ok: %u frames (%s), TX fill %.2f ms (%.0f ns CPU/frame), RX verify %.2f ms "
           "(%.0f ns CPU/frame; %u corrupted frames dropped)\n",
           n, source, tx_ms, tx_cpu * 1e6 / n, rx_ms, rx_cpu * 1e6 / n, corrupted);
    if (slab) free(slab_mem);
    else
        for (uint32_t i = 0; i < n; i++) free(fr[i].head);
    free(fr);
    free(verdict);
    return 0;
}
