/*
 * tests/sanitize/host_san.c — the library's host C code under sanitizers.
 *
 * TEST INFRASTRUCTURE ONLY (built and run by tests/test_sanitize_host.py).
 * level-ip's `make debug` builds with -fsanitize=thread
 * (Makefile:17-18) and its test runner greps ThreadSanitizer reports
 * (tests/test-run-all:41).  The counterpart here builds the per-call drop-in
 * (level-ip_amd/csrc/csum_cpu.c) and the exported frame plan / apply steps
 * (level-ip_amd/csrc/skb_batch.c) with ASan + UBSan, and again with TSan, and
 * drives them with:
 *   1. every length 0..600 plus MTU/jumbo/64 KiB sizes at all 16 alignments,
 *      each buffer allocated to its exact end, checked against the oracle;
 *   2. eight threads calling checksum / tcp_udp_checksum at once (the
 *      reference calls checksum() from its core, IPC and timer threads);
 *   3. 40 000 frames, each in an allocation of exactly its length, through
 *      lvlip_tx_plan / lvlip_tx_apply and lvlip_rx_plan / lvlip_rx_apply with
 *      the oracle summing the planned entries, plus malformed frames that must
 *      be refused (TX) or given their verdict (RX) without reading past their
 *      ends.
 *
 * The product's host frame calls (frames_host.cpp, HIP host code) run under
 * ASan/TSan in tests/sanitize/frames_san.cpp; the skb-queue walkers of
 * skb_batch.c, which call them, are linked here against the plan + oracle
 * compositions below.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

uint32_t oracle_sum_every_16bits(const void *addr, int count);
uint16_t oracle_checksum(const void *addr, int count, int start_sum);
int oracle_tcp_udp_checksum(uint32_t saddr, uint32_t daddr, uint8_t proto, const uint8_t *data,
                            uint16_t len);

static int g_fail;
#define CHECK(c, ...)                                            \
    do {                                                         \
        if (!(c)) {                                              \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fputc('\n', stderr);                                 \
            if (++g_fail > 20) exit(1);                          \
        }                                                        \
    } while (0)

/* The frame calls' decisions as the exported host steps (plan, the oracle
 * over the planned entries, apply): stand-ins for the product's calls
 * (frames_host.cpp), which skb_batch.c's skb-queue walkers reach. */
static void sum_entries(const lvlip_csum_iov *iov, uint32_t m, uint16_t *cs)
{
    for (uint32_t k = 0; k < m; k++) cs[k] = oracle_checksum(iov[k].ptr, iov[k].len, (int)iov[k].start_sum);
}

int lvlip_rx_verify(lvlip_csum_ctx *ctx, const lvlip_frame *frames, uint32_t n, uint32_t flags,
                    uint8_t *verdict)
{
    if (!ctx || (n && (!frames || !verdict))) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    lvlip_csum_iov *iov = malloc(sizeof *iov * 2u * n);
    uint32_t *tag = malloc(sizeof *tag * 2u * n);
    uint16_t *cs = malloc(sizeof *cs * 2u * n);
    const uint32_t m = lvlip_rx_plan(frames, n, flags, verdict, iov, tag);
    sum_entries(iov, m, cs);
    lvlip_rx_apply(n, verdict, m, tag, cs);
    free(iov);
    free(tag);
    free(cs);
    return LVLIP_OK;
}

int lvlip_tx_checksum(lvlip_csum_ctx *ctx, lvlip_frame *frames, uint32_t n)
{
    if (!ctx || (n && !frames)) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    lvlip_csum_iov *iov = malloc(sizeof *iov * 2u * n);
    uint8_t **field = malloc(sizeof *field * 2u * n);
    uint16_t *cs = malloc(sizeof *cs * 2u * n);
    /* the plan reads and refuses before anything is written */
    const uint32_t m = lvlip_tx_plan(frames, n, iov, field);
    int rc = LVLIP_EINVAL;
    if (m != 0xFFFFFFFFu) {
        sum_entries(iov, m, cs);
        lvlip_tx_apply(m, field, cs);
        rc = LVLIP_OK;
    }
    free(iov);
    free(field);
    free(cs);
    return rc;
}

static uint64_t g_rng = 0x1E7E1C5ull;
static uint32_t rnd(void)
{
    g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(g_rng >> 33);
}

/* ------------------------------------------------------------- 1. sweep -- */

static void sweep_one(int len, int off)
{
    /* the allocation ends at the packet's last byte */
    uint8_t *buf = (uint8_t *)malloc((size_t)off + (size_t)len + (len == 0));
    uint8_t *p = buf + off;
    for (int i = 0; i < len; i++) p[i] = (uint8_t)rnd();
    if (len > 8 && (rnd() & 7u) == 0) memset(p, 0xff, (size_t)len); /* wrap-heavy */
    const int seed = (int)rnd();
    CHECK(sum_every_16bits(p, len) == oracle_sum_every_16bits(p, len), "sum len %d off %d", len, off);
    CHECK(checksum(p, len, seed) == oracle_checksum(p, len, seed), "csum len %d off %d", len, off);
    free(buf);
}

static void sweep(void)
{
    for (int len = 0; len <= 600; len++)
        for (int off = 0; off < 16; off++) sweep_one(len, off);
    const int big[] = {1499, 1500, 1501, 8999, 9000, 65535, 65536, 262147};
    for (size_t k = 0; k < sizeof big / sizeof big[0]; k++)
        for (int off = 0; off < 16; off++) sweep_one(big[k], off);
    CHECK(sum_every_16bits(NULL, 0) == 0 && sum_every_16bits(NULL, -5) == 0, "count <= 0");
    CHECK(checksum(NULL, 0, 0) == 0xffff, "empty");
}

/* ----------------------------------------------------------- 2. threads -- */

typedef struct {
    const uint8_t *buf;
    int len, id, bad;
} th_arg;

static void *th_main(void *p)
{
    th_arg *a = (th_arg *)p;
    for (int it = 0; it < 400; it++) {
        const int off = it & 15;
        int len = (it * 37 + a->id * 11) % a->len - off;
        if (len < 0) len = 0;
        const int seed = (int)((uint32_t)it * 0x01000193u + (uint32_t)a->id);
        if (checksum((void *)(a->buf + off), len, seed) != oracle_checksum(a->buf + off, len, seed))
            a->bad++;
        const uint16_t l16 = (uint16_t)(len > 20 ? len : 20);
        const uint32_t s = 0x0400000Au + (uint32_t)it, d = 0x0500000Au + (uint32_t)a->id;
        if (tcp_udp_checksum(s, d, 6, (uint8_t *)a->buf, l16) !=
            oracle_tcp_udp_checksum(s, d, 6, a->buf, l16))
            a->bad++;
    }
    return NULL;
}

static void threads(void)
{
    const int len = 9000;
    uint8_t *buf = (uint8_t *)malloc((size_t)len);
    for (int i = 0; i < len; i++) buf[i] = (uint8_t)rnd();
    pthread_t th[8];
    th_arg a[8];
    for (int t = 0; t < 8; t++) {
        a[t] = (th_arg){buf, len, t, 0};
        pthread_create(&th[t], NULL, th_main, &a[t]);
    }
    for (int t = 0; t < 8; t++) {
        pthread_join(th[t], NULL);
        CHECK(a[t].bad == 0, "thread %d: %d mismatches", t, a[t].bad);
    }
    free(buf);
}

/* ------------------------------------------------------------ 3. frames -- */

/* Ethernet + IPv4 (ihl 5..7) + TCP (20..40 B header) or ICMP, 10.0.0.1-120
 * addresses (no carry is lost in the reference's pseudo-header sum, so RX
 * verify of the TX result must pass), checksum fields holding junk. */
static lvlip_frame make_frame(int proto_tcp)
{
    const uint32_t ihl = 5u + rnd() % 3u;
    const uint32_t l4hdr = proto_tcp ? 20u + 4u * (rnd() % 6u) : 8u;
    const uint32_t pay = rnd() % 1461u;
    const uint32_t iplen = ihl * 4u + l4hdr + pay;
    const uint32_t flen = 14u + iplen;
    uint8_t *f = (uint8_t *)malloc(flen);
    for (uint32_t i = 0; i < flen; i++) f[i] = (uint8_t)rnd();
    f[12] = 0x08;
    f[13] = 0x00;
    uint8_t *ih = f + 14;
    ih[0] = (uint8_t)(0x40u | ihl);
    ih[2] = (uint8_t)(iplen >> 8);
    ih[3] = (uint8_t)iplen;
    ih[8] = 64;
    ih[9] = proto_tcp ? 6 : 1;
    ih[12] = 10, ih[13] = 0, ih[14] = 0, ih[15] = (uint8_t)(1u + rnd() % 120u);
    ih[16] = 10, ih[17] = 0, ih[18] = 0, ih[19] = (uint8_t)(1u + rnd() % 120u);
    if (proto_tcp) ih[ihl * 4u + 12u] = (uint8_t)((l4hdr / 4u) << 4);
    return (lvlip_frame){f, flen};
}

static void frames(void)
{
    const uint32_t n = 40000;
    lvlip_frame *fr = (lvlip_frame *)malloc(sizeof(lvlip_frame) * n);
    for (uint32_t i = 0; i < n; i++) fr[i] = make_frame((rnd() & 1u) != 0);
    lvlip_csum_ctx *ctx = (lvlip_csum_ctx *)(void *)&g_fail; /* opaque, unused by the stand-in */

    CHECK(lvlip_tx_checksum(ctx, fr, n) == LVLIP_OK, "tx");
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *ih = fr[i].head + 14;
        const uint32_t ihl = ih[0] & 15u, iplen = ((uint32_t)ih[2] << 8) | ih[3];
        CHECK(oracle_checksum(ih, (int)(ihl * 4u), 0) == 0, "frame %u: ip header", i);
        uint8_t *l4 = ih + ihl * 4u;
        const uint32_t l4len = iplen - ihl * 4u;
        if (ih[9] == 6) {
            uint16_t fld;
            memcpy(&fld, l4 + 16, 2);
            l4[16] = l4[17] = 0;
            uint32_t s, d;
            memcpy(&s, ih + 12, 4);
            memcpy(&d, ih + 16, 4);
            CHECK((uint16_t)oracle_tcp_udp_checksum(s, d, 6, l4, (uint16_t)l4len) == fld,
                  "frame %u: tcp", i);
            memcpy(l4 + 16, &fld, 2);
        } else {
            CHECK(oracle_checksum(l4, (int)l4len, 0) == 0, "frame %u: icmp", i);
        }
    }
    uint8_t *v = (uint8_t *)malloc(n);
    for (uint32_t flags = 0; flags <= LVLIP_RX_VERIFY_L4; flags++) {
        memset(v, 0, n);
        CHECK(lvlip_rx_verify(ctx, fr, n, flags, v) == LVLIP_OK, "rx");
        uint32_t ok = 0;
        for (uint32_t i = 0; i < n; i++) ok += v[i] == LVLIP_RX_OK;
        CHECK(ok == n, "rx flags %u: %u of %u ok", flags, ok, n);
    }

    /* malformed frames: each kind in the middle of a batch, in
     * an allocation that ends where the frame's len says */
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t at = n / 2u + k;
        const lvlip_frame keep = fr[at];
        lvlip_frame bad = make_frame(1);
        uint8_t *ih = bad.head + 14;
        uint8_t want_rx = 0;
        switch (k) {
        case 0: bad.len = 13; want_rx = LVLIP_RX_SHORT; break;      /* < Ethernet header */
        case 1: bad.len = 14 + 19; want_rx = LVLIP_RX_SHORT; break; /* < 20-B IPv4 header */
        case 2: ih[0] = 0x65; want_rx = LVLIP_RX_BAD_VERSION; break;
        case 3: ih[0] = 0x44; want_rx = LVLIP_RX_BAD_IHL; break;
        case 4: bad.len = 14 + (ih[0] & 15u) * 4u - 1u; want_rx = LVLIP_RX_SHORT; break;
        case 5: ih[2] = 0xff; ih[3] = 0xff; want_rx = 0xff; break; /* total length past the end */
        case 6: bad.head[12] = 0x86; bad.head[13] = 0xdd; want_rx = LVLIP_RX_NOT_IP; break;
        default: ih[8] = 0; want_rx = LVLIP_RX_TTL0; break;
        }
        uint8_t *exact = (uint8_t *)malloc(bad.len);
        memcpy(exact, bad.head, bad.len);
        free(bad.head);
        bad.head = exact;
        fr[at] = bad;
        if (k != 6 && k != 7) { /* 6 and 7 are well-formed IPv4 as far as TX cares */
            uint8_t *snap = (uint8_t *)malloc(bad.len);
            memcpy(snap, bad.head, bad.len);
            CHECK(lvlip_tx_checksum(ctx, fr, n) == LVLIP_EINVAL, "tx kind %u refused", k);
            CHECK(memcmp(snap, bad.head, bad.len) == 0, "tx kind %u untouched", k);
            free(snap);
        }
        CHECK(lvlip_rx_verify(ctx, fr, n, LVLIP_RX_VERIFY_L4, v) == LVLIP_OK, "rx kind %u", k);
        if (want_rx != 0xff)
            CHECK(v[at] == want_rx, "rx kind %u: verdict %u want %u", k, v[at], want_rx);
        else
            CHECK(v[at] != LVLIP_RX_OK, "rx kind %u accepted", k);
        CHECK(v[at - 1] == LVLIP_RX_OK && v[at + 1] == LVLIP_RX_OK, "rx kind %u neighbours", k);
        free(bad.head);
        fr[at] = keep;
    }
    CHECK(lvlip_rx_verify(ctx, fr, 0, 0, v) == LVLIP_OK && lvlip_tx_checksum(ctx, fr, 0) == LVLIP_OK,
          "n = 0");
    CHECK(lvlip_rx_verify(NULL, fr, n, 0, v) == LVLIP_EINVAL, "NULL ctx");
    for (uint32_t i = 0; i < n; i++) free(fr[i].head);
    free(fr);
    free(v);
}

/* 4. lvlip_partition_bytes (Group 4) on exact-size descriptor arrays against
 *    the definition: cut p is the first index whose byte prefix reaches
 *    p * T / parts (T the total of max(len, 0)), by count when T is 0. */
static void partition(void)
{
    for (int trial = 0; trial < 400; trial++) {
        const uint32_t n = rnd() % 700, parts = 1 + rnd() % 12;
        lvlip_csum_desc *d = malloc((n ? n : 1) * sizeof *d);
        uint32_t *cuts = malloc((parts + 1) * sizeof *cuts);
        unsigned __int128 total = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t k = rnd() % 10;
            d[i].offset = 0;
            d[i].len = k == 0 ? -(int32_t)(rnd() % 5) : k == 1 ? 0 : k == 2 ? 0x7fffffff : (int32_t)(rnd() % 9001);
            d[i].start_sum = 0;
            total += d[i].len > 0 ? (uint32_t)d[i].len : 0u;
        }
        CHECK(lvlip_partition_bytes(n ? d : NULL, n, parts, cuts) == LVLIP_OK, "partition rc");
        CHECK(cuts[0] == 0 && cuts[parts] == n, "partition ends");
        for (uint32_t p = 1; p < parts; p++) {
            uint32_t want = n;
            if (n == 0)
                want = 0;
            else if (total == 0)
                want = (uint32_t)((uint64_t)n * p / parts);
            else {
                const unsigned __int128 t = total * p / parts;
                unsigned __int128 pre = 0;
                for (uint32_t i = 0; i <= n; i++) {
                    if (pre >= t) {
                        want = i;
                        break;
                    }
                    if (i < n)
                        pre += d[i].len > 0 ? (uint32_t)d[i].len : 0u;
                }
            }
            CHECK(cuts[p] == want, "partition trial %d n %u parts %u cut %u: %u != %u", trial, n, parts, p,
                  cuts[p], want);
        }
        free(d);
        free(cuts);
    }
    CHECK(lvlip_partition_bytes(NULL, 3, 2, NULL) == LVLIP_EINVAL, "partition NULL");
}

int main(void)
{
    sweep();
    threads();
    frames();
    partition();
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("host_san: all checks passed\n");
    return 0;
}
