// tests/sanitize/frames_san.cpp — TEST INFRASTRUCTURE ONLY: the host frame
// calls (level-ip_amd/csrc/frames_host.cpp) and the host context
// (csum_ctx.cpp) under ASan + UBSan and under TSan on the CPU, over the HIP
// stand-in of tests/sanitize/hip_emu.cpp (tests/test_sanitize_host.py).
//
// Every frame sits in an allocation that ends at its last byte.  Contexts have
// a 1 MiB arena (many pieces), once reading the arena in place and once through
// the copies (LVLIP_DIRECT_MAX=0); frames come scattered, in a slab registered
// for DMA and for zero-copy (shuffled order), as BUFLEN-long RX skbs, with a
// malformed frame in a late piece (every frame must come back untouched), and
// from three contexts on three threads at once.  One more slab per kind is
// registered from an address that is not 16-B aligned, with the bytes before
// it poisoned under ASan: no copy may start before a region's first byte.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

#if defined(__SANITIZE_ADDRESS__)  // gcc's -fsanitize=address (the test builds with g++)
#include <sanitizer/asan_interface.h>
#define POISON(p, n) __asan_poison_memory_region((p), (n))
#define UNPOISON(p, n) __asan_unpoison_memory_region((p), (n))
#endif
#ifndef POISON
#define POISON(p, n) ((void)(p), (void)(n))
#define UNPOISON(p, n) ((void)(p), (void)(n))
#endif

extern "C" uint16_t oracle_checksum(const void* addr, int count, int start_sum);
extern "C" int oracle_tcp_udp_checksum(uint32_t saddr, uint32_t daddr, uint8_t proto, const uint8_t* data,
                                       uint16_t len);

static int g_fail = 0;
#define CHECK(c, ...)                                            \
    do {                                                         \
        if (!(c)) {                                              \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fputc('\n', stderr);                                 \
            if (__atomic_add_fetch(&g_fail, 1, __ATOMIC_RELAXED) > 20) exit(1); \
        }                                                        \
    } while (0)

struct Rng {
    uint64_t s;
    uint32_t operator()() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(s >> 33);
    }
};

// Ethernet + IPv4 (ihl 5-7) + TCP (20-40 B header) or ICMP, 10.0.0.1-120
// (no carry lost in the reference's pseudo-header sum), fields junk.
static uint32_t frame_len(Rng& r, bool& tcp, uint32_t& ihl, uint32_t& l4hdr) {
    tcp = r() & 1u;
    ihl = 5u + r() % 3u;
    l4hdr = tcp ? 20u + 4u * (r() % 6u) : 8u;
    return 14u + ihl * 4u + l4hdr + r() % 1461u;
}
static void fill_frame(Rng& r, uint8_t* f, uint32_t flen, bool tcp, uint32_t ihl, uint32_t l4hdr) {
    const uint32_t iplen = flen - 14u;
    for (uint32_t b = 0; b < flen; ++b) f[b] = (uint8_t)r();
    f[12] = 0x08, f[13] = 0x00;
    uint8_t* ih = f + 14;
    ih[0] = (uint8_t)(0x40u | ihl), ih[2] = (uint8_t)(iplen >> 8), ih[3] = (uint8_t)iplen;
    ih[8] = 64, ih[9] = tcp ? 6 : 1;
    ih[12] = 10, ih[13] = 0, ih[14] = 0, ih[15] = (uint8_t)(1u + r() % 120u);
    ih[16] = 10, ih[17] = 0, ih[18] = 0, ih[19] = (uint8_t)(1u + r() % 120u);
    if (tcp) ih[ihl * 4u + 12u] = (uint8_t)((l4hdr / 4u) << 4);
}

// After TX: every frame's fields are the reference's (src/tcp.c:87-98,
// src/icmpv4.c:46-47, src/ip_output.c:8-12), and RX accepts every frame.
static void check_filled(lvlip_csum_ctx* ctx, std::vector<lvlip_frame>& fr, const char* what) {
    const uint32_t n = (uint32_t)fr.size();
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* ih = fr[i].head + 14;
        const uint32_t ihl = ih[0] & 15u, iplen = ((uint32_t)ih[2] << 8) | ih[3];
        CHECK(oracle_checksum(ih, (int)(ihl * 4u), 0) == 0, "%s: frame %u ip header", what, i);
        uint8_t* l4 = ih + ihl * 4u;
        const uint32_t l4len = iplen - ihl * 4u;
        if (ih[9] == 6) {
            uint16_t fld;
            memcpy(&fld, l4 + 16, 2);
            uint8_t save[2] = {l4[16], l4[17]};
            l4[16] = l4[17] = 0;
            uint32_t s, d;
            memcpy(&s, ih + 12, 4);
            memcpy(&d, ih + 16, 4);
            CHECK((uint16_t)oracle_tcp_udp_checksum(s, d, 6, l4, (uint16_t)l4len) == fld, "%s: frame %u tcp", what, i);
            l4[16] = save[0], l4[17] = save[1];
        } else {
            CHECK(oracle_checksum(l4, (int)l4len, 0) == 0, "%s: frame %u icmp", what, i);
        }
    }
    std::vector<uint8_t> v(n, 0);
    for (uint32_t flags = 0; flags <= LVLIP_RX_VERIFY_L4; ++flags) {
        std::fill(v.begin(), v.end(), 0);
        CHECK(lvlip_rx_verify(ctx, fr.data(), n, flags, v.data()) == LVLIP_OK, "%s: rx", what);
        uint32_t ok = 0;
        for (uint32_t i = 0; i < n; ++i) ok += v[i] == LVLIP_RX_OK;
        CHECK(ok == n, "%s: rx flags %u: %u of %u ok", what, flags, ok, n);
    }
}

static void scattered(lvlip_csum_ctx* ctx, uint32_t n, uint64_t seed) {
    Rng r{seed};
    std::vector<lvlip_frame> fr(n);
    for (uint32_t i = 0; i < n; ++i) {
        bool tcp;
        uint32_t ihl, l4hdr;
        const uint32_t flen = frame_len(r, tcp, ihl, l4hdr);
        uint8_t* f = (uint8_t*)malloc(flen);
        fill_frame(r, f, flen, tcp, ihl, l4hdr);
        fr[i] = {f, flen};
    }
    CHECK(lvlip_tx_checksum(ctx, fr.data(), n) == LVLIP_OK, "scattered tx");
    check_filled(ctx, fr, "scattered");
    // a malformed frame in a late piece: the earlier pieces were already
    // written, and must be restored
    fr[n - n / 8].head[14] = 0x65;
    for (auto& f : fr) f.head[24] ^= 0x5a;
    std::vector<uint8_t> snap;
    for (auto& f : fr) snap.insert(snap.end(), f.head, f.head + f.len);
    CHECK(lvlip_tx_checksum(ctx, fr.data(), n) == LVLIP_EINVAL, "malformed refused");
    size_t o = 0;
    uint32_t changed = 0;
    for (auto& f : fr) {
        changed += memcmp(snap.data() + o, f.head, f.len) != 0;
        o += f.len;
    }
    CHECK(changed == 0, "malformed: %u frames changed", changed);
    for (auto& f : fr) free(f.head);
}

// lead > 0: the region starts lead bytes into its allocation (not 16-B
// aligned), the first frame at its first byte, the lead bytes poisoned (ASan
// poisons whole 8-B granules from the allocation's start: lead 13 poisons
// the first 8, which a span rounded down to 16 from address 0 would read).
static void slab(lvlip_csum_ctx* ctx, uint32_t n, uint64_t seed, uint32_t reg, uint32_t lead = 0) {
    Rng r{seed};
    std::vector<uint32_t> len(n), off(n), ihl(n), l4h(n);
    std::vector<bool> tcp(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        bool t;
        len[i] = frame_len(r, t, ihl[i], l4h[i]);
        tcp[i] = t;
        if (i || !lead) pos += r() % 24u;
        off[i] = (uint32_t)pos;
        pos += len[i];
    }
    uint8_t* raw = (uint8_t*)malloc(lead + pos);
    uint8_t* s = raw + lead;
    POISON(raw, lead);
    for (uint32_t i = 0; i < n; ++i) fill_frame(r, s + off[i], len[i], tcp[i], ihl[i], l4h[i]);
    CHECK(lvlip_csum_register(ctx, s, pos, reg) == LVLIP_OK, "register");
    std::vector<lvlip_frame> fr(n);
    for (uint32_t i = 0; i < n; ++i) fr[i] = {s + off[i], len[i]};
    for (uint32_t i = n - 1; i > 0; --i) std::swap(fr[i], fr[r() % (i + 1)]);
    CHECK(lvlip_tx_checksum(ctx, fr.data(), n) == LVLIP_OK, "slab tx reg %u", reg);
    check_filled(ctx, fr, reg == LVLIP_REG_DMA ? "slab dma" : "slab zerocopy");
    CHECK(lvlip_csum_unregister(ctx, s) == LVLIP_OK, "unregister");
    // as received skbs: each frame at the start of a BUFLEN (1600-B) buffer
    // whose end is the frame's end, garbage past the IP total length, some
    // total lengths past the buffer
    const uint32_t m = n < 3000 ? n : 3000, buflen = 1600;
    std::vector<uint8_t*> bufs(m);
    std::vector<lvlip_frame> sk(m);
    std::vector<uint8_t> want(m);
    for (uint32_t i = 0; i < m; ++i) {
        bufs[i] = (uint8_t*)malloc(buflen);
        for (uint32_t b = 0; b < buflen; ++b) bufs[i][b] = (uint8_t)r();
        const uint32_t l = len[i] < buflen ? len[i] : buflen;
        memcpy(bufs[i], s + off[i], l);
        want[i] = len[i] <= buflen ? LVLIP_RX_OK : LVLIP_RX_SHORT;
        if (i % 97 == 5) {  // total length past the buffer, the header checksum fixed up
            uint8_t* ih = bufs[i] + 14;
            ih[2] = 0x07, ih[3] = 0xd0, ih[10] = ih[11] = 0;
            const uint16_t c = oracle_checksum(ih, (int)((ih[0] & 15u) * 4u), 0);
            memcpy(ih + 10, &c, 2);
            want[i] = LVLIP_RX_SHORT;
        }
        sk[i] = {bufs[i], buflen};
    }
    std::vector<uint8_t> v(m, 0);
    CHECK(lvlip_rx_verify(ctx, sk.data(), m, LVLIP_RX_VERIFY_L4, v.data()) == LVLIP_OK, "rx skbs");
    for (uint32_t i = 0; i < m; ++i) CHECK(v[i] == want[i], "rx skb %u: %u want %u", i, v[i], want[i]);
    for (auto* b : bufs) free(b);
    UNPOISON(raw, lead);
    free(raw);
}

// The packet batches of the same context (csum_ctx.cpp): scattered exact-size
// packets at every alignment (lvlip_csum_batch_host: a gather per packet) and
// one flat buffer ending at its last packet's last byte (a gather per span).
static void packets(lvlip_csum_ctx* ctx, uint32_t n, uint64_t seed) {
    Rng r{seed};
    std::vector<uint8_t*> mem(n);
    std::vector<lvlip_csum_iov> iov(n);
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t len = (r() % 97u == 0) ? -(int32_t)(r() % 5u) : (int32_t)(r() % 3001u);
        const uint32_t off = r() % 16u;
        const size_t bytes = off + (len > 0 ? (size_t)len : 0) + (len <= 0);
        mem[i] = (uint8_t*)malloc(bytes);
        for (size_t b = 0; b < bytes; ++b) mem[i][b] = (uint8_t)r();
        iov[i] = {mem[i] + off, len, r()};
    }
    std::vector<uint16_t> out(n, 0);
    CHECK(lvlip_csum_batch_host(ctx, iov.data(), n, out.data()) == LVLIP_OK, "batch_host");
    for (uint32_t i = 0; i < n; ++i)
        CHECK(out[i] == oracle_checksum(iov[i].ptr, iov[i].len, (int)iov[i].start_sum), "batch_host %u", i);
    for (auto* p : mem) free(p);
    std::vector<lvlip_csum_desc> d(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        pos += r() % 40u;
        d[i] = {pos, (int32_t)(r() % 1601u), r()};
        pos += (uint64_t)d[i].len;
    }
    uint8_t* base = (uint8_t*)malloc(pos ? pos : 1);
    for (uint64_t b = 0; b < pos; ++b) base[b] = (uint8_t)r();
    CHECK(lvlip_csum_batch_host_flat(ctx, base, pos, d.data(), n, out.data()) == LVLIP_OK, "batch_host_flat");
    for (uint32_t i = 0; i < n; ++i)
        CHECK(out[i] == oracle_checksum(base + d[i].offset, d[i].len, (int)d[i].start_sum), "flat %u", i);
    free(base);
}

int main() {
    for (int direct = 0; direct < 2; ++direct) {
        // direct: pieces read in place; else through the H2D / D2H copies.
        // And the host steps on the pool (LVLIP_INLINE_MAX 0) or, for calls
        // of up to 32 768 items, on the calling thread (the default)
        setenv("LVLIP_DIRECT_MAX", direct ? "4194304" : "0", 1);
        setenv("LVLIP_INLINE_MAX", direct ? "32768" : "0", 1);
        lvlip_csum_ctx* ctx = nullptr;
        CHECK(lvlip_csum_ctx_create(&ctx, 0, 1u << 20) == LVLIP_OK, "ctx_create");
        scattered(ctx, 12000, 1 + direct);
        packets(ctx, 12000, 7 + direct);
        slab(ctx, 12000, 3 + direct, LVLIP_REG_DMA);
        slab(ctx, 6000, 5 + direct, LVLIP_REG_ZEROCOPY);
        slab(ctx, 4000, 9 + direct, LVLIP_REG_DMA, 13);
        slab(ctx, 4000, 13 + direct, LVLIP_REG_ZEROCOPY, 13);
        CHECK(lvlip_csum_ctx_destroy(ctx) == LVLIP_OK, "destroy");
    }
    unsetenv("LVLIP_DIRECT_MAX");
    setenv("LVLIP_INLINE_MAX", "0", 1);  // the threads below use their pools
    // one context per thread, at once (the reference's core, IPC and timer
    // threads, src/main.c:83-89)
    std::vector<std::thread> th;
    for (int t = 0; t < 3; ++t)
        th.emplace_back([t] {
            lvlip_csum_ctx* c = nullptr;
            CHECK(lvlip_csum_ctx_create(&c, 0, 1u << 20) == LVLIP_OK, "thread ctx");
            scattered(c, 4000, 100 + t);
            CHECK(lvlip_csum_ctx_destroy(c) == LVLIP_OK, "thread destroy");
        });
    for (auto& x : th) x.join();
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("frames_san: all checks passed\n");
    return 0;
}
