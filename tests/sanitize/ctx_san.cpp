// tests/sanitize/ctx_san.cpp — the host-resident GPU batch paths with
// AddressSanitizer on their host code (run on the MI355X box by
// tests/test_skb_gpu.py::test_host_batches_under_asan).
//
// TEST INFRASTRUCTURE ONLY.  tests/sanitize/Makefile compiles the product's
// own sources (csum_ctx.cpp, frames_host.cpp, skb_batch.c, csum_cpu.c,
// csum_kernels.hip) with `-Xarch_host -fsanitize=address` into one executable,
// so the context's pieces, slots, double-buffering, registered regions and the
// frame calls' gather, records and apply run under ASan against real GPU
// batches.  Every
// packet and frame sits in an allocation that ends at its last byte.  Results
// are checked against the oracle (oracle/csum_oracle.c).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <thread>
#include <vector>

#include <sanitizer/allocator_interface.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

extern "C" uint16_t oracle_checksum(const void* addr, int count, int start_sum);

static int g_fail = 0;
#define CHECK(c, ...)                                            \
    do {                                                         \
        if (!(c)) {                                              \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fputc('\n', stderr);                                 \
            if (++g_fail > 20) exit(1);                          \
        }                                                        \
    } while (0)

struct Rng {
    uint64_t s;
    uint32_t operator()() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (uint32_t)(s >> 33);
    }
};

// Scattered packets, each in its own exact-size allocation, through a context
// whose small arena forces many double-buffered pieces.
static void scattered(lvlip_csum_ctx* ctx, uint32_t n, uint32_t max_len, uint64_t seed) {
    Rng r{seed};
    std::vector<uint8_t*> mem(n);
    std::vector<lvlip_csum_iov> iov(n);
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t len = (r() % 97u == 0) ? -(int32_t)(r() % 5u) : (int32_t)(r() % (max_len + 1));
        const uint32_t off = r() % 16u;
        const size_t bytes = off + (len > 0 ? (size_t)len : 0) + (len <= 0);
        mem[i] = (uint8_t*)malloc(bytes);
        for (size_t b = 0; b < bytes; ++b) mem[i][b] = (uint8_t)r();
        iov[i].ptr = mem[i] + off;
        iov[i].len = len;
        iov[i].start_sum = r();
    }
    std::vector<uint16_t> out(n, 0);
    CHECK(lvlip_csum_batch_host(ctx, iov.data(), n, out.data()) == LVLIP_OK, "batch_host n=%u", n);
    for (uint32_t i = 0; i < n; ++i)
        CHECK(out[i] == oracle_checksum(iov[i].ptr, iov[i].len, (int)iov[i].start_sum),
              "scattered %u len %d", i, iov[i].len);
    for (auto* p : mem) free(p);
}

// One flat buffer that ends at the last packet's last byte (not a multiple of
// 16), packets at every alignment with gaps; optionally registered.
static void flat(lvlip_csum_ctx* ctx, uint32_t n, uint32_t max_len, uint64_t seed, int reg, uint32_t gap = 40,
                 bool shuffle = false) {
    Rng r{seed};
    std::vector<lvlip_csum_desc> d(n);
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        off += r() % gap;
        d[i].offset = off;
        d[i].len = (int32_t)(r() % (max_len + 1));
        d[i].start_sum = r();
        off += (uint64_t)d[i].len;
    }
    const size_t bytes = off ? off : 1;
    uint8_t* base = (uint8_t*)malloc(bytes);
    for (size_t b = 0; b < bytes; ++b) base[b] = (uint8_t)r();
    // out of address order: the span paths would cut one-packet pieces each
    // moving a whole span, so these go packet by packet (dense_ordered)
    if (shuffle)
        for (uint32_t i = n - 1; i > 0; --i) std::swap(d[i], d[r() % (i + 1)]);
    if (reg >= 0)
        CHECK(lvlip_csum_register(ctx, base, bytes, (uint32_t)reg) == LVLIP_OK, "register %d", reg);
    std::vector<uint16_t> out(n, 0);
    CHECK(lvlip_csum_batch_host_flat(ctx, base, bytes, d.data(), n, out.data()) == LVLIP_OK,
          "batch_host_flat n=%u reg=%d", n, reg);
    for (uint32_t i = 0; i < n; ++i)
        CHECK(out[i] == oracle_checksum(base + d[i].offset, d[i].len, (int)d[i].start_sum),
              "flat %u reg %d", i, reg);
    if (reg >= 0) {  // the same packets as an iov array inside the region: a flat
                     // batch over it when dense, else in place (zero-copy) or gathered (DMA)
        std::vector<lvlip_csum_iov> iov(n);
        for (uint32_t i = 0; i < n; ++i) iov[i] = {base + d[i].offset, d[i].len, d[i].start_sum};
        std::fill(out.begin(), out.end(), 0);
        CHECK(lvlip_csum_batch_host(ctx, iov.data(), n, out.data()) == LVLIP_OK, "zc batch_host");
        for (uint32_t i = 0; i < n; ++i)
            CHECK(out[i] == oracle_checksum(iov[i].ptr, iov[i].len, (int)iov[i].start_sum), "zc %u", i);
    }
    if (reg >= 0) CHECK(lvlip_csum_unregister(ctx, base) == LVLIP_OK, "unregister");
    free(base);
}

// One random well-formed frame (Ethernet + IPv4 ihl 5-7 + TCP or ICMP) at f,
// flen = frame_len(r) bytes; checksum fields hold junk.
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
    // 10.0.0.1-120: the reference's u32 pseudo-header sum keeps its carry
    ih[12] = 10, ih[13] = 0, ih[14] = 0, ih[15] = (uint8_t)(1u + r() % 120u);
    ih[16] = 10, ih[17] = 0, ih[18] = 0, ih[19] = (uint8_t)(1u + r() % 120u);
    if (tcp) ih[ihl * 4u + 12u] = (uint8_t)((l4hdr / 4u) << 4);
}

// TX then RX + L4 over the frames; every header must then sum to zero.
static void tx_rx_check(lvlip_csum_ctx* ctx, std::vector<lvlip_frame>& fr, const char* what) {
    const uint32_t n = (uint32_t)fr.size();
    CHECK(lvlip_tx_checksum(ctx, fr.data(), n) == LVLIP_OK, "%s: tx", what);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* ih = fr[i].head + 14;
        CHECK(oracle_checksum(ih, (ih[0] & 15) * 4, 0) == 0, "%s: frame %u header", what, i);
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

// f1/f2 frame calls with a real context: exact-size scattered frames, TX then
// RX; then one malformed frame in the middle, which must leave every frame
// untouched.
static void frame_calls(lvlip_csum_ctx* ctx, uint32_t n, uint64_t seed) {
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
    tx_rx_check(ctx, fr, "scattered");
    fr[n / 2].head[14] = 0x65;                   // version 6
    for (auto& f : fr) f.head[14 + 10] ^= 0x5a;  // stale header fields
    std::vector<uint8_t> snap;
    for (auto& f : fr) snap.insert(snap.end(), f.head, f.head + f.len);
    CHECK(lvlip_tx_checksum(ctx, fr.data(), n) == LVLIP_EINVAL, "malformed refused");
    size_t o = 0;
    bool same = true;
    for (auto& f : fr) {
        same = same && memcmp(snap.data() + o, f.head, f.len) == 0;
        o += f.len;
    }
    CHECK(same, "malformed: frames untouched");
    std::vector<uint8_t> v(n, 0);
    CHECK(lvlip_rx_verify(ctx, fr.data(), n, LVLIP_RX_VERIFY_L4, v.data()) == LVLIP_OK, "rx malformed");
    CHECK(v[n / 2] == LVLIP_RX_BAD_VERSION, "rx malformed verdict %u", v[n / 2]);
    for (auto& f : fr) free(f.head);
}

// The same frames packed into one slab (an allocation ending at the last
// frame's last byte, frames at every alignment, in shuffled order),
// registered in `reg` mode (DMA: the copy engine reads spans; ZEROCOPY: the
// kernel reads in place), and as received skbs: BUFLEN-long buffers holding
// shorter frames (src/netdev.c:89-91), unregistered.
static void frame_slab(lvlip_csum_ctx* ctx, uint32_t n, uint64_t seed, int reg, uint32_t gap = 24) {
    Rng r{seed};
    std::vector<uint32_t> len(n), off(n);
    std::vector<bool> tcp(n);
    std::vector<uint32_t> ihl(n), l4h(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        bool t;
        len[i] = frame_len(r, t, ihl[i], l4h[i]);
        tcp[i] = t;
        pos += r() % gap;
        off[i] = (uint32_t)pos;
        pos += len[i];
    }
    uint8_t* slab = (uint8_t*)malloc(pos);
    for (uint32_t i = 0; i < n; ++i) fill_frame(r, slab + off[i], len[i], tcp[i], ihl[i], l4h[i]);
    if (reg >= 0) CHECK(lvlip_csum_register(ctx, slab, pos, (uint32_t)reg) == LVLIP_OK, "register frames");
    std::vector<lvlip_frame> fr(n);
    for (uint32_t i = 0; i < n; ++i) fr[i] = {slab + off[i], len[i]};
    for (uint32_t i = n - 1; i > 0; --i) std::swap(fr[i], fr[r() % (i + 1)]);
    tx_rx_check(ctx, fr, reg < 0 ? "slab" : reg == (int)LVLIP_REG_DMA ? "slab dma" : "slab zerocopy");
    if (reg >= 0) CHECK(lvlip_csum_unregister(ctx, slab) == LVLIP_OK, "unregister frames");
    // as skbs from netdev_rx_loop: the frame at the start of a 1600-B buffer,
    // the buffer's end as the frame's end
    if (reg < 0) {
        const uint32_t buflen = 1600, m = n < 2000 ? n : 2000;
        uint8_t* skbs = (uint8_t*)calloc((size_t)m, buflen);
        std::vector<lvlip_frame> sk(m);
        for (uint32_t i = 0; i < m; ++i) {
            const uint32_t l = len[i] < buflen ? len[i] : buflen;
            memcpy(skbs + (size_t)i * buflen, slab + off[i], l);
            sk[i] = {skbs + (size_t)i * buflen, buflen};
        }
        std::vector<uint8_t> v(m, 0);
        CHECK(lvlip_rx_verify(ctx, sk.data(), m, LVLIP_RX_VERIFY_L4, v.data()) == LVLIP_OK, "rx skbs");
        for (uint32_t i = 0; i < m; ++i)
            CHECK(v[i] == (len[i] <= buflen ? LVLIP_RX_OK : LVLIP_RX_SHORT), "rx skb %u: %u", i, v[i]);
        free(skbs);
    }
    free(slab);
}

int main() {
    printf("build_id: %s\n", lvlip_build_id());
    if (lvlip_device_count() < 1) {
        fprintf(stderr, "no HIP device\n");
        return 2;
    }
    lvlip_csum_ctx* ctx = nullptr;
    // this context's host steps on its pool threads whatever the call's size
    // (LVLIP_INLINE_MAX 0); the per-thread contexts below keep the default
    // (calls of up to 32 768 items on the calling thread)
    setenv("LVLIP_INLINE_MAX", "0", 1);
    CHECK(lvlip_csum_ctx_create(&ctx, 0, 1u << 20) == LVLIP_OK, "ctx_create");
    unsetenv("LVLIP_INLINE_MAX");
    scattered(ctx, 20000, 3000, 1);   // ~30 MB through a 1 MiB arena: many pieces
    scattered(ctx, 3, 9000, 2);
    flat(ctx, 20000, 1600, 3, -1);
    flat(ctx, 20000, 1600, 4, (int)LVLIP_REG_DMA);
    flat(ctx, 5000, 1600, 5, (int)LVLIP_REG_ZEROCOPY);
    // packets spread thinly over a zero-copy region: read in place (a dense
    // batch moves as spans, as from a DMA region)
    flat(ctx, 3000, 1600, 11, (int)LVLIP_REG_ZEROCOPY, 8192);
    // shuffled descriptors over a slab far larger than the arena: gathered
    flat(ctx, 20000, 1600, 12, -1, 40, true);
    flat(ctx, 20000, 1600, 13, (int)LVLIP_REG_DMA, 40, true);
    frame_calls(ctx, 20000, 6);
    frame_slab(ctx, 20000, 7, -1);
    frame_slab(ctx, 20000, 8, (int)LVLIP_REG_DMA);
    frame_slab(ctx, 5000, 9, (int)LVLIP_REG_ZEROCOPY);
    // frames spread thinly over a zero-copy region (gaps of up to 8 KiB): read
    // in place rather than moved as spans
    frame_slab(ctx, 3000, 10, (int)LVLIP_REG_ZEROCOPY, 8192);

    // the CPU side of the threshold (lvlip_csum_ctx_set_cpu_max): the same
    // kinds of batches on the calling thread, over exact-size allocations
    {
        lvlip_ctx_stats s0, s1;
        CHECK(lvlip_csum_ctx_stats(ctx, &s0) == LVLIP_OK, "stats");
        CHECK(lvlip_csum_ctx_set_cpu_max(ctx, 1u << 30) == LVLIP_OK && lvlip_csum_ctx_cpu_max(ctx) == (1u << 30),
              "cpu_max");
        scattered(ctx, 3000, 3000, 21);
        flat(ctx, 3000, 1600, 22, -1);
        frame_calls(ctx, 3000, 23);
        frame_slab(ctx, 3000, 24, -1);
        CHECK(lvlip_csum_ctx_stats(ctx, &s1) == LVLIP_OK && s1.gpu_calls == s0.gpu_calls &&
                  s1.cpu_calls > s0.cpu_calls,
              "cpu side: %llu gpu calls", (unsigned long long)(s1.gpu_calls - s0.gpu_calls));
        CHECK(lvlip_csum_ctx_set_cpu_max(ctx, 0) == LVLIP_OK, "cpu_max 0");
    }

    // a packet larger than the arena is refused; nothing is read
    std::vector<uint8_t> big((2u << 20) + 5u, 0xab);
    lvlip_csum_iov one{big.data(), (int32_t)big.size(), 0};
    uint16_t o = 0;
    CHECK(lvlip_csum_batch_host(ctx, &one, 1, &o) == LVLIP_ERANGE, "oversize");
    // argument errors
    CHECK(lvlip_csum_batch_host(nullptr, &one, 1, &o) == LVLIP_EINVAL, "null ctx");
    CHECK(lvlip_csum_batch_host(ctx, nullptr, 0, nullptr) == LVLIP_OK, "n = 0");
    lvlip_csum_desc bad{10, 20, 0};
    CHECK(lvlip_csum_batch_host_flat(ctx, big.data(), 25, &bad, 1, &o) == LVLIP_EINVAL, "flat bounds");
    // the up-front checks run on the pool threads over ranges of the batch
    // (first_failure): the refusal is still the first bad descriptor's, in
    // batch order, whichever thread sees which (n spans several ranges)
    {
        const uint32_t n = 400000;
        std::vector<lvlip_csum_desc> d(n, lvlip_csum_desc{0, 64, 0});
        std::vector<uint16_t> out(n);
        lvlip_csum_desc past{big.size() - 8, 16, 0};              // past base_bytes: EINVAL
        lvlip_csum_desc huge{0, (int32_t)(big.size() - 16), 0};  // span > the 1 MiB arena: ERANGE
        d[300001] = past;
        d[350002] = huge;
        CHECK(lvlip_csum_batch_host_flat(ctx, big.data(), big.size(), d.data(), n, out.data()) == LVLIP_EINVAL,
              "first bad descriptor EINVAL");
        d[100003] = huge;
        CHECK(lvlip_csum_batch_host_flat(ctx, big.data(), big.size(), d.data(), n, out.data()) == LVLIP_ERANGE,
              "first bad descriptor ERANGE");
        std::vector<lvlip_csum_iov> iov(n, lvlip_csum_iov{big.data(), 64, 0});
        iov[200000] = lvlip_csum_iov{nullptr, 8, 0};
        CHECK(lvlip_csum_batch_host(ctx, iov.data(), n, out.data()) == LVLIP_EINVAL, "null iov refused");
        iov[200000] = one;
        CHECK(lvlip_csum_batch_host(ctx, iov.data(), n, out.data()) == LVLIP_ERANGE, "oversize iov refused");
    }

    // a region left registered is released by destroy
    uint8_t* left = (uint8_t*)malloc(1u << 16);
    CHECK(lvlip_csum_register(ctx, left, 1u << 16, LVLIP_REG_DMA) == LVLIP_OK, "register left");
    CHECK(lvlip_csum_ctx_destroy(ctx) == LVLIP_OK, "destroy");
    free(left);

    // Group 4: one batch over three contexts, a host thread each
    // (lvlip_csum_batch_host_flat_multi; every part's span gathered from one
    // buffer that ends at its last packet's last byte)
    {
        Rng r{300};
        const uint32_t n = 30000;
        std::vector<lvlip_csum_desc> d(n);
        uint64_t off = 0;
        for (uint32_t i = 0; i < n; ++i) {
            off += r() % 24u;
            d[i].offset = off;
            d[i].len = (r() % 61u == 0) ? -(int32_t)(r() % 3u) : (int32_t)(r() % 1601u);
            d[i].start_sum = r();
            off += d[i].len > 0 ? (uint64_t)d[i].len : 0u;
        }
        const size_t bytes = off ? off : 1;
        uint8_t* base = (uint8_t*)malloc(bytes);
        for (size_t b = 0; b < bytes; ++b) base[b] = (uint8_t)r();
        lvlip_csum_ctx* mc[3] = {nullptr, nullptr, nullptr};
        for (auto& c : mc) CHECK(lvlip_csum_ctx_create(&c, 0, 1u << 20) == LVLIP_OK, "multi ctx");
        std::vector<uint16_t> out(n, 0);
        CHECK(lvlip_csum_batch_host_flat_multi(mc, 3, base, bytes, d.data(), n, out.data()) == LVLIP_OK,
              "batch_host_flat_multi");
        for (uint32_t i = 0; i < n; ++i)
            CHECK(out[i] == oracle_checksum(base + d[i].offset, d[i].len, (int)d[i].start_sum), "multi %u", i);
        uint32_t cuts[4];
        CHECK(lvlip_partition_bytes(d.data(), n, 3, cuts) == LVLIP_OK && cuts[0] == 0 && cuts[3] == n,
              "partition");
        for (auto& c : mc) CHECK(lvlip_csum_ctx_destroy(c) == LVLIP_OK, "multi destroy");
        free(base);
    }

    // one context per thread, concurrently (src/main.c:83-89 threads)
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([t] {
            lvlip_csum_ctx* c = nullptr;
            CHECK(lvlip_csum_ctx_create(&c, 0, 1u << 20) == LVLIP_OK, "thread ctx");
            scattered(c, 4000, 2000, 100 + t);
            flat(c, 4000, 1600, 200 + t, t & 1 ? (int)LVLIP_REG_DMA : -1);
            CHECK(lvlip_csum_ctx_destroy(c) == LVLIP_OK, "thread destroy");
        });
    for (auto& x : th) x.join();

    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("ctx_san: all checks passed\n");
    fflush(stdout);
    // Why the process used to abort at exit (sanitizer_allocator_device.h:125
    // under libhsa-runtime64's __cxa_finalize): with ASan, hipFree's HSA pool
    // frees go through ASan's device allocator, which parks every freed device
    // chunk in the quarantine.  The contexts above freed their arenas there.
    // During the HSA runtime's own teardown its frees push the quarantine over
    // its limit, and ASan recycles the oldest parked chunks by calling back
    // into an HSA runtime that is already half torn down: the CHECK on that
    // free fails.  Nothing in the library frees device memory from a static
    // destructor (every context is destroyed explicitly above).  So drain the
    // quarantine now, while HSA is fully alive: the parked chunks are really
    // freed here, and the teardown's own frees no longer overflow it.
    __sanitizer_purge_allocator();
    return 0;
}
