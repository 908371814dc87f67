// csum_ctx.cpp — Group 3 of include/lvlip_csum.h: host-resident batches.
//
// level-ip's packets live in malloc'd skb heads (src/skbuff.c:5-20) at offsets
// 14 (IPv4 header, include/ip.h:47-50) and 34 (TCP/ICMP, include/tcp.h:224-227),
// i.e. 2 mod 4.  The context's slots, arenas and streams are described in
// ctx_impl.h; the host frame calls over the same context are frames_host.cpp.
//
// One context belongs to one thread at a time (no locks on the hot path):
// the reference calls checksum() from the core, IPC and timer threads
// (src/main.c:83-89, src/timer.c:74), so each gets its own context.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "ctx_impl.h"

namespace {

constexpr size_t kDefaultArena = 64ull << 20;
constexpr uint64_t kDirectMax = 4ull << 20;  // measured: DESIGN.md §5
constexpr uint64_t kPieceMax = 32ull << 20;  // measured: DESIGN.md §5
constexpr uint64_t kBlockMin = 4ull << 20;   // ~80 us of PCIe: DESIGN.md §9

}  // namespace

namespace lvlip_ctx {

int fail(lvlip_csum_ctx* c, hipError_t e, const char* what, int code) {
    char msg[256];
    snprintf(msg, sizeof msg, "%s: %s", what, hipGetErrorString(e));
    if (c) snprintf(c->err, sizeof c->err, "%s", msg);
    lvlip_set_last_hip_error(msg);  // what lvlip_last_hip_error() returns on this thread
    fprintf(stderr, "lvlip_csum: %s\n", msg);
    return code;
}

int drain(lvlip_csum_ctx* c, Slot& s) {
    if (!s.busy) return LVLIP_OK;
    hipError_t e = hipSuccess;
    if (s.sleep) {
        // hipEventSynchronize spins (with or without hipEventBlockingSync, as
        // measured: DESIGN.md §9), so a long piece is polled between 20-us sleeps
        const timespec nap{0, 20000};
        while ((e = hipEventQuery(s.done)) == hipErrorNotReady) nanosleep(&nap, nullptr);
    }
    if (e == hipSuccess) e = hipEventSynchronize(s.done);
    s.busy = false;
    if (e != hipSuccess) return fail(c, e, "hipEventSynchronize");
    memcpy(s.user_out, s.h_out, s.out_bytes);
    return LVLIP_OK;
}

int count_piece(lvlip_csum_ctx* c, uint64_t bytes) {
    c->stats.pieces++;
    c->stats.h2d_bytes += bytes;
    if (c->fail_piece && ++c->call_pieces == c->fail_piece)
        return fail(c, hipErrorLaunchFailure, "injected failure (LVLIP_FAIL_PIECE)");
    return LVLIP_OK;
}

int arm_slot(lvlip_csum_ctx* c, Slot& s, void* user_out, size_t out_bytes, uint64_t piece_bytes) {
    const hipError_t e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) return fail(c, e, "hipEventRecord");
    s.sleep = c->block_min && piece_bytes >= c->block_min;
    s.user_out = user_out;
    s.out_bytes = out_bytes;
    s.busy = true;
    return LVLIP_OK;
}

// Two slots' copies issued on their own streams run side by side, share the
// link and finish together; each slot's kernel and result copy then ran with
// the link idle, 8.5 % of a registered batch's time (the pipeline's trace,
// DESIGN.md §5).  Each piece's copy now waits for the previous piece's (the
// other slot's) copy event, so the copies run one after the other in issue
// order and each piece is summed while the next one's copy runs.  The first
// piece of a call waits for nothing: a cross-stream wait in front of a
// call's only piece cost small batches up to ~0.5 ms (a copy stream shared
// by both slots, tried first, did that for every piece).
int h2d_ordered(lvlip_csum_ctx* c, Slot& s, void* dst, const void* src, size_t n, const char* what) {
    hipError_t e;
    if (c->copy_order && c->last_copy && c->last_copy != &s &&
        (e = hipStreamWaitEvent(s.stream, c->last_copy->copied, 0)) != hipSuccess)
        return fail(c, e, "hipStreamWaitEvent");
    if ((e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s.stream)) != hipSuccess) return fail(c, e, what);
    if (c->copy_order) {
        if ((e = hipEventRecord(s.copied, s.stream)) != hipSuccess) return fail(c, e, "hipEventRecord");
        c->last_copy = &s;
    }
    return LVLIP_OK;
}

int finish_pieces(lvlip_csum_ctx* c, int rc) {
    for (auto& s : c->slot) {
        const int r2 = drain(c, s);
        if (rc == LVLIP_OK) rc = r2;
    }
    if (rc != LVLIP_OK)
        for (auto& s : c->slot) (void)hipStreamSynchronize(s.stream);
    c->last_copy = nullptr;  // the next call's first piece waits for nothing
    return rc;
}

const Region* find_region(const lvlip_csum_ctx* c, const void* p, uint64_t len) {
    const uint8_t* a = (const uint8_t*)p;
    for (const Region& r : c->regions)
        if (a >= r.host && a + len <= r.host + r.bytes) return &r;
    return nullptr;
}

}  // namespace lvlip_ctx

namespace {

using namespace lvlip_ctx;

void free_slot(Slot& s) {
    if (s.h_bytes) (void)hipHostFree(s.h_bytes);
    if (s.h_desc) (void)hipHostFree(s.h_desc);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_bytes) (void)hipFree(s.d_bytes);
    if (s.d_desc) (void)hipFree(s.d_desc);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Slot{};
}

// Copy a piece to the device, checksum it, copy results back.  The bytes come
// from `src` (the slot's pinned arena, or a registered region: DMA straight
// from it), or, when `dev_base` is set, are read by the kernel in place
// (zero-copy: `bytes` is then only the length hint's numerator).
int launch_piece(lvlip_csum_ctx* c, Slot& s, uint64_t bytes, uint32_t count, uint16_t* user_out,
                 const uint8_t* src = nullptr, const uint8_t* dev_base = nullptr) {
    hipError_t e;
    if (const int rc = count_piece(c, bytes); rc != LVLIP_OK) return rc;
    lvlip_launch_cfg cfg{};
    cfg.kernel = LVLIP_KERNEL_AUTO;  // the piece's average length picks the kernel
    cfg.len_hint = (int32_t)(bytes / count > 0x7fffffffull ? 0x7fffffff : bytes / count);
    if (dev_base && cfg.len_hint >= 896) {
        // packets read in place over PCIe: the flat sweep (U 8) reads them
        // faster than the stream kernel AUTO picks from 896 B for HBM
        // (scripts/lab_zerocopy.py)
        cfg.kernel = LVLIP_KERNEL_FLAT;
        cfg.unroll = 8;
    }
    if (bytes <= c->direct_max && (dev_base || !src || src == s.h_bytes)) {
        // A small piece: the copies' fixed costs (an SDMA round trip each way)
        // outweigh moving the bytes, so the kernel reads the pinned arena (or
        // the zero-copy region) and the descriptors over PCIe and writes the
        // results straight into the pinned result buffer.
        const int rc = lvlip_csum_batch_dev_ex(dev_base ? dev_base : s.dh_bytes, s.dh_desc, count,
                                               s.dh_out, s.stream, &cfg);
        if (rc != LVLIP_OK) return rc;
        return arm_slot(c, s, user_out, (size_t)count * sizeof(uint16_t), bytes);
    }
    // the descriptors first: the bytes' copy may wait for the previous piece's
    if ((e = hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)count * sizeof(lvlip_csum_desc),
                            hipMemcpyHostToDevice, s.stream)) != hipSuccess)
        return fail(c, e, "H2D descriptors");
    if (!dev_base) {
        const uint64_t nb = src && src != s.h_bytes ? bytes : align16(bytes);
        const int rc = h2d_ordered(c, s, s.d_bytes, src ? src : s.h_bytes, nb, "H2D bytes");
        if (rc != LVLIP_OK) return rc;
    }
    int rc = lvlip_csum_batch_dev_ex(dev_base ? dev_base : s.d_bytes, s.d_desc, count, s.d_out,
                                     s.stream, &cfg);
    if (rc != LVLIP_OK) return rc;
    if ((e = hipMemcpyAsync(s.h_out, s.d_out, (size_t)count * sizeof(uint16_t),
                            hipMemcpyDeviceToHost, s.stream)) != hipSuccess)
        return fail(c, e, "D2H results");
    return arm_slot(c, s, user_out, (size_t)count * sizeof(uint16_t), bytes);
}

// The code of the first item (in batch order) that `check` refuses, or
// LVLIP_OK, checked on the pool threads: the host calls' up-front passes over
// a whole batch ran on the calling thread before the first piece, 1-2 ms per
// 1M descriptors with the link idle.
template <class F>
int first_failure(lvlip_csum_ctx* c, uint32_t n, const F& check) {
    std::atomic<uint64_t> first{~0ull};  // (item << 8) | -code of the earliest refusal seen
    parallel_ranges(c, n, 65536, [&first, &check](uint64_t lo, uint64_t hi) {
        for (uint64_t q = lo; q < hi; ++q) {
            const int r = check((uint32_t)q);
            if (r == LVLIP_OK) continue;
            const uint64_t key = (q << 8) | (uint64_t)(-r);
            uint64_t cur = first.load(std::memory_order_relaxed);
            while (key < cur && !first.compare_exchange_weak(cur, key, std::memory_order_relaxed)) {
            }
            return;  // the rest of this range comes later in batch order
        }
    });
    const uint64_t f = first.load(std::memory_order_relaxed);
    return f == ~0ull ? LVLIP_OK : -(int)(f & 0xffu);
}

// The context's scratch array for the host batch calls, at least `bytes`
// (kept across calls: fresh pages would fault on every call; trim_scratch
// releases one above kScratchKeep when the call ends).
void* host_scratch(lvlip_csum_ctx* c, size_t bytes) {
    if (c->host_scratch_bytes < bytes) {
        free(c->host_scratch);
        c->host_scratch = malloc(bytes);
        c->host_scratch_bytes = c->host_scratch ? bytes : 0;
    }
    return c->host_scratch;
}

// The packets of a host call on the calling thread (cpu_max): Group 1's
// checksum() per packet, the reference's own arithmetic (src/utils.c:40-55).
template <class Ptr, class Len, class Seed>
int cpu_batch(lvlip_csum_ctx* c, uint32_t n, uint16_t* out, const Ptr& ptr_of, const Len& len_of,
              const Seed& seed_of) {
    c->stats.cpu_calls++;
    for (uint32_t q = 0; q < n; ++q) {
        const int32_t l = len_of(q);
        out[q] = checksum(l > 0 ? (void*)ptr_of(q) : nullptr, l, (int)seed_of(q));
    }
    return LVLIP_OK;
}

// Gathers n packets (ptr_of, len_of, seed_of) into the pinned arena, each at
// the next 16-B aligned offset, piece by piece over the two slots (the
// scattered path of lvlip_csum_batch_host, and the flat call's path for
// descriptors that do not cover their span densely in order).  Every packet
// fits the arena (checked by the callers).
template <class Ptr, class Len, class Seed>
int gather_batch(lvlip_csum_ctx* c, uint32_t n, uint16_t* out, const Ptr& ptr_of, const Len& len_of,
                 const Seed& seed_of) {
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        // lay out a piece: packet k at the next 16-B aligned offset ...
        uint64_t off = 0;
        uint32_t k = 0;
        const uint32_t first = i;
        while (i < n && k < c->max_desc) {
            const int32_t len = len_of(i);
            const uint64_t need = len > 0 ? (uint64_t)len : 0;
            if (off + need > (k ? c->piece : c->arena)) break;
            s.h_desc[k].offset = off;
            s.h_desc[k].len = len;
            s.h_desc[k].start_sum = seed_of(i);
            off = align16(off + need);
            ++k;
            ++i;
        }
        // ... then gather the bytes, packets split over the host threads,
        // nontemporal stores (copy_nt), the next packets prefetched
        {
            uint8_t* dst = s.h_bytes;
            const lvlip_csum_desc* hd = s.h_desc;
            parallel_ranges(c, k, 1024, [=](uint64_t lo, uint64_t hi) {
                for (uint64_t q = lo; q < hi; ++q) {
                    if (q + 8 < hi && hd[q + 8].len > 0)
                        for (int32_t l = 0; l < hd[q + 8].len; l += 64)
                            __builtin_prefetch((const uint8_t*)ptr_of(first + (uint32_t)q + 8) + l);
                    if (hd[q].len > 0)
                        copy_nt(dst + hd[q].offset, (const uint8_t*)ptr_of(first + (uint32_t)q), (uint64_t)hd[q].len);
                }
                _mm_sfence();
            });
        }
        rc = launch_piece(c, s, off ? off : 16, k, out + first);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

// Zero-copy: descriptors only (offsets from the region's first byte rounded
// down to 16), kernel reads the registered pages in place.  `offset_of(i)`
// gives packet i's byte address; the whole batch lies in region `r`.  Pieces
// of at most c->piece bytes (the descriptors of the next piece are written,
// on the pool threads, while the kernel reads the previous one's packets;
// a piece was max_desc descriptors before, for a 1M-packet batch one piece
// whose 16 MB of descriptors were written before the kernel started).
template <class AddrOf, class DescOf, class LenOf>
int zerocopy_batch(lvlip_csum_ctx* c, const Region& r, uint32_t n, uint16_t* out, AddrOf addr_of,
                   DescOf desc_of, LenOf len_of) {
    const uint8_t* h0 = (const uint8_t*)((uintptr_t)r.host & ~(uintptr_t)15);
    const uint8_t* d0 = r.dev - (r.host - h0);
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        const uint32_t first = i;
        uint32_t k = 0;
        uint64_t bytes = 0;
        while (i < n && k < c->max_desc) {
            const int32_t l = len_of(i);
            const uint64_t need = l > 0 ? (uint64_t)l : 0u;
            if (k && bytes + need > c->arena) break;
            bytes += need;
            ++k;
            ++i;
        }
        lvlip_csum_desc* hd = s.h_desc;
        parallel_ranges(c, k, 16384, [&, hd, first](uint64_t lo, uint64_t hi) {
            for (uint64_t q = lo; q < hi; ++q) {
                lvlip_csum_desc dq = desc_of(first + (uint32_t)q);
                dq.offset = (uint64_t)((const uint8_t*)addr_of(first + (uint32_t)q) - h0);
                hd[q] = dq;
            }
        });
        rc = launch_piece(c, s, bytes ? bytes : 16, k, out + first, nullptr, d0);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

// lvlip_csum_batch_host_flat's GPU path over validated descriptors.  dense:
// 1 / 0 when the caller has scanned the batch (dense_ordered's rule), -1 to
// scan here.  Dense batches move their spans (the copy engine straight from a
// registered region, else one nontemporal copy per span into the pinned
// arena); other batches are read in place from a zero-copy region, or
// gathered packet by packet.
int host_flat_impl(lvlip_csum_ctx* c, const uint8_t* b, size_t base_bytes, const lvlip_csum_desc* d, uint32_t n,
                   uint16_t* out, int dense) {
    const Region* reg = c->regions.empty() ? nullptr : find_region(c, b, base_bytes);
    if (dense < 0)
        dense = dense_ordered(
            c, n, [b, d](uint32_t q) { return (uint64_t)(uintptr_t)(b + d[q].offset); },
            [d](uint32_t q) { return d[q].len; });
    if (!dense) {
        if (reg && (reg->flags & LVLIP_REG_ZEROCOPY))
            return zerocopy_batch(
                c, *reg, n, out, [&](uint32_t q) { return b + d[q].offset; }, [&](uint32_t q) { return d[q]; },
                [&](uint32_t q) { return d[q].len; });
        // every packet fits the arena: the flat call's rule is the stricter
        return gather_batch(
            c, n, out, [b, d](uint32_t q) { return b + d[q].offset; }, [d](uint32_t q) { return d[q].len; },
            [d](uint32_t q) { return d[q].start_sum; });
    }
    // a piece's bytes: from a registered region the whole arena (no gather to
    // overlap with the copies, and each copy costs the copy engine ~18 us
    // between pieces: DESIGN.md §5), else LVLIP_PIECE_MAX.  A dense batch in
    // a zero-copy region moves its spans as from a DMA region (tcp1500:
    // 54.6-55.2 against 52.5 GB/s in place)
    const uint64_t limit = reg ? c->arena : c->piece;
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        // A piece is a run of descriptors whose byte span [lo16, hi) fits the
        // arena.  The span is copied with one memcpy, keeping each packet's
        // offset mod 16 (so odd/unaligned starts stay exactly as given).
        const uint32_t first = i;
        uint64_t lo16 = ~0ull, hi = 0;
        uint32_t k = 0;
        while (i < n && k < c->max_desc) {
            const uint64_t o = d[i].offset;
            const uint64_t e = o + (d[i].len > 0 ? (uint64_t)d[i].len : 0);
            const uint64_t nlo = (o & ~15ull) < lo16 ? (o & ~15ull) : lo16;
            const uint64_t nhi = e > hi ? e : hi;
            // k >= 1 here: a single span always fits the arena (checked by the caller)
            if (align16(nhi) - nlo > (k ? limit : c->arena)) break;
            lo16 = nlo;
            hi = nhi;
            ++k;
            ++i;
        }
        const uint64_t span = hi > lo16 ? hi - lo16 : 0;
        const uint8_t* from = nullptr;
        if (span && reg) {
            // f3 DMA: the copy engine reads the registered span directly.  Its
            // last bytes up to the next 16 B may lie past base_bytes, so copy
            // exactly `span` and let the kernel's 16-B tail read the arena.
            from = b + lo16;
        } else if (span) {
            // the span in 64-B blocks over the threads, nontemporal stores
            uint8_t* dst = s.h_bytes;
            const uint8_t* src = b + lo16;
            const uint64_t nblk = (span + 63) / 64;
            parallel_ranges(c, nblk, 8192, [=](uint64_t lo, uint64_t hi) {
                const uint64_t e = hi * 64 < span ? hi * 64 : span;
                copy_nt(dst + lo * 64, src + lo * 64, e - lo * 64);
                _mm_sfence();
            });
        }
        {
            lvlip_csum_desc* hd = s.h_desc;
            const lvlip_csum_desc* src = d + first;
            const uint64_t base16 = lo16;
            parallel_ranges(c, k, 16384, [hd, src, base16](uint64_t lo, uint64_t hi) {
                for (uint64_t q = lo; q < hi; ++q) {
                    hd[q] = src[q];
                    hd[q].offset = src[q].offset - base16;
                }
            });
        }
        rc = launch_piece(c, s, span ? span : 16, k, out + first, from);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

}  // namespace

extern "C" {

int lvlip_csum_ctx_create(lvlip_csum_ctx** out, int device, size_t arena_bytes) {
    if (!out) return LVLIP_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LVLIP_ENODEV;
    if (device < 0 || device >= ndev) return LVLIP_ENODEV;
    if (arena_bytes == 0) arena_bytes = kDefaultArena;
    if (arena_bytes < 4096) arena_bytes = 4096;
    arena_bytes = align16(arena_bytes);

    auto* c = new (std::nothrow) lvlip_csum_ctx();
    if (!c) return LVLIP_ENOMEM;
    c->device = device;
    c->arena = arena_bytes;
    {
        const char* e = getenv("LVLIP_GATHER_THREADS");
        const unsigned hw = std::thread::hardware_concurrency();
        int t = e ? atoi(e) : (int)(hw ? (hw < 16 ? hw : 16) : 1);
        c->threads = t < 1 ? 1 : (t > 64 ? 64 : t);
    }
    // LVLIP_DIRECT_MAX: pieces of at most this many bytes skip the H2D/D2H
    // copies (launch_piece); 0 turns that off
    {
        const char* e = getenv("LVLIP_DIRECT_MAX");
        const long long v = e ? atoll(e) : (long long)kDirectMax;
        c->direct_max = v > 0 ? (uint64_t)v : 0u;
    }
    // LVLIP_PIECE_MAX: bytes per piece, so that even a batch of a few MB is cut
    // into pieces whose gather, copies and kernel overlap across the two slots
    {
        const char* e = getenv("LVLIP_PIECE_MAX");
        const long long v = e ? atoll(e) : (long long)kPieceMax;
        const uint64_t pm = v > 0 ? align16((uint64_t)v) : arena_bytes;
        c->piece = pm < arena_bytes ? pm : arena_bytes;
    }
    // LVLIP_FIRST_PIECE: the host frame calls' first piece, in bytes; later
    // pieces double up to the piece size (0 or unset: 4 MiB; a value >= the
    // piece size turns the ramp off)
    {
        const char* e = getenv("LVLIP_FIRST_PIECE");
        const long long v = e ? atoll(e) : 0;
        c->first_piece = v > 0 ? align16((uint64_t)v) : (4ull << 20);
        if (c->first_piece > c->piece) c->first_piece = c->piece;  // the ramp's shifts never overflow
    }
    // LVLIP_INLINE_MAX: host calls of at most this many packets / frames keep
    // their host steps on the calling thread (ctx_impl.h; 0: never)
    {
        const char* e = getenv("LVLIP_INLINE_MAX");
        const long long v = e ? atoll(e) : 32768;
        c->inline_max = v > 0 ? (uint32_t)(v > 0xffffffffll ? 0xffffffffll : v) : 0u;
    }
    // LVLIP_SPAN_RATIO (1-64): the density rule's span-to-bytes ratio (span_dense)
    {
        const char* e = getenv("LVLIP_SPAN_RATIO");
        const long long v = e ? atoll(e) : 2;
        c->span_ratio = (uint32_t)(v < 1 ? 1 : v > 64 ? 64 : v);
    }
    // LVLIP_CPU_MAX: host calls of at most this many packets / frames run on
    // the calling thread (lvlip_csum_ctx_set_cpu_max; 0: always the GPU)
    {
        const char* e = getenv("LVLIP_CPU_MAX");
        const long long v = e ? atoll(e) : (long long)LVLIP_CPU_MAX_DEFAULT;
        c->cpu_max = v > 0 ? (uint32_t)(v > 0xffffffffll ? 0xffffffffll : v) : 0u;
    }
    {
        const char* e = getenv("LVLIP_FAIL_PIECE");
        const long long v = e ? atoll(e) : 0;
        c->fail_piece = v > 0 ? (uint32_t)(v > 0xffffffffll ? 0xffffffffll : v) : 0u;
    }
    // LVLIP_BLOCK_MIN: a piece of at least this many bytes is waited for by
    // polling between short sleeps instead of by spinning: the pipeline's
    // other slot keeps the GPU busy meanwhile, so the late wake-up costs no
    // throughput and the waiting thread little CPU (0: always spin)
    {
        const char* e = getenv("LVLIP_BLOCK_MIN");
        const long long v = e ? atoll(e) : (long long)kBlockMin;
        c->block_min = v > 0 ? (uint64_t)v : 0u;
    }
    {
        const char* e = getenv("LVLIP_COPY_ORDER");
        c->copy_order = e ? atoi(e) != 0 : 1;
    }
    {
        const char* e = getenv("LVLIP_FRAME_TRACE");
        c->frame_trace = e && *e == '1';
    }
    // descriptors per piece: one per 64 B of arena (a piece of smaller packets
    // simply ends at this count; the next piece takes the rest)
    c->max_desc = (uint32_t)(arena_bytes / 64 < 4096 ? 4096 : arena_bytes / 64);

    DeviceGuard g(device);
    for (auto& s : c->slot) {
        hipError_t e;
        if ((e = hipHostMalloc((void**)&s.h_bytes, arena_bytes, hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostMalloc((void**)&s.h_desc, (size_t)c->max_desc * sizeof(lvlip_csum_desc),
                               hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostMalloc((void**)&s.h_out, (size_t)c->max_desc * sizeof(uint16_t),
                               hipHostMallocDefault)) != hipSuccess ||
            (e = hipMalloc((void**)&s.d_bytes, arena_bytes)) != hipSuccess ||
            (e = hipMalloc((void**)&s.d_desc, (size_t)c->max_desc * sizeof(lvlip_csum_desc))) != hipSuccess ||
            (e = hipMalloc((void**)&s.d_out, (size_t)c->max_desc * sizeof(uint16_t))) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&s.copied, hipEventDisableTiming)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&s.dh_bytes, s.h_bytes, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&s.dh_desc, s.h_desc, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&s.dh_out, s.h_out, 0)) != hipSuccess) {
            fail(c, e, "lvlip_csum_ctx_create");
            for (auto& t : c->slot) free_slot(t);
            delete c;
            return LVLIP_ENOMEM;
        }
    }
    // Start the copy engine now: the first piece that goes through it (a call
    // larger than direct_max) otherwise pays its start-up, ~7 ms measured on
    // the first 15K-frame TX call of a context against 0.9 ms for the next.
    // Each slot copies `warm` bytes of its arena each way once
    // (LVLIP_WARM_BYTES, default 1 MiB; 0 skips it).
    {
        size_t warm = 1u << 20;
        if (const char* e = getenv("LVLIP_WARM_BYTES")) warm = strtoull(e, nullptr, 10);
        if (warm > arena_bytes) warm = arena_bytes;
        hipError_t e = hipSuccess;
        for (auto& s : c->slot) {
            if (!warm || e != hipSuccess) break;
            if ((e = hipMemcpyAsync(s.d_bytes, s.h_bytes, warm, hipMemcpyHostToDevice, s.stream)) == hipSuccess)
                e = hipMemcpyAsync(s.h_bytes, s.d_bytes, warm, hipMemcpyDeviceToHost, s.stream);
        }
        for (auto& s : c->slot)
            if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
        // and the kernels' code object, so the first call launches at once
        if (e == hipSuccess && lvlip_kernels_load() != 0) e = hipErrorInvalidDeviceFunction;
        if (e != hipSuccess) {
            fail(c, e, "lvlip_csum_ctx_create (copy engine start)");
            for (auto& t : c->slot) free_slot(t);
            delete c;
            return LVLIP_EHIP;
        }
    }
    *out = c;
    return LVLIP_OK;
}

int lvlip_csum_ctx_destroy(lvlip_csum_ctx* c) {
    if (!c) return LVLIP_EINVAL;
    DeviceGuard g(c->device);
    for (auto& s : c->slot) {
        if (s.busy) (void)hipEventSynchronize(s.done);
        free_slot(s);
    }
    for (const Region& r : c->regions) (void)hipHostUnregister(r.host);
    free(c->frame_scratch);
    free(c->frame_scratch2);
    free(c->host_scratch);
    delete c;
    return LVLIP_OK;
}

int lvlip_csum_ctx_set_cpu_max(lvlip_csum_ctx* c, uint32_t cpu_max) {
    if (!c) return LVLIP_EINVAL;
    c->cpu_max = cpu_max;
    return LVLIP_OK;
}

uint32_t lvlip_csum_ctx_cpu_max(const lvlip_csum_ctx* c) { return c ? c->cpu_max : 0u; }

int lvlip_csum_ctx_stats(const lvlip_csum_ctx* c, lvlip_ctx_stats* out) {
    if (!c || !out) return LVLIP_EINVAL;
    *out = c->stats;
    return LVLIP_OK;
}

int lvlip_csum_register(lvlip_csum_ctx* c, void* ptr, size_t bytes, uint32_t flags) {
    if (!c || !ptr || bytes == 0 || flags > LVLIP_REG_ZEROCOPY) return LVLIP_EINVAL;
    uint8_t* p = (uint8_t*)ptr;
    for (const Region& r : c->regions)
        if (p < r.host + r.bytes && r.host < p + bytes) return LVLIP_EINVAL;  // overlap
    DeviceGuard g(c->device);
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return fail(c, e, "hipHostRegister");
    void* dev = nullptr;
    if ((e = hipHostGetDevicePointer(&dev, ptr, 0)) != hipSuccess) {
        (void)hipHostUnregister(ptr);
        return fail(c, e, "hipHostGetDevicePointer");
    }
    Region r;
    r.host = p;
    r.bytes = bytes;
    r.dev = (uint8_t*)dev;
    r.flags = flags;
    try {  // no exception leaves the C ABI
        c->regions.push_back(r);
    } catch (...) {
        (void)hipHostUnregister(ptr);
        return LVLIP_ENOMEM;
    }
    return LVLIP_OK;
}

int lvlip_csum_unregister(lvlip_csum_ctx* c, void* ptr) {
    if (!c || !ptr) return LVLIP_EINVAL;
    for (size_t k = 0; k < c->regions.size(); ++k) {
        if (c->regions[k].host != (uint8_t*)ptr) continue;
        DeviceGuard g(c->device);
        for (auto& s : c->slot) {  // nothing in flight may still read it
            const int rc = drain(c, s);
            if (rc != LVLIP_OK) return rc;
        }
        const hipError_t e = hipHostUnregister(ptr);
        c->regions.erase(c->regions.begin() + (long)k);
        return e == hipSuccess ? LVLIP_OK : fail(c, e, "hipHostUnregister");
    }
    return LVLIP_EINVAL;
}

int lvlip_csum_batch_host(lvlip_csum_ctx* c, const lvlip_csum_iov* pkts, uint32_t n,
                          uint16_t* out) {
    if (!c || (n && (!pkts || !out)) || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    begin_call(c, n);
    if (first_failure(c, n, [pkts](uint32_t i) { return pkts[i].len > 0 && !pkts[i].ptr ? LVLIP_EINVAL : LVLIP_OK; }) !=
        LVLIP_OK)
        return LVLIP_EINVAL;
    const uint64_t arena = c->arena;
    if (first_failure(c, n, [pkts, arena](uint32_t i) {
            return pkts[i].len > 0 && align16((uint64_t)pkts[i].len) > arena ? LVLIP_ERANGE : LVLIP_OK;
        }) != LVLIP_OK)
        return LVLIP_ERANGE;  // a single packet larger than the arena (on every path)
    auto ptr_of = [pkts](uint32_t q) { return (const uint8_t*)pkts[q].ptr; };
    auto len_of = [pkts](uint32_t q) { return pkts[q].len; };
    auto seed_of = [pkts](uint32_t q) { return pkts[q].start_sum; };
    if (n <= c->cpu_max) return cpu_batch(c, n, out, ptr_of, len_of, seed_of);
    DeviceGuard g(c->device);
    begin_gpu_call(c);
    int rc = LVLIP_ERANGE;  // "not handled by a region path yet"
    if (!c->regions.empty()) {
        // f3: all packets inside one registered region (the region of the
        // first non-empty packet; regions never overlap) -> no gather at all:
        // packets that cover their span densely and in order go as a flat
        // batch over the region (the copy engine moves the spans); a
        // zero-copy region's other batches are read in place; a DMA region's
        // are gathered below
        uint32_t i0 = 0;
        while (i0 < n && pkts[i0].len <= 0) ++i0;
        const Region* r = i0 < n ? find_region(c, pkts[i0].ptr, (uint64_t)pkts[i0].len) : nullptr;
        if (r) {
            // one pass on the pool threads: every packet inside r, the
            // packets' span, bytes and jumps (dense_ordered's scan), and
            // their flat descriptors relative to r (written whether or not
            // they are used; the array is trimmed after a huge call)
            lvlip_csum_desc* fd = (lvlip_csum_desc*)host_scratch(c, sizeof(lvlip_csum_desc) * (size_t)n);
            const uint8_t *r0 = r->host, *r1 = r->host + r->bytes;
            std::atomic<bool> outside{false};
            constexpr uint32_t kParts = 256;
            SpanScan part[kParts];
            const uint32_t np = n / 4096u < 1u ? 1u : (n / 4096u > kParts ? kParts : n / 4096u);
            parallel_ranges(c, np, 1, [&, fd, r0, r1](uint64_t plo, uint64_t phi) {
                for (uint64_t j = plo; j < phi; ++j) {
                    SpanScan sc;
                    const uint32_t a = (uint32_t)((uint64_t)n * j / np), z = (uint32_t)((uint64_t)n * (j + 1) / np);
                    for (uint32_t q = a; q < z; ++q) {
                        const int32_t len = pkts[q].len;
                        uint64_t o = 0;
                        if (len > 0) {
                            const uint8_t* p = (const uint8_t*)pkts[q].ptr;
                            if (p < r0 || p + len > r1) {
                                outside.store(true, std::memory_order_relaxed);
                                return;
                            }
                            o = (uint64_t)(p - r0);
                            span_add(sc, o, (uint64_t)len);
                        }
                        if (fd) fd[q] = lvlip_csum_desc{o, len, pkts[q].start_sum};
                    }
                    part[j] = sc;
                }
            });
            const bool inside = !outside.load();
            if (inside && fd && span_dense(span_merge(part, np), c->span_ratio))
                // refused only when one packet's 16-B span exceeds the arena
                // (the flat call's rule): then the gather below takes it
                rc = host_flat_impl(c, r->host, r->bytes, fd, n, out, 1);
            else if (inside && (r->flags & LVLIP_REG_ZEROCOPY))
                rc = zerocopy_batch(
                    c, *r, n, out, [&](uint32_t q) { return pkts[q].len > 0 ? (const uint8_t*)pkts[q].ptr : r->host; },
                    [&](uint32_t q) {
                        lvlip_csum_desc d{};
                        d.len = pkts[q].len;
                        d.start_sum = pkts[q].start_sum;
                        return d;
                    },
                    [&](uint32_t q) { return pkts[q].len; });
        }
    }
    if (rc == LVLIP_ERANGE) rc = gather_batch(c, n, out, ptr_of, len_of, seed_of);
    trim_scratch(c);
    return rc;
}

int lvlip_csum_batch_host_flat(lvlip_csum_ctx* c, const void* base, size_t base_bytes,
                               const lvlip_csum_desc* d, uint32_t n, uint16_t* out) {
    if (!c || (n && (!base || !d || !out)) || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    begin_call(c, n);
    const uint8_t* b = (const uint8_t*)base;
    const uint64_t arena = c->arena;
    const int bad = first_failure(c, n, [d, base_bytes, arena](uint32_t q) {
        const uint64_t e = d[q].offset + (d[q].len > 0 ? (uint64_t)d[q].len : 0u);
        if (e > base_bytes) return LVLIP_EINVAL;
        // a single packet whose 16-B span exceeds the arena: refuse before any
        // piece is in flight (a piece still in flight would later write into out[])
        if (align16(e) - (d[q].offset & ~15ull) > arena) return LVLIP_ERANGE;
        return LVLIP_OK;
    });
    if (bad != LVLIP_OK) return bad;
    if (n <= c->cpu_max)
        return cpu_batch(
            c, n, out, [b, d](uint32_t q) { return b + d[q].offset; }, [d](uint32_t q) { return d[q].len; },
            [d](uint32_t q) { return d[q].start_sum; });
    DeviceGuard g(c->device);
    begin_gpu_call(c);
    const int rc = host_flat_impl(c, b, base_bytes, d, n, out, -1);
    trim_scratch(c);
    return rc;
}

// Group 4: one host thread per context, each on its part of the batch.  The
// parts' descriptors keep their offsets from `base`, so each context gathers
// (or DMAs) only its own span.
int lvlip_csum_batch_host_flat_multi(lvlip_csum_ctx* const* ctxs, uint32_t nctx, const void* base,
                                     size_t base_bytes, const lvlip_csum_desc* d, uint32_t n, uint16_t* out) {
    if (!ctxs || nctx == 0 || (n && (!base || !d || !out)) || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    for (uint32_t k = 0; k < nctx; ++k) {
        if (!ctxs[k]) return LVLIP_EINVAL;
        for (uint32_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return LVLIP_EINVAL;  // one thread per context
    }
    if (n == 0) return LVLIP_OK;
    std::vector<uint32_t> cuts;
    std::vector<int> rcs;
    std::vector<std::thread> th;
    std::vector<std::string> errs;  // each part's lvlip_last_hip_error() (thread-local)
    try {  // no exception leaves the C ABI
        cuts.resize(nctx + 1u);
        rcs.assign(nctx, LVLIP_OK);
        errs.resize(nctx);
        th.reserve(nctx);
    } catch (...) {
        return LVLIP_ENOMEM;
    }
    int rc = lvlip_partition_bytes(d, n, nctx, cuts.data());
    if (rc != LVLIP_OK) return rc;
    auto part = [&](uint32_t k) noexcept {
        const uint32_t lo = cuts[k], hi = cuts[k + 1];
        if (hi > lo) rcs[k] = lvlip_csum_batch_host_flat(ctxs[k], base, base_bytes, d + lo, hi - lo, out + lo);
        if (rcs[k] != LVLIP_OK) {
            try {
                errs[k] = lvlip_last_hip_error();
            } catch (...) {
            }
        }
    };
    // parts 1.. on threads of their own; a part whose thread cannot be
    // started runs on the calling thread after part 0 (a thread shortage
    // costs the overlap, not the call)
    uint32_t started = 1;
    try {
        for (; started < nctx; ++started) th.emplace_back(part, started);
    } catch (...) {
    }
    part(0);
    for (uint32_t k = started; k < nctx; ++k) part(k);
    for (auto& t : th) t.join();
    for (uint32_t k = 0; k < nctx; ++k)
        if (rcs[k] != LVLIP_OK) {
            // the failing part's HIP message, on the caller's thread
            lvlip_set_last_hip_error(errs[k].c_str());
            return rcs[k];
        }
    return LVLIP_OK;
}

}  // extern "C"
