// ctx_impl.h — the host context's internals (include/lvlip_csum.h, Group 3),
// shared by csum_ctx.cpp (host packet batches) and frames_host.cpp (host frame
// batches, include/lvlip_skb.h f1/f2).  Not installed; nothing here is
// exported (the library is built with -fvisibility=hidden).
//
// A context owns, per pipeline slot (two slots):
//   - a pinned host arena the bytes are gathered into (each packet or frame at
//     a 16-B aligned slot, so the GPU's 16-B chunks never straddle two),
//   - the matching device arena, descriptor and result buffers,
//   - its own non-blocking stream and a completion event.
// A batch is cut into arena-sized pieces; piece k is gathered on the CPU while
// piece k-1's H2D copy, kernel and D2H copy run on the other slot's stream.
#pragma once

#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "gather_pool.h"
#include "lvlip_csum.h"
#include "lvlip_skb.h"

namespace lvlip_ctx {

constexpr int kSlots = 2;

inline uint64_t align16(uint64_t x) { return (x + 15ull) & ~15ull; }

struct Slot {
    uint8_t* h_bytes = nullptr;         // pinned
    lvlip_csum_desc* h_desc = nullptr;  // pinned (frame calls: lvlip_frame_desc, also 16 B)
    uint16_t* h_out = nullptr;          // pinned, max_desc u16 (frame calls: records / verdicts)
    // the same three pinned buffers as device addresses (small pieces are read
    // and written by the kernel in place, see launch_piece)
    uint8_t* dh_bytes = nullptr;
    lvlip_csum_desc* dh_desc = nullptr;
    uint16_t* dh_out = nullptr;
    uint8_t* d_bytes = nullptr;
    lvlip_csum_desc* d_desc = nullptr;
    uint16_t* d_out = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t copied = nullptr;  // after the slot's last H2D of a piece's bytes (h2d_ordered)
    // how drain() waits for `done`: spinning in hipEventSynchronize (short
    // pieces: the lowest latency), or polling it between short sleeps (long
    // pieces: the waiting thread costs no CPU while the other slot's piece
    // keeps the GPU busy)
    bool sleep = false;
    // piece bookkeeping: the in-flight piece's results (out_bytes of them in
    // h_out) go to user_out when the slot drains
    void* user_out = nullptr;
    size_t out_bytes = 0;
    bool busy = false;
};

// A registered host region (f3): pinned in place, mapped into the device's
// address space.
struct Region {
    uint8_t* host = nullptr;
    size_t bytes = 0;
    uint8_t* dev = nullptr;  // device address of host[0]
    uint32_t flags = 0;
};

}  // namespace lvlip_ctx

struct lvlip_csum_ctx {
    int device = 0;
    size_t arena = 0;         // bytes per slot
    uint32_t max_desc = 0;    // descriptors per slot (h_out holds 2 B each)
    int threads = 1;          // host threads for the gather into the pinned arena
    uint64_t direct_max = 0;  // pieces up to this many bytes skip the copies
    uint64_t piece = 0;       // bytes per piece (<= arena; a larger packet gets its own)
    uint64_t first_piece = 0; // frame calls: the first piece's bytes (doubling up to `piece`)
    uint64_t block_min = 0;   // pieces of at least this many bytes are waited for asleep (0: never)
    // LVLIP_COPY_ORDER (default 1): in the packet batch calls each piece's
    // H2D of its bytes waits for the previous piece's of the same call
    // (h2d_ordered; the frame calls do not); last_copy is the slot that
    // issued that one (nullptr at a call's start)
    int copy_order = 1;
    lvlip_ctx::Slot* last_copy = nullptr;
    // frame calls' per-call host arrays (TX records and undo values, RX + L4
    // lengths), kept across calls: fresh pages would fault on every call
    void* frame_scratch = nullptr;
    size_t frame_scratch_bytes = 0;
    void* frame_scratch2 = nullptr;
    size_t frame_scratch2_bytes = 0;
    // the iov call's flat descriptors over a registered region, kept likewise
    void* host_scratch = nullptr;
    size_t host_scratch_bytes = 0;
    int frame_trace = 0;      // LVLIP_FRAME_TRACE=1: per-step host times on stderr
    // host calls of at most this many packets / frames run on the calling
    // thread (lvlip_csum_ctx_set_cpu_max; 0: never)
    uint32_t cpu_max = LVLIP_CPU_MAX_DEFAULT;
    lvlip_ctx_stats stats{};
    // test hook LVLIP_FAIL_PIECE=k (k >= 1): the k-th device piece of every GPU
    // call fails with LVLIP_EHIP before it is launched, so the tests can drive
    // the error paths (a TX call's undo, a caller's CPU fill) on a healthy GPU
    uint32_t fail_piece = 0;
    uint32_t call_pieces = 0;  // pieces launched by the current call
    // host calls of at most this many packets / frames do their host steps
    // (checks, gather, descriptors, TX field stores) on the calling thread
    // only (LVLIP_INLINE_MAX; 0: never).  Such a call's frames are the
    // working set the caller has just built and touches again right after
    // (level-ip's stack): the pool's 16 threads pulled their cache lines to
    // other cores and made the composed stack up to 2x costlier per frame
    // ("Where batch-and-dispatch pays")
    uint32_t inline_max = 32768;
    // LVLIP_SPAN_RATIO: a registered region's items move as spans with the
    // copy engine when their span is at most this many times their bytes
    // (plus 1 MiB) and in address order (span_dense)
    uint32_t span_ratio = 2;
    bool inline_call = false;  // the current call is one of those
    lvlip_ctx::Slot slot[lvlip_ctx::kSlots];
    std::vector<lvlip_ctx::Region> regions;
    lvlip::GatherPool pool;
    char err[256] = "";
};

namespace lvlip_ctx {

// Records a HIP failure in the context (and on stderr); returns `code`.
int fail(lvlip_csum_ctx* c, hipError_t e, const char* what, int code = LVLIP_EHIP);
// H2D of a piece's bytes into the slot, on the slot's stream, queued behind
// the previous piece's copy of the same call when c->copy_order is set.
int h2d_ordered(lvlip_csum_ctx* c, Slot& s, void* dst, const void* src, size_t n, const char* what);
// Waits for a slot's in-flight piece and copies its results to user_out.
int drain(lvlip_csum_ctx* c, Slot& s);
// End of a batch call: drains both slots; after a failure also waits for what
// a half-enqueued piece left on the slot streams.
int finish_pieces(lvlip_csum_ctx* c, int rc);
// The registered region holding [p, p + len), or nullptr.
const Region* find_region(const lvlip_csum_ctx* c, const void* p, uint64_t len);
// Marks the slot busy with a piece whose results (out_bytes) go to user_out.
// records the slot's completion after its piece of `piece_bytes` bytes; the
// wait for it sleeps from c->block_min bytes up, else spins
int arm_slot(lvlip_csum_ctx* c, Slot& s, void* user_out, size_t out_bytes, uint64_t piece_bytes);
// Counts a device piece of the current call moving `bytes` from the host
// (stats, LVLIP_FAIL_PIECE): LVLIP_OK, or the injected LVLIP_EHIP.
int count_piece(lvlip_csum_ctx* c, uint64_t bytes);
// Start of a host call over n packets / frames: whether its host steps stay
// on the calling thread (inline_max).
inline void begin_call(lvlip_csum_ctx* c, uint64_t n) { c->inline_call = c->inline_max && n <= c->inline_max; }
// Start of a host call that goes to the GPU (counters, the per-call piece count).
inline void begin_gpu_call(lvlip_csum_ctx* c) {
    c->stats.gpu_calls++;
    c->call_pieces = 0;
}

// The per-call host arrays are kept for the next call (fresh pages would fault
// on every call), except one above this size, released when its call ends so
// that one huge batch does not hold memory for the context's lifetime
// (the iov call's 16 n bytes of flat descriptors).
constexpr size_t kScratchKeep = 64ull << 20;
inline void trim_scratch(lvlip_csum_ctx* c) {
    auto trim = [](void*& p, size_t& b) {
        if (b > kScratchKeep) {
            free(p);
            p = nullptr;
            b = 0;
        }
    };
    trim(c->frame_scratch, c->frame_scratch_bytes);
    trim(c->frame_scratch2, c->frame_scratch2_bytes);
    trim(c->host_scratch, c->host_scratch_bytes);
}

// Whether items cover their byte span densely AND in call order, the condition
// for moving whole spans (DMA, or the flat call's span copy): the span at most
// span_ratio (2) times their bytes plus 1 MiB, and the jumps between consecutive start
// addresses summing to at most twice the span plus 1 MiB.  Pieces are runs in
// call order cut at the piece size, so a shuffled batch over a large buffer
// would cut into pieces of one or two items, each moving a whole span (ADVICE
// r05).  A scan is kept per part of the batch (pool threads), then merged in
// part order.
struct SpanScan {
    uint64_t lo = ~0ull, hi = 0, sum = 0, jumps = 0;
    uint64_t first = ~0ull, last = ~0ull;  // the part's first and last start address
    bool any() const { return first != ~0ull; }
};
inline void span_add(SpanScan& s, uint64_t a, uint64_t len) {
    s.lo = a < s.lo ? a : s.lo;
    s.hi = a + len > s.hi ? a + len : s.hi;
    s.sum += len;
    if (s.last != ~0ull) s.jumps += a > s.last ? a - s.last : s.last - a;
    if (s.first == ~0ull) s.first = a;
    s.last = a;
}
// parts in call order -> the whole batch's scan (the jump between parts included)
inline SpanScan span_merge(const SpanScan* p, uint32_t np) {
    SpanScan t;
    for (uint32_t j = 0; j < np; ++j) {
        if (!p[j].any()) continue;
        if (t.any()) t.jumps += p[j].first > t.last ? p[j].first - t.last : t.last - p[j].first;
        else t.first = p[j].first;
        t.lo = p[j].lo < t.lo ? p[j].lo : t.lo;
        t.hi = p[j].hi > t.hi ? p[j].hi : t.hi;
        t.sum += p[j].sum;
        t.jumps += p[j].jumps;
        t.last = p[j].last;
    }
    return t;
}
// ratio: the context's span_ratio (2; LVLIP_SPAN_RATIO).  A span moved by the
// copy engine costs the link its bytes and the host nothing; a gather costs
// the host a copy of every item's bytes.  Inside level-ip's stack, replies
// in a slab's 1 792-B granules (2.2x their bytes) moved as spans (ratio 3)
// ran 3-6 % faster per frame than gathered at 16K frames and tied at 4K
// (DESIGN.md §9); for an isolated call the pool's gather keeps the link
// time at the items' own bytes, so the default stays 2.
inline bool span_dense(const SpanScan& s, uint32_t ratio) {
    if (!s.any() || s.hi <= s.lo) return false;
    const uint64_t span = s.hi - s.lo;
    return span <= (uint64_t)ratio * s.sum + (1ull << 20) && s.jumps <= 2 * span + (1ull << 20);
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// len bytes from src (any alignment) to the 16-B aligned dst with nontemporal
// 16-B stores: the gathers into the pinned arena, which the copy engine (or
// the kernel, over PCIe) reads next.  Stores that bypass the CPU caches leave
// no dirty lines for those reads to snoop and need no read for ownership of
// the arena's lines (measured).  The last partial chunk goes
// through a zeroed 16-B temporary: nothing past src + len is read, and the
// chunk's bytes past len become zero.  The caller fences (_mm_sfence) before
// the data is handed to the device.
inline void copy_nt(uint8_t* dst, const uint8_t* src, uint64_t len) {
    uint64_t k = 0;
    for (; k + 64 <= len; k += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(src + k));
        const __m128i b = _mm_loadu_si128((const __m128i*)(src + k + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(src + k + 32));
        const __m128i d = _mm_loadu_si128((const __m128i*)(src + k + 48));
        _mm_stream_si128((__m128i*)(dst + k), a);
        _mm_stream_si128((__m128i*)(dst + k + 16), b);
        _mm_stream_si128((__m128i*)(dst + k + 32), c);
        _mm_stream_si128((__m128i*)(dst + k + 48), d);
    }
    for (; k + 16 <= len; k += 16) _mm_stream_si128((__m128i*)(dst + k), _mm_loadu_si128((const __m128i*)(src + k)));
    if (k < len) {
        alignas(16) uint8_t t[16] = {0};
        memcpy(t, src + k, (size_t)(len - k));
        _mm_stream_si128((__m128i*)(dst + k), _mm_load_si128((const __m128i*)t));
    }
}

// Runs fn(lo, hi) over [0, n) split into up to c->threads contiguous ranges of
// at least min_per_thread.  The gather into pinned memory is host-memory-
// bandwidth bound: one core moves ~25-30 GB/s, below PCIe Gen5 x16, so a piece
// is copied by several of the context's pool threads.
template <class F>
void parallel_ranges(lvlip_csum_ctx* c, uint64_t n, uint64_t min_per_thread, F fn) {
    if (c->inline_call) {  // a cache-sized call: every host step on the calling thread
        fn(0, n);
        return;
    }
    uint64_t t = c->threads > 1 ? (uint64_t)c->threads : 1u;
    if (n / min_per_thread < t) t = n / min_per_thread ? n / min_per_thread : 1u;
    if (t <= 1) {
        fn(0, n);
        return;
    }
    c->pool.run((int)t, [&](int k) { fn(n * (uint64_t)k / t, n * (uint64_t)(k + 1) / t); });
}

// span_dense over n items (start address addr_of(q), length len_of(q); items
// of length <= 0 skipped), scanned in parts of at least 4096 items (at most
// 256 parts) on the pool threads.
template <class Addr, class Len>
bool dense_ordered(lvlip_csum_ctx* c, uint32_t n, const Addr& addr_of, const Len& len_of) {
    constexpr uint32_t kParts = 256;
    SpanScan part[kParts];
    const uint32_t np = n / 4096u < 1u ? 1u : (n / 4096u > kParts ? kParts : n / 4096u);
    parallel_ranges(c, np, 1, [&](uint64_t plo, uint64_t phi) {
        for (uint64_t j = plo; j < phi; ++j) {
            SpanScan s;
            const uint32_t a = (uint32_t)((uint64_t)n * j / np), b = (uint32_t)((uint64_t)n * (j + 1) / np);
            for (uint32_t q = a; q < b; ++q) {
                const int64_t l = (int64_t)len_of(q);
                if (l > 0) span_add(s, (uint64_t)addr_of(q), (uint64_t)l);
            }
            part[j] = s;
        }
    });
    return span_dense(span_merge(part, np), c->span_ratio);
}

}  // namespace lvlip_ctx

extern "C" {
// csum_kernels.hip
int lvlip_csum_batch_dev_ex(const void*, const lvlip_csum_desc*, uint32_t, uint16_t*, void*,
                            const lvlip_launch_cfg*);
// lvlip_last_hip_error()'s thread-local message, set (hidden).
void lvlip_set_last_hip_error(const char* msg);
// The host frame calls' device step: mode 0 TX records (u64 per frame), 1 RX
// header, 2 RX + L4 (u8 verdicts).  Hidden.
int lvlip_kernels_load(void);  // csum_kernels.hip
int lvlip_frames_host_launch(int mode, const void* base, const lvlip_frame_desc* frames, uint32_t n,
                             void* out, void* stream);
}
