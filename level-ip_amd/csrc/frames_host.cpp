// frames_host.cpp — f1/f2 of SURVEY.md §8f on frames in HOST memory:
// lvlip_rx_verify and lvlip_tx_checksum of include/lvlip_skb.h.
//
// level-ip's frames live in skbs: netdev_rx_loop reads each received frame
// into its own alloc_skb(BUFLEN) buffer (src/netdev.c:86-101), and ip_output
// hands each outgoing one to dst_neigh_output (src/ip_output.c:14-56).  These
// calls take N such frames and do on the GPU what ip_rcv (src/ip_input.c:17-60)
// and tcp_transmit_skb / icmpv4_reply / ip_send_check (src/tcp_output.c:126,
// src/icmpv4.c:47, src/ip_output.c:53) do per frame.
//
// The device parses every frame itself (the fused frame kernels of
// flat_src.h: k_flat2 with a FrameSrc, k_rx_hdr), so the host never plans a
// frame, and never reads one except to move it:
//   - frames inside one LVLIP_REG_ZEROCOPY region: only frame descriptors go
//     down; the kernel reads the frames in place over PCIe;
//   - frames inside one LVLIP_REG_DMA region, packed densely: the copy engine
//     moves each piece's span straight from the region;
//   - anywhere else (scattered skbs): each frame is copied whole, one memcpy,
//     into a 16-B aligned slot of the pinned arena by the context's pool
//     threads, then one H2D copy per piece.
// RX verdicts come back as 1 B per frame.  TX comes back as one 8-B record per
// frame (the two fields and where the L4 one goes, FrameSrc<FR_TX_REC>); the
// host stores the fields into the caller's frames once every frame is known
// to be well formed, so a malformed frame still leaves the whole batch
// untouched (include/lvlip_skb.h).  Pieces are double-buffered over the two
// slots as in csum_ctx.cpp.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>

#include "ctx_impl.h"

namespace {

using namespace lvlip_ctx;

enum { M_TX = 0, M_RX = 1, M_RX_L4 = 2 };  // lvlip_frames_host_launch's modes
constexpr uint32_t kEth = 14;              // include/ethernet.h: struct eth_hdr
// Ethernet + the longest IPv4 header (ihl 15): every byte the header-only RX
// call reads (ip_rcv's decisions and the header checksum, src/ip_input.c:17-43)
constexpr uint32_t kHdrWin = kEth + 60;
// a frame's result: an 8-B record (TX) or a 1-B verdict (RX)
inline uint32_t out_bytes(int mode) { return mode == M_TX ? 8u : 1u; }

inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
// frames ahead whose first lines the gather and the apply prefetch
constexpr uint64_t kPrefetch = 8;

// The bytes of a frame the device step reads, so the gather moves no more.
// Every decision the kernels take compares the frame length with 14 + 20,
// 14 + ihl * 4 (<= kHdrWin) or 14 + the IP total length, and a length cut to
// max(kHdrWin, 14 + total length) gives each comparison the same outcome.
//   RX header only: min(len, kHdrWin) (no frame byte is read here)
//   RX + L4: min(len, max(kHdrWin, 14 + IP total length)): reads the frame's
//     total length field (skbs from netdev_rx_loop are BUFLEN long whatever the
//     frame, src/netdev.c:89-91)
//   TX: len (frames from ip_output are exactly the packet)
inline uint32_t need_len(int mode, const lvlip_frame& f) {
    if (!f.head) return 0;
    if (mode == M_RX) return f.len < kHdrWin ? f.len : kHdrWin;
    if (mode == M_RX_L4 && f.len > kHdrWin) {
        const uint32_t want = kEth + be16(f.head + kEth + 2);
        const uint32_t m = want > kHdrWin ? want : kHdrWin;
        return f.len < m ? f.len : m;
    }
    return f.len;
}

// The context's scratch array of at least `bytes` (kept for later calls).
void* scratch(lvlip_csum_ctx* c, size_t bytes) {
    if (c->frame_scratch_bytes < bytes) {
        free(c->frame_scratch);
        c->frame_scratch = malloc(bytes);
        c->frame_scratch_bytes = c->frame_scratch ? bytes : 0;
    }
    return c->frame_scratch;
}

// A second scratch array (the gather's prefix sums and RX + L4's lengths),
// kept like the first.
void* scratch2(lvlip_csum_ctx* c, size_t bytes) {
    if (c->frame_scratch2_bytes < bytes) {
        free(c->frame_scratch2);
        c->frame_scratch2 = malloc(bytes);
        c->frame_scratch2_bytes = c->frame_scratch2 ? bytes : 0;
    }
    return c->frame_scratch2;
}

// Frames per piece: the slot's descriptor array and its result buffer.
inline uint32_t frames_per_piece(const lvlip_csum_ctx* c, int mode) {
    const uint64_t by_out = (uint64_t)c->max_desc * sizeof(uint16_t) / out_bytes(mode);
    return by_out < c->max_desc ? (uint32_t)by_out : c->max_desc;
}

// Bytes of piece number `idx` of a call: the pipeline starts with small
// pieces (the GPU waits for the first gather or copy, and the first piece's
// results gate the host's first apply), doubling from the context's
// first_piece (LVLIP_FIRST_PIECE, 4 MiB) up to its piece size
// (LVLIP_PIECE_MAX, 32 MiB).
inline uint64_t piece_bytes(const lvlip_csum_ctx* c, uint32_t idx) {
    // first_piece <= piece (lvlip_csum_ctx_create), and the shift is taken only
    // while it stays below piece: no overflow for any LVLIP_FIRST_PIECE
    return idx < 16 && c->first_piece <= (c->piece >> idx) ? c->first_piece << idx : c->piece;
}

// LVLIP_FRAME_TRACE=1 (read when the context is made): one line per call on
// stderr with the host's time in each step (diagnostics for the pipeline's
// balance; off by default).
struct Trace {
    bool on = false;
    std::chrono::steady_clock::time_point t0;
    double pass1 = 0, gather = 0, wait = 0, apply = 0;
    uint32_t pieces = 0;
    static double ms(std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    }
};
thread_local Trace g_trace;

// Called with each piece's frame range once its results are in the caller's
// array (TX: the host applies that piece's records while later pieces run).
struct PieceDone {
    virtual void done(uint32_t first, uint32_t k) = 0;
    // no further piece is worth issuing (TX: a malformed frame was seen, the
    // call will undo and fail)
    virtual bool stop() const { return false; }
};

// drain() plus the piece callback; the slot remembers its piece's range.
struct FrameSlots {
    lvlip_csum_ctx* c;
    PieceDone* cb;
    uint32_t first[kSlots] = {0, 0}, count[kSlots] = {0, 0};
    int drain_slot(int k) {
        Slot& s = c->slot[k];
        const bool was = s.busy;
        auto t = std::chrono::steady_clock::now();
        const int rc = drain(c, s);
        if (g_trace.on) g_trace.wait += Trace::ms(t);
        t = std::chrono::steady_clock::now();
        if (rc == LVLIP_OK && was && cb) cb->done(first[k], count[k]);
        if (g_trace.on && was) g_trace.apply += Trace::ms(t), g_trace.pieces++;
        return rc;
    }
    // finish_pieces with the callback: the older piece first
    int finish(int rc, int next) {
        for (int j = 0; j < kSlots; ++j) {
            const int r2 = drain_slot((next + j) % kSlots);
            if (rc == LVLIP_OK) rc = r2;
        }
        if (rc != LVLIP_OK)
            for (auto& s : c->slot) (void)hipStreamSynchronize(s.stream);
        return rc;
    }
};

// One piece of k frames (descriptors in the slot's pinned h_desc) through the
// device step, as csum_ctx.cpp's launch_piece: the frames come from the
// slot's pinned arena, from `src` (a registered region: DMA), or are read in
// place at `dev_base` (zero-copy).  A piece of at most direct_max bytes skips
// the copies: the kernel reads the arena (or region) and the descriptors over
// PCIe and writes its results into the pinned result buffer.
int launch_frame_piece(lvlip_csum_ctx* c, Slot& s, int mode, uint64_t bytes, uint32_t k, void* user_out,
                       const uint8_t* src = nullptr, const uint8_t* dev_base = nullptr) {
    hipError_t e;
    if (const int rc = count_piece(c, bytes); rc != LVLIP_OK) return rc;
    const size_t nout = (size_t)k * out_bytes(mode);
    if (bytes <= c->direct_max && (dev_base || !src)) {
        const int rc = lvlip_frames_host_launch(mode, dev_base ? dev_base : s.dh_bytes,
                                                (const lvlip_frame_desc*)s.dh_desc, k, s.dh_out, s.stream);
        if (rc != LVLIP_OK) return rc;
        return arm_slot(c, s, user_out, nout, bytes);
    }
    // the descriptors, then the frames, on the slot's stream.  The frame calls
    // do not order their pieces' copies behind each other (h2d_ordered): in
    // one process that cost the registered-slab calls 1.5-3 % and tripled
    // their host CPU time per frame
    if ((e = hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)k * sizeof(lvlip_frame_desc), hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess)
        return fail(c, e, "H2D frame descriptors");
    if (!dev_base) {
        const uint64_t nb = src ? bytes : align16(bytes);
        if ((e = hipMemcpyAsync(s.d_bytes, src ? src : s.h_bytes, nb, hipMemcpyHostToDevice, s.stream)) !=
            hipSuccess)
            return fail(c, e, "H2D frames");
    }
    const int rc = lvlip_frames_host_launch(mode, dev_base ? dev_base : s.d_bytes,
                                            (const lvlip_frame_desc*)s.d_desc, k, s.d_out, s.stream);
    if (rc != LVLIP_OK) return rc;
    if ((e = hipMemcpyAsync(s.h_out, s.d_out, nout, hipMemcpyDeviceToHost, s.stream)) != hipSuccess)
        return fail(c, e, "D2H frame results");
    return arm_slot(c, s, user_out, nout, bytes);
}

// Scattered frames: each frame's need_len bytes (len[i] when given) copied
// whole into its 16-B aligned slot of the pinned arena.  pre[i] is frame i's
// slot offset in the batch's virtual arena stream (pre[n] the total), so a
// piece is the run of frames whose slots fit the piece, found by binary
// search, and the pool threads write its descriptors as they copy.
int frames_gather(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out,
                  const uint32_t* len, const uint64_t* pre, PieceDone* cb) {
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    FrameSlots fs{c, cb};
    int cur = 0;
    uint32_t i = 0, idx = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = fs.drain_slot(cur)) != LVLIP_OK) break;
        if (cb && cb->stop()) break;
        lvlip_frame_desc* hd = (lvlip_frame_desc*)s.h_desc;
        const uint32_t first = i;
        const uint64_t pb = piece_bytes(c, idx++);
        // the last frame whose slot ends within pb of the piece's start
        const uint32_t cap = n - first < fmax ? n : first + fmax;
        uint32_t e = (uint32_t)(std::upper_bound(pre + first + 1, pre + cap + 1, pre[first] + pb) - pre) - 1;
        if (e == first) e = first + 1;  // one frame larger than a piece: alone (it fits the arena)
        const uint32_t k = e - first;
        const uint64_t off = pre[e] - pre[first];
        i = e;
        {
            const auto t = std::chrono::steady_clock::now();
            uint8_t* dst = s.h_bytes;
            const lvlip_frame* src = fr + first;
            const uint64_t* pf = pre + first;
            const uint32_t* lf = len ? len + first : nullptr;
            parallel_ranges(c, k, 256, [=](uint64_t lo, uint64_t hi) {
                for (uint64_t q = lo; q < hi; ++q) {
                    // scattered frames: what the copy reads of the frame
                    // kPrefetch frames ahead (scattered 1616-B slots: +25-40 %
                    // over its first two lines)
                    const uint64_t pq = q + kPrefetch;
                    if (pq < hi && src[pq].head) {
                        const uint32_t pl = lf ? lf[pq] : need_len(mode, src[pq]);
                        for (uint32_t l = 0; l < pl; l += 64) __builtin_prefetch(src[pq].head + l);
                    }
                    const uint32_t l = lf ? lf[q] : need_len(mode, src[q]);
                    hd[q].offset = pf[q] - pf[0];
                    hd[q].len = l;
                    hd[q].reserved = 0;
                    if (l) copy_nt(dst + hd[q].offset, src[q].head, l);
                }
                _mm_sfence();  // the nontemporal stores land before the copy engine reads
            });
            if (g_trace.on) g_trace.gather += Trace::ms(t);
        }
        fs.first[cur] = first;
        fs.count[cur] = k;
        rc = launch_frame_piece(c, s, mode, off ? off : 16, k, out + (size_t)first * ob);
        cur ^= 1;
    }
    return fs.finish(rc, cur);
}

// Frame descriptors {head - base, len} of k frames, on the pool threads.
void write_descs(lvlip_csum_ctx* c, lvlip_frame_desc* hd, const lvlip_frame* f, uint32_t k, uintptr_t base) {
    parallel_ranges(c, k, 8192, [=](uint64_t lo, uint64_t hi) {
        for (uint64_t q = lo; q < hi; ++q) {
            hd[q].offset = (uint64_t)((uintptr_t)f[q].head - base);
            hd[q].len = f[q].len;
            hd[q].reserved = 0;
        }
    });
}

// Frames inside one LVLIP_REG_ZEROCOPY region: descriptors only, offsets from
// the region's first byte rounded down to 16; the kernel reads in place.
int frames_zerocopy(lvlip_csum_ctx* c, const Region& r, const lvlip_frame* fr, uint32_t n, int mode,
                    uint8_t* out, PieceDone* cb) {
    const uint8_t* h0 = (const uint8_t*)((uintptr_t)r.host & ~(uintptr_t)15);
    const uint8_t* d0 = r.dev - (r.host - h0);
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    FrameSlots fs{c, cb};
    int cur = 0;
    uint32_t i = 0, idx = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = fs.drain_slot(cur)) != LVLIP_OK) break;
        if (cb && cb->stop()) break;
        lvlip_frame_desc* hd = (lvlip_frame_desc*)s.h_desc;
        const uint32_t first = i;
        const uint64_t pb = piece_bytes(c, idx++);
        uint64_t bytes = 0;
        uint32_t k = 0;
        while (i < n && k < fmax && (k == 0 || bytes + fr[i].len <= pb)) {
            bytes += fr[i].len;
            ++k;
            ++i;
        }
        write_descs(c, hd, fr + first, k, (uintptr_t)h0);
        fs.first[cur] = first;
        fs.count[cur] = k;
        rc = launch_frame_piece(c, s, mode, bytes ? bytes : 16, k, out + (size_t)first * ob, nullptr, d0);
        cur ^= 1;
    }
    return fs.finish(rc, cur);
}

// Frames inside one LVLIP_REG_DMA region: a piece is a run of frames whose
// byte span [lo, hi) fits the piece size; the copy engine reads the span from
// the region.  lo is rounded down to 16 from the region's first byte, not from
// address 0, so the span never starts before the registered bytes (the copy
// engine reads them as pinned memory; the kernels take any alignment).
int frames_dma(lvlip_csum_ctx* c, const Region& r, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out,
               PieceDone* cb) {
    const uintptr_t r0 = (uintptr_t)r.host;
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    FrameSlots fs{c, cb};
    int cur = 0;
    uint32_t i = 0, idx = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = fs.drain_slot(cur)) != LVLIP_OK) break;
        if (cb && cb->stop()) break;
        const uint32_t first = i;
        uintptr_t lo = ~(uintptr_t)0, hi = 0;
        uint32_t k = 0;
        // (pieces grown to the whole arena, as the flat host call's DMA pieces,
        // lost here: TX's last piece's field stores no longer overlap a copy;
        // DESIGN.md §9)
        const uint64_t pb = piece_bytes(c, idx++);
        while (i < n && k < fmax) {
            const uintptr_t a = (uintptr_t)fr[i].head, e = a + fr[i].len;
            const uintptr_t a16 = r0 + ((a - r0) & ~(uintptr_t)15);
            const uintptr_t nlo = a16 < lo ? a16 : lo;
            const uintptr_t nhi = e > hi ? e : hi;
            if (align16(nhi - nlo) > (k ? pb : c->arena)) break;  // k = 0: fits (checked)
            lo = nlo;
            hi = nhi;
            ++k;
            ++i;
        }
        write_descs(c, (lvlip_frame_desc*)s.h_desc, fr + first, k, lo);
        fs.first[cur] = first;
        fs.count[cur] = k;
        rc = launch_frame_piece(c, s, mode, hi - lo, k, out + (size_t)first * ob, (const uint8_t*)lo);
        cur ^= 1;
    }
    return fs.finish(rc, cur);
}

// The region holding every frame (nullptr if there is none), whether the
// frames cover their span densely and in order (span_dense, ctx_impl.h: the
// condition for DMA of whole spans), and whether each one's 16-B span fits
// the arena.  One pass over the frame array on the pool threads (it precedes
// the first piece).
struct RegionScan {
    const Region* r = nullptr;
    bool dense = false;
    bool fits = true;
};
RegionScan scan_region(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n) {
    RegionScan out;
    if (c->regions.empty() || !fr[0].head) return out;
    const Region* r = find_region(c, fr[0].head, fr[0].len);
    if (!r) return out;
    constexpr uint32_t kParts = 256;
    SpanScan part[kParts];
    bool in[kParts], fits[kParts];
    // parts of at least 2048 frames (a small call scans on the calling thread)
    const uint32_t np = n / 2048u < 1u ? 1u : (n / 2048u > kParts ? kParts : n / 2048u);
    const uint8_t *r0 = r->host, *r1 = r->host + r->bytes;
    const uint64_t arena = c->arena;
    parallel_ranges(c, np, 1, [&](uint64_t plo, uint64_t phi) {
        for (uint64_t j = plo; j < phi; ++j) {
            SpanScan p;
            bool pin = true, pfits = true;
            const uint32_t a = (uint32_t)((uint64_t)n * j / np), b = (uint32_t)((uint64_t)n * (j + 1) / np);
            for (uint32_t i = a; i < b; ++i) {
                const uint8_t* h = (const uint8_t*)fr[i].head;
                pin = pin && h && h >= r0 && h + fr[i].len <= r1;
                span_add(p, (uint64_t)(uintptr_t)h, fr[i].len);
                pfits = pfits && align16((uint64_t)fr[i].len + 15u) <= arena;
            }
            part[j] = p;
            in[j] = pin;
            fits[j] = pfits;
        }
    });
    for (uint32_t j = 0; j < np; ++j) {
        if (!in[j]) return RegionScan{};
        out.fits = out.fits && fits[j];
    }
    out.r = r;
    out.dense = out.fits && span_dense(span_merge(part, np), c->span_ratio);
    return out;
}

// Runs the device step over all n frames; out gets n results (records or
// verdicts).  Frames are only read.
int frames_run_(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out,
                PieceDone* cb) {
    DeviceGuard g(c->device);
    begin_gpu_call(c);
    const RegionScan rs = scan_region(c, fr, n);
    if (const Region* r = rs.r) {
        const bool dense = rs.dense;
        // a zero-copy region is read in place, unless the frames lie densely
        // in it and the call sums whole frames: then the copy engine moves
        // the spans, as for a DMA region (the region is pinned and mapped
        // either way; a frame's parse is two dependent reads, which over PCIe
        // cost the in-place kernel ~15 %)
        if (r->flags & LVLIP_REG_ZEROCOPY) {
            if (mode != M_RX && dense) return frames_dma(c, *r, fr, n, mode, out, cb);
            return frames_zerocopy(c, *r, fr, n, mode, out, cb);
        }
        // a DMA region: the spans, except for the header-only RX call, which
        // needs 74 B of each ~800-B frame: those are gathered (mixed frames,
        // 512K: 7.0-7.3 GB/s of headers gathered, 3.2-3.4 read in place,
        // 1.2 as DMA'd spans)
        // DMA only when the frames lie densely and in order in the region (a
        // slab of frames): the spans are copied whole, gaps included
        if (mode != M_RX && dense) return frames_dma(c, *r, fr, n, mode, out, cb);
    }
    // scattered: every frame's slot offset (a prefix sum over the frames'
    // 16-B rounded need_len, in chunks on the pool threads); RX + L4 reads each
    // frame's total length for it (need_len), prefetching ahead
    constexpr uint32_t kChunk = 4096;
    const uint32_t nch = (n + kChunk - 1) / kChunk;
    const size_t lbytes = mode == M_RX_L4 ? align16(sizeof(uint32_t) * (size_t)n) : 0;
    uint8_t* sc = (uint8_t*)scratch2(c, lbytes + 8 * ((size_t)n + 1) + 16 * (size_t)nch);
    if (!sc) return LVLIP_ENOMEM;
    uint32_t* len = mode == M_RX_L4 ? (uint32_t*)sc : nullptr;
    uint64_t* pre = (uint64_t*)(sc + lbytes);
    uint64_t* tot = pre + n + 1;  // per chunk: its slots' bytes, then the largest frame
    const auto t = std::chrono::steady_clock::now();
    parallel_ranges(c, nch, 1, [=](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; ++j) {
            const uint32_t a = (uint32_t)j * kChunk, b = a + kChunk < n ? a + kChunk : n;
            uint64_t sum = 0, big = 0;
            for (uint32_t i = a; i < b; ++i) {
                uint32_t l;
                if (len) {
                    if (i + 16 < b && fr[i + 16].head) __builtin_prefetch(fr[i + 16].head + kEth);
                    l = len[i] = need_len(mode, fr[i]);
                } else {
                    l = need_len(mode, fr[i]);
                }
                pre[i + 1] = sum += align16(l);  // within the chunk, for now
                big = l > big ? l : big;
            }
            tot[2 * j] = sum;
            tot[2 * j + 1] = big;
        }
    });
    uint64_t base = 0;
    bool fits = true;
    for (uint32_t j = 0; j < nch; ++j) {
        const uint64_t b = tot[2 * j];
        tot[2 * j] = base;
        base += b;
        fits = fits && tot[2 * j + 1] <= c->arena;
    }
    pre[0] = 0;
    parallel_ranges(c, nch, 1, [=](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; ++j) {
            const uint32_t a = (uint32_t)j * kChunk, b = a + kChunk < n ? a + kChunk : n;
            for (uint32_t i = a; i < b; ++i) pre[i + 1] += tot[2 * j];
        }
    });
    if (g_trace.on) g_trace.pass1 += Trace::ms(t);
    if (!fits) return LVLIP_ERANGE;  // a frame larger than the arena
    return frames_gather(c, fr, n, mode, out, len, pre, cb);
}

int frames_run(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out,
               PieceDone* cb = nullptr) {
    g_trace = Trace{};
    g_trace.on = c->frame_trace != 0;
    g_trace.t0 = std::chrono::steady_clock::now();
    const int rc = frames_run_(c, fr, n, mode, out, cb);
    if (g_trace.on)
        fprintf(stderr,
                "lvlip frames: mode %d n %u pieces %u total %.3f ms pass1 %.3f gather %.3f wait %.3f apply %.3f\n",
                mode, n, g_trace.pieces, Trace::ms(g_trace.t0), g_trace.pass1, g_trace.gather, g_trace.wait,
                g_trace.apply);
    return rc;
}

// TX: the records of each finished piece are stored into the caller's frames
// while the later pieces run (the raw u16 stores of tcp_transmit_skb /
// icmpv4_reply, L4 field, and ip_send_check, frame + 14 + 10), each frame's
// old field values kept in undo[].  A piece holding a malformed frame (status
// 0: not IPv4, short, ...) stops the applying, and the call then restores
// every frame it wrote, so a malformed frame leaves the batch untouched as
// include/lvlip_skb.h promises.
constexpr uint64_t kApplied = 1ull << 48;  // record bit: this frame was written
struct TxApply final : PieceDone {
    lvlip_csum_ctx* c;
    lvlip_frame* fr;
    uint64_t* rec;
    uint32_t* undo;
    bool bad = false;
    TxApply(lvlip_csum_ctx* c_, lvlip_frame* f, uint64_t* r, uint32_t* u) : c(c_), fr(f), rec(r), undo(u) {}
    bool stop() const override { return bad; }
    void done(uint32_t first, uint32_t k) override {
        if (bad) return;
        for (uint32_t i = first; i < first + k; ++i)
            if (((rec[i] >> 40) & 0xffu) != 1u) {
                bad = true;
                return;
            }
        lvlip_frame* f = fr;
        uint64_t* r = rec;
        uint32_t* u = undo;
        parallel_ranges(c, k, 2048, [=](uint64_t lo, uint64_t hi) {
            for (uint64_t q = first + lo; q < first + hi; ++q) {
                if (q + kPrefetch < first + hi) __builtin_prefetch(f[q + kPrefetch].head + kEth + 10, 1);
                uint8_t* h = f[q].head;
                const uint32_t o = (uint32_t)(r[q] >> 32) & 0xffu;
                uint16_t oh, ol = 0;
                memcpy(&oh, h + kEth + 10, 2);
                if (o) memcpy(&ol, h + o, 2);
                u[q] = oh | ((uint32_t)ol << 16);
                const uint16_t hc = (uint16_t)r[q];
                memcpy(h + kEth + 10, &hc, 2);
                if (o) {
                    const uint16_t lc = (uint16_t)(r[q] >> 16);
                    memcpy(h + o, &lc, 2);
                }
                r[q] |= kApplied;
            }
        });
    }
    // the frames written so far back to their old bytes, in reverse order of
    // writing (the pieces were applied in index order; within a frame the L4
    // field was written after the header's)
    void undo_all(uint32_t n) {
        // last written first: a frame listed twice (in two pieces) gets back
        // the bytes its first entry saved, the ones from before the call
        for (uint32_t q = n; q-- > 0;) {
            if (!(rec[q] & kApplied)) continue;
            uint8_t* h = fr[q].head;
            const uint32_t o = (uint32_t)(rec[q] >> 32) & 0xffu;
            const uint16_t oh = (uint16_t)undo[q], ol = (uint16_t)(undo[q] >> 16);
            if (o) memcpy(h + o, &ol, 2);
            memcpy(h + kEth + 10, &oh, 2);
        }
    }
};

// Whether a frame is longer than the context's arena (the frame calls'
// LVLIP_ERANGE, on every path and on both sides of cpu_max).
bool any_too_long(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n) {
    std::atomic<bool> big{false};
    const uint64_t arena = c->arena;
    parallel_ranges(c, n, 65536, [&big, fr, arena](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i)
            if (fr[i].len > arena) {
                big.store(true, std::memory_order_relaxed);
                return;
            }
    });
    return big.load(std::memory_order_relaxed);
}

}  // namespace

extern "C" {

int lvlip_rx_verify(lvlip_csum_ctx* ctx, const lvlip_frame* frames, uint32_t n, uint32_t flags,
                    uint8_t* verdict) {
    // two checksums per frame at most: n as the _dev call
    if (!ctx || (n && (!frames || !verdict)) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    begin_call(ctx, n);
    const int mode = (flags & LVLIP_RX_VERIFY_L4) ? M_RX_L4 : M_RX;
    // a frame longer than the arena: LVLIP_ERANGE on every path (the header-
    // only call moves at most kHdrWin <= 4096 B of a frame and never refuses)
    if (mode == M_RX_L4 && any_too_long(ctx, frames, n)) return LVLIP_ERANGE;
    if (n <= ctx->cpu_max) {  // the calling thread (lvlip_csum_ctx_set_cpu_max)
        ctx->stats.cpu_calls++;
        return lvlip_rx_verify_cpu(frames, n, flags, verdict);
    }
    const int rc = frames_run(ctx, frames, n, mode, verdict);
    trim_scratch(ctx);
    return rc;
}

int lvlip_tx_checksum(lvlip_csum_ctx* ctx, lvlip_frame* frames, uint32_t n) {
    if (!ctx || (n && !frames) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    begin_call(ctx, n);
    if (n <= ctx->cpu_max) {
        // the calling thread (lvlip_csum_ctx_set_cpu_max), with the GPU
        // path's checks in its order: a NULL or short frame, then a frame
        // longer than the arena, then a malformed one (the CPU call)
        for (uint32_t i = 0; i < n; ++i)
            if (!frames[i].head || frames[i].len < kEth + 20u) return LVLIP_EINVAL;
        if (any_too_long(ctx, frames, n)) return LVLIP_ERANGE;
        ctx->stats.cpu_calls++;
        return lvlip_tx_checksum_cpu(frames, n);
    }
    // the context's scratch: n records, then n undo words
    uint64_t* rec = (uint64_t*)scratch(ctx, 12 * (size_t)n);
    if (!rec) return LVLIP_ENOMEM;
    uint32_t* undo = (uint32_t*)(rec + n);
    // On the pool threads, before the first piece: what needs no frame byte
    // (the rest is the device's status), and the records zeroed (undo_all
    // reads the applied bit of every record, drained or not).  On the calling
    // thread alone this pass took 0.3-1 ms per 512K frames, with the link idle.
    std::atomic<bool> bad{false};
    const lvlip_frame* fr = frames;
    parallel_ranges(ctx, n, 16384, [&bad, fr, rec](uint64_t lo, uint64_t hi) {
        bool b = false;
        for (uint64_t i = lo; i < hi; ++i) b |= !fr[i].head || fr[i].len < kEth + 20u;
        memset(rec + lo, 0, 8 * (size_t)(hi - lo));
        if (b) bad.store(true, std::memory_order_relaxed);
    });
    if (bad.load(std::memory_order_relaxed)) return LVLIP_EINVAL;
    if (any_too_long(ctx, frames, n)) return LVLIP_ERANGE;
    TxApply ap(ctx, frames, rec, undo);
    int rc = frames_run(ctx, frames, n, M_TX, (uint8_t*)rec, &ap);
    if (rc == LVLIP_OK && ap.bad) rc = LVLIP_EINVAL;
    if (rc != LVLIP_OK) ap.undo_all(n);  // a malformed frame (or a failure): every frame as it was
    trim_scratch(ctx);
    return rc;
}

}  // extern "C"
