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
//
// LVLIP_FRAME_PATH=hostplan (read at context creation) runs round 4's path
// instead, which plans every frame on the CPU and gathers the two checksummed
// pieces per frame through lvlip_csum_batch_host (skb_batch.c), for A/B.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ctx_impl.h"

extern "C" {
// skb_batch.c: round 4's host-plan path (hidden)
int lvlip_rx_verify_hostplan(lvlip_csum_ctx* ctx, const lvlip_frame* frames, uint32_t n, uint32_t flags,
                             uint8_t* verdict);
int lvlip_tx_checksum_hostplan(lvlip_csum_ctx* ctx, lvlip_frame* frames, uint32_t n);
}

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

// Frames per piece: the slot's descriptor array and its result buffer.
inline uint32_t frames_per_piece(const lvlip_csum_ctx* c, int mode) {
    const uint64_t by_out = (uint64_t)c->max_desc * sizeof(uint16_t) / out_bytes(mode);
    return by_out < c->max_desc ? (uint32_t)by_out : c->max_desc;
}

// One piece of k frames (descriptors in the slot's pinned h_desc) through the
// device step, as csum_ctx.cpp's launch_piece: the frames come from the
// slot's pinned arena, from `src` (a registered region: DMA), or are read in
// place at `dev_base` (zero-copy).  A piece of at most direct_max bytes skips
// the copies: the kernel reads the arena (or region) and the descriptors over
// PCIe and writes its results into the pinned result buffer.
int launch_frame_piece(lvlip_csum_ctx* c, Slot& s, int mode, uint64_t bytes, uint32_t k, void* user_out,
                       const uint8_t* src = nullptr, const uint8_t* dev_base = nullptr) {
    hipError_t e;
    const size_t nout = (size_t)k * out_bytes(mode);
    if (bytes <= c->direct_max && (dev_base || !src)) {
        const int rc = lvlip_frames_host_launch(mode, dev_base ? dev_base : s.dh_bytes,
                                                (const lvlip_frame_desc*)s.dh_desc, k, s.dh_out, s.stream);
        if (rc != LVLIP_OK) return rc;
        return arm_slot(c, s, user_out, nout);
    }
    if (!dev_base) {
        const uint64_t nb = src ? bytes : align16(bytes);
        if ((e = hipMemcpyAsync(s.d_bytes, src ? src : s.h_bytes, nb, hipMemcpyHostToDevice, s.stream)) !=
            hipSuccess)
            return fail(c, e, "H2D frames");
    }
    if ((e = hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)k * sizeof(lvlip_frame_desc), hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess)
        return fail(c, e, "H2D frame descriptors");
    const int rc = lvlip_frames_host_launch(mode, dev_base ? dev_base : s.d_bytes,
                                            (const lvlip_frame_desc*)s.d_desc, k, s.d_out, s.stream);
    if (rc != LVLIP_OK) return rc;
    if ((e = hipMemcpyAsync(s.h_out, s.d_out, nout, hipMemcpyDeviceToHost, s.stream)) != hipSuccess)
        return fail(c, e, "D2H frame results");
    return arm_slot(c, s, user_out, nout);
}

// Scattered frames: each frame's need_len bytes (len[i] when given) copied
// whole into the next 16-B aligned slot of the pinned arena.
int frames_gather(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out,
                  const uint32_t* len) {
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        lvlip_frame_desc* hd = (lvlip_frame_desc*)s.h_desc;
        uint64_t off = 0;
        uint32_t k = 0;
        const uint32_t first = i;
        while (i < n && k < fmax) {
            const uint32_t l = len ? len[i] : need_len(mode, fr[i]);
            if (off + l > (k ? c->piece : c->arena)) break;  // k = 0: fits (checked by the caller)
            hd[k].offset = off;
            hd[k].len = l;
            hd[k].reserved = 0;
            off = align16(off + l);
            ++k;
            ++i;
        }
        {
            uint8_t* dst = s.h_bytes;
            const lvlip_frame* src = fr + first;
            parallel_ranges(c, k, 256, [=](uint64_t lo, uint64_t hi) {
                for (uint64_t q = lo; q < hi; ++q)
                    if (hd[q].len) memcpy(dst + hd[q].offset, src[q].head, hd[q].len);
            });
        }
        rc = launch_frame_piece(c, s, mode, off ? off : 16, k, out + (size_t)first * ob);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

// Frames inside one LVLIP_REG_ZEROCOPY region: descriptors only, offsets from
// the region's first byte rounded down to 16; the kernel reads in place.
int frames_zerocopy(lvlip_csum_ctx* c, const Region& r, const lvlip_frame* fr, uint32_t n, int mode,
                    uint8_t* out) {
    const uint8_t* h0 = (const uint8_t*)((uintptr_t)r.host & ~(uintptr_t)15);
    const uint8_t* d0 = r.dev - (r.host - h0);
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        lvlip_frame_desc* hd = (lvlip_frame_desc*)s.h_desc;
        const uint32_t first = i;
        const uint32_t k = n - i < fmax ? n - i : fmax;
        uint64_t bytes = 0;
        for (uint32_t q = 0; q < k; ++q) {
            hd[q].offset = (uint64_t)(fr[first + q].head - h0);
            hd[q].len = fr[first + q].len;
            hd[q].reserved = 0;
            bytes += fr[first + q].len;
        }
        i += k;
        rc = launch_frame_piece(c, s, mode, bytes ? bytes : 16, k, out + (size_t)first * ob, nullptr, d0);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

// Frames inside one LVLIP_REG_DMA region: a piece is a run of frames whose
// byte span [lo, hi) (lo rounded down to 16, so every frame keeps its address
// mod 16) fits the piece size; the copy engine reads the span from the region.
int frames_dma(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out) {
    const uint32_t fmax = frames_per_piece(c, mode), ob = out_bytes(mode);
    int cur = 0;
    uint32_t i = 0;
    int rc = LVLIP_OK;
    while (i < n && rc == LVLIP_OK) {
        Slot& s = c->slot[cur];
        if ((rc = drain(c, s)) != LVLIP_OK) break;
        const uint32_t first = i;
        uintptr_t lo = ~(uintptr_t)0, hi = 0;
        uint32_t k = 0;
        while (i < n && k < fmax) {
            const uintptr_t a = (uintptr_t)fr[i].head, e = a + fr[i].len;
            const uintptr_t nlo = (a & ~(uintptr_t)15) < lo ? (a & ~(uintptr_t)15) : lo;
            const uintptr_t nhi = e > hi ? e : hi;
            if (align16(nhi) - nlo > (k ? c->piece : c->arena)) break;  // k = 0: fits (checked)
            lo = nlo;
            hi = nhi;
            ++k;
            ++i;
        }
        lvlip_frame_desc* hd = (lvlip_frame_desc*)s.h_desc;
        for (uint32_t q = 0; q < k; ++q) {
            hd[q].offset = (uint64_t)((uintptr_t)fr[first + q].head - lo);
            hd[q].len = fr[first + q].len;
            hd[q].reserved = 0;
        }
        rc = launch_frame_piece(c, s, mode, hi - lo, k, out + (size_t)first * ob, (const uint8_t*)lo);
        cur ^= 1;
    }
    return finish_pieces(c, rc);
}

// The region holding every frame, or nullptr.
const Region* one_region(const lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n) {
    if (c->regions.empty()) return nullptr;
    const Region* r = nullptr;
    for (uint32_t i = 0; i < n; ++i) {
        if (!fr[i].head) return nullptr;
        const Region* ri = (r && (const uint8_t*)fr[i].head >= r->host &&
                            (const uint8_t*)fr[i].head + fr[i].len <= r->host + r->bytes)
                               ? r
                               : find_region(c, fr[i].head, fr[i].len);
        if (!ri || (r && ri != r)) return nullptr;
        r = ri;
    }
    return r;
}

// Runs the device step over all n frames; out gets n results (records or
// verdicts).  Frames are only read.
int frames_run(lvlip_csum_ctx* c, const lvlip_frame* fr, uint32_t n, int mode, uint8_t* out) {
    DeviceGuard g(c->device);
    if (const Region* r = one_region(c, fr, n)) {
        if (r->flags & LVLIP_REG_ZEROCOPY) return frames_zerocopy(c, *r, fr, n, mode, out);
        // DMA only when the frames lie densely in the region (a slab of
        // frames): the spans are copied whole, gaps included
        uintptr_t lo = ~(uintptr_t)0, hi = 0;
        uint64_t sum = 0;
        bool fits = true;
        for (uint32_t i = 0; i < n; ++i) {
            const uintptr_t a = (uintptr_t)fr[i].head;
            lo = a < lo ? a : lo;
            hi = a + fr[i].len > hi ? a + fr[i].len : hi;
            sum += fr[i].len;
            fits = fits && align16(fr[i].len + 15u) <= c->arena;
        }
        if (fits && hi - lo <= 2 * sum + (1ull << 20)) return frames_dma(c, fr, n, mode, out);
    }
    // scattered: RX + L4 first reads each frame's total length (need_len),
    // on the pool threads, prefetching ahead
    uint32_t* len = nullptr;
    if (mode == M_RX_L4) {
        len = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
        if (!len) return LVLIP_ENOMEM;
        parallel_ranges(c, n, 4096, [=](uint64_t lo, uint64_t hi) {
            for (uint64_t i = lo; i < hi; ++i) {
                if (i + 16 < hi && fr[i + 16].head) __builtin_prefetch(fr[i + 16].head + kEth);
                len[i] = need_len(mode, fr[i]);
            }
        });
    }
    int rc = LVLIP_OK;
    for (uint32_t i = 0; i < n && rc == LVLIP_OK; ++i)
        if ((uint64_t)(len ? len[i] : need_len(mode, fr[i])) > c->arena) rc = LVLIP_ERANGE;
    if (rc == LVLIP_OK) rc = frames_gather(c, fr, n, mode, out, len);
    free(len);
    return rc;
}

}  // namespace

extern "C" {

int lvlip_rx_verify(lvlip_csum_ctx* ctx, const lvlip_frame* frames, uint32_t n, uint32_t flags,
                    uint8_t* verdict) {
    // two checksums per frame at most: n as the _dev call
    if (!ctx || (n && (!frames || !verdict)) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    if (ctx->frame_hostplan) return lvlip_rx_verify_hostplan(ctx, frames, n, flags, verdict);
    return frames_run(ctx, frames, n, (flags & LVLIP_RX_VERIFY_L4) ? M_RX_L4 : M_RX, verdict);
}

int lvlip_tx_checksum(lvlip_csum_ctx* ctx, lvlip_frame* frames, uint32_t n) {
    if (!ctx || (n && !frames) || n > LVLIP_MAX_BATCH / 2u) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    if (ctx->frame_hostplan) return lvlip_tx_checksum_hostplan(ctx, frames, n);
    for (uint32_t i = 0; i < n; ++i)  // what needs no frame byte (the rest: the device's status)
        if (!frames[i].head || frames[i].len < kEth + 20u) return LVLIP_EINVAL;
    uint64_t* rec = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
    if (!rec) return LVLIP_ENOMEM;
    int rc = frames_run(ctx, frames, n, M_TX, (uint8_t*)rec);
    // tx_frame_ok of every frame (status 1) before any frame is written
    for (uint32_t i = 0; i < n && rc == LVLIP_OK; ++i)
        if (((rec[i] >> 40) & 0xffu) != 1u) rc = LVLIP_EINVAL;
    if (rc == LVLIP_OK) {
        // the raw u16 stores of tcp_transmit_skb / icmpv4_reply (L4 field) and
        // ip_send_check (header field, frame + 14 + 10)
        lvlip_frame* fr = frames;
        parallel_ranges(ctx, n, 8192, [=](uint64_t lo, uint64_t hi) {
            for (uint64_t i = lo; i < hi; ++i) {
                if (i + 16 < hi) __builtin_prefetch(fr[i + 16].head + kEth + 10, 1);
                const uint64_t r = rec[i];
                uint8_t* h = fr[i].head;
                const uint16_t hc = (uint16_t)r;
                memcpy(h + kEth + 10, &hc, 2);
                const uint32_t o = (uint32_t)(r >> 32) & 0xffu;
                if (o) {
                    const uint16_t lc = (uint16_t)(r >> 16);
                    memcpy(h + o, &lc, 2);
                }
            }
        });
    }
    free(rec);
    return rc;
}

}  // extern "C"
