// flat_src.h — where k_flat2 (csum_kernels.hip) takes its entries from and
// where its results go.
//
//   get(i, ctx): entry i as {offset, len, start_sum}; ctx is a word the source
//       wants back in put
//   put(i, c, ctx, valid, addr): called by every thread of the workgroup (valid =
//       i < n), so a source may exchange results between neighbouring lanes;
//       addr is the entry's first byte (when its len > 0)
//
// DescSrc is the plain batch of include/lvlip_csum.h: a descriptor array in, a
// u16 array out.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

namespace lvlip {

struct DescSrc {
    static constexpr bool WIN_SUM = false;  // no parse window (see FrameSrc)
    const lvlip_csum_desc* descs;
    uint16_t* out;
    // One 16-B load: read field by field, hipcc splits the descriptor into a
    // len load and an offset load behind it, two round trips at the start of
    // every tile.
    __device__ __forceinline__ lvlip_csum_desc get(uint32_t i, uint32_t& ctx) const {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const v4u gv4u;
        ctx = 0;
        const v4u v = *reinterpret_cast<gv4u*>(reinterpret_cast<uint64_t>(descs + i));
        lvlip_csum_desc d;
        d.offset = ((uint64_t)v.y << 32) | v.x;
        d.len = (int32_t)v.z;
        d.start_sum = v.w;
        return d;
    }
    __device__ __forceinline__ void put(uint32_t i, uint16_t c, uint32_t, bool valid, uint64_t) const {
        if (valid) out[i] = c;
    }
    __device__ __forceinline__ const lvlip_csum_desc* desc_ptr(uint32_t i) const { return descs + i; }
};

// FrameSrc<MODE>: f1/f2 of SURVEY.md §8f on frames in HBM (include/lvlip_skb.h).
// Phase 1 of the sweep parses each frame's header bytes into its checksum
// entries; phase 4 applies the results to the frame (TX) or turns them into
// ip_rcv's verdict (RX).  That fuses the plan and apply steps into the
// checksum kernel: no descriptor, plan or result array goes through HBM, and
// the TX field writes land in lines the sweep has just read.
constexpr uint32_t FR_ETH = 14;
constexpr uint32_t FR_PENDING = 0x80;   // verdict waits for the header checksum
constexpr uint32_t FR_HAS_HDR = 0x100;  // plan word: the IPv4 header entry exists
constexpr uint32_t FR_HAS_L4 = 0x200;   // plan word: the TCP/ICMP entry exists
// FR_TX_REC: TX's decisions and sums, but the two fields go to a record per
// frame instead of into the frame (the host frame calls, frames_host.cpp,
// apply them to the caller's frames once every frame of the batch is known to
// be well formed).  Record (u64): bits 0-15 the IPv4 header field, 16-31 the
// TCP/ICMP field, 32-39 the TCP/ICMP field's offset from the frame's first
// byte (0 = the frame has no such field), 40-47 status (1 filled, 0 malformed).
// FR_ECHO: f4's LVLIP_ECHO_FULL (lvlip_icmp_echo_reply_dev_ex): one entry per
// frame, the ICMP message of an echo request, seeded so that its result is
// icmpv4_reply's field; put() writes the reply's type and field.
enum { FR_TX = 0, FR_RX = 1, FR_RX_L4 = 2, FR_TX_REC = 3, FR_ECHO = 4 };
constexpr bool fr_is_tx(int mode) { return mode == FR_TX || mode == FR_TX_REC; }

__device__ __forceinline__ uint32_t fr_be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t fr_le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t fr_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t fr_bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }
// src/tcp.c:92-95: whole u32 words, the carry out of bit 31 lost (lvlip_pseudo_sum)
__device__ __forceinline__ uint32_t fr_pseudo_lossy(uint32_t s, uint32_t d, uint32_t proto, uint32_t len) {
    return s + d + fr_bswap16(proto) + fr_bswap16(len);
}
// the same words as 16-bit halves (lvlip_pseudo_sum_rfc)
__device__ __forceinline__ uint32_t fr_pseudo_rfc(uint32_t s, uint32_t d, uint32_t proto, uint32_t len) {
    return (s & 0xffffu) + (s >> 16) + (d & 0xffffu) + (d >> 16) + fr_bswap16(proto) + fr_bswap16(len);
}
__device__ __forceinline__ lvlip_csum_desc fr_mk(uint64_t off, uint32_t len, uint32_t start) {
    lvlip_csum_desc d;
    d.offset = off;
    d.len = (int32_t)len;
    d.start_sum = start;
    return d;
}

// The header bytes a frame's decisions read, [12, 56) of the frame, from four
// 16-B aligned loads issued together (instead of one dependent byte load per
// field): A[j] = frame bytes 12+4j .. 15+4j, little-endian.  A chunk is read
// only when it holds a byte of the frame, so it lies inside the frame buffer
// (its length is rounded up to 16 B, include/lvlip_skb.h); bytes past the
// frame's len read as whatever the chunk holds and are never used.
struct FrWin {
    uint32_t A[11];
    uint4 raw[4];     // the window's chunks as loaded (zero past the frame's end)
    uint64_t abase;   // address of raw[0]
    // safe: a readable 16-B aligned address for a frame with no byte in the
    // window (a chunk of the frame's own descriptor).  NCH = 3 loads only the
    // first three chunks (frame bytes [12, cov) with cov = 60 - ((h + 12) & 15)
    // >= 45 are then valid; the header-only RX kernel, which reads no field
    // past byte 23 and sums the header words past cov from memory).
    template <int NCH = 4>
    __device__ __forceinline__ void load(const uint8_t* h, uint32_t len, uint64_t safe) {
        const uint64_t p = reinterpret_cast<uint64_t>(h) + 12u;
        const uint64_t a = p & ~15ull, end = reinterpret_cast<uint64_t>(h) + len;
        const uint64_t a0 = a < end ? a : len ? reinterpret_cast<uint64_t>(h) & ~15ull : safe;
        // four loads back to back, no branch between them: a chunk past the
        // frame reloads a valid one and is then zeroed
        // (one asm statement, waited inside it: the compiler would otherwise
        // sink each load into the branch that first reads it)
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        v4u c[4];
        uint64_t ad[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) ad[k] = a + 16u * k < end ? a + 16u * k : a0;
        if (NCH == 4) {
            asm volatile(
                "global_load_dwordx4 %0, %4, off\n\t"
                "global_load_dwordx4 %1, %5, off\n\t"
                "global_load_dwordx4 %2, %6, off\n\t"
                "global_load_dwordx4 %3, %7, off\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3])
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3])
                : "memory");
        } else {
            asm volatile(
                "global_load_dwordx4 %0, %3, off\n\t"
                "global_load_dwordx4 %1, %4, off\n\t"
                "global_load_dwordx4 %2, %5, off\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2])
                : "v"(ad[0]), "v"(ad[1]), "v"(ad[2])
                : "memory");
            c[3] = v4u{0u, 0u, 0u, 0u};
        }
        uint32_t W[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t m = (k < NCH && a + 16u * k < end) ? 0xffffffffu : 0u;
            W[4 * k] = c[k].x & m;
            W[4 * k + 1] = c[k].y & m;
            W[4 * k + 2] = c[k].z & m;
            W[4 * k + 3] = c[k].w & m;
            raw[k] = make_uint4(W[4 * k], W[4 * k + 1], W[4 * k + 2], W[4 * k + 3]);
        }
        abase = a;
        // L[j] = W[j + q] by bit selects (no divergent branch), then one
        // alignbyte per output dword
        const uint32_t q = (uint32_t)(p & 15u) >> 2, r = (uint32_t)p & 3u;
        const uint32_t m1 = 0u - (q & 1u), m2 = 0u - (q >> 1);
        uint32_t L[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const uint32_t t01 = (W[j] & ~m1) | (W[j + 1] & m1);
            const uint32_t t23 = (W[j + 2] & ~m1) | (W[j + 3] & m1);
            L[j] = (t01 & ~m2) | (t23 & m2);
        }
#pragma unroll
        for (int j = 0; j < 11; ++j) A[j] = __builtin_amdgcn_alignbyte(L[j + 1], L[j], r);
    }
    // byte o of the frame, 12 <= o < 56 (o a constant)
    __device__ __forceinline__ uint32_t b(uint32_t o) const { return (A[(o - 12u) >> 2] >> (8u * ((o - 12u) & 3u))) & 0xffu; }
    __device__ __forceinline__ uint32_t be16(uint32_t o) const { return (b(o) << 8) | b(o + 1u); }
    __device__ __forceinline__ uint32_t le16(uint32_t o) const { return b(o) | (b(o + 1u) << 8); }
    __device__ __forceinline__ uint32_t le32(uint32_t o) const { return le16(o) | (le16(o + 2u) << 16); }
};

// TX plan-word bits of the whole-sector field stores (FrameSrc<FR_TX, SEC>,
// SEC > 0): the aligned SEC-byte block around the header / L4 checksum field
// lies wholly inside the frame; both fields share one block.  Bits 24-31 hold
// the L4 field's distance from the header field.
constexpr uint32_t FR_SEC_HDR = 0x2;
constexpr uint32_t FR_SEC_L4 = 0x4;
constexpr uint32_t FR_SEC_SHARED = 0x8;

// A u16 stored raw at byte o (0 <= o <= 4N - 2, any parity) of N dwords.
template <int N>
__device__ __forceinline__ void fr_patch16(uint32_t (&v)[N], uint32_t o, uint32_t c) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int sh = 8 * ((int)o - 4 * k);
        if (sh >= -8 && sh <= 24) {
            const uint32_t val = sh < 0 ? (c >> 8) : (c << sh);
            const uint32_t m = sh < 0 ? 0xffu : (0xffffu << sh);
            v[k] = (v[k] & ~m) | (val & m);
        }
    }
}

// The SEC-byte block at `sa` (SEC-aligned, inside one frame) rewritten whole
// with one or two checksum fields patched in: loaded, patched, stored back
// with nontemporal 16-B stores.  The other bytes are the frame's own, which
// nothing else writes during the call, so they are stored back unchanged.
template <int SEC>
__device__ __forceinline__ void fr_block_put(uint64_t sa, uint32_t o0, uint32_t c0, bool two, uint32_t o1,
                                             uint32_t c1) {
    constexpr int NQ = SEC / 16;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) v4u gv4u;
    v4u q[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) q[k] = *reinterpret_cast<gv4u*>(sa + 16u * k);
    uint32_t v[4 * NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        v[4 * k] = q[k].x;
        v[4 * k + 1] = q[k].y;
        v[4 * k + 2] = q[k].z;
        v[4 * k + 3] = q[k].w;
    }
    fr_patch16<4 * NQ>(v, o0, c0);
    if (two) fr_patch16<4 * NQ>(v, o1, c1);
#pragma unroll
    for (int k = 0; k < NQ; ++k)
        __builtin_nontemporal_store(v4u{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]},
                                    reinterpret_cast<gv4u*>(sa + 16u * k));
}

// A u16 field stored raw at `a` with an explicit cache policy (TX: FrameSrc's
// STP): 2 sc0, 3 sc1, 4 sc0 sc1, 5 nt sc1, 6 nt sc0 sc1 (the product's;
// vector stores, an odd address takes two byte stores).
template <int STP>
__device__ __forceinline__ void fr_store16_pol(uint64_t a, uint32_t c) {
#define LVLIP_ST(BITS)                                                                                      \
    if (a & 1ull) {                                                                                         \
        const uint32_t hi = c >> 8;                                                                         \
        asm volatile("global_store_byte %0, %1, off " BITS "\n\tglobal_store_byte %2, %3, off " BITS         \
                     ::"v"(a), "v"(c), "v"(a + 1ull), "v"(hi) : "memory");                                  \
    } else {                                                                                                \
        asm volatile("global_store_short %0, %1, off " BITS ::"v"(a), "v"(c) : "memory");                    \
    }
    if constexpr (STP == 2) { LVLIP_ST("sc0") }
    else if constexpr (STP == 3) { LVLIP_ST("sc1") }
    else if constexpr (STP == 4) { LVLIP_ST("sc0 sc1") }
    else if constexpr (STP == 5) { LVLIP_ST("nt sc1") }
    else { LVLIP_ST("nt sc0 sc1") }
#undef LVLIP_ST
}

// An echo reply's type and checksum field at the message's first bytes m
// (icmpv4_reply: type ICMP_V4_REPLY, src/icmpv4.c:45; the field stored raw,
// :47).  STP 0: three byte stores (type, then the field's two bytes); 2-6:
// two u16 stores with fr_store16_pol's policy, {type 0, code 0} then the
// field (the request's code is 0: both callers checked it).
template <int STP>
__device__ __forceinline__ void fr_store_echo_reply(uint8_t* m, uint32_t field) {
    if constexpr (STP == 7) {  // lab timing only: no reply written (wrong bytes)
        (void)m, (void)field;
    } else if constexpr (STP == 0) {
        m[0] = 0u;
        m[2] = (uint8_t)field;
        m[3] = (uint8_t)(field >> 8);
    } else {
        fr_store16_pol<STP>(reinterpret_cast<uint64_t>(m), 0u);
        fr_store16_pol<STP>(reinterpret_cast<uint64_t>(m) + 2u, field & 0xffffu);
    }
}
// The product's echo-reply stores (k_echo_reply, FrameSrc<FR_ECHO>).
constexpr int kEchoStore = 0;

// The decisions are those of skb_batch.c (host), which cites the reference line
// of each.  Entry slots: RX with L4 and TX use two per frame (lanes 2f, 2f+1 of
// one wave, so the pair exchanges results by shuffle), RX header-only one.  An
// entry the frame does not have is empty (len 0).  Header bytes come from the
// FrWin window; a field outside it is read with byte loads, never past the
// frame's len.
// SEC (TX, lab A/B): 0 = each field stored as 2 bytes; 32 / 64 = the aligned
// SEC-byte block around a field is rewritten whole when it lies inside the
// frame (no partial-sector write reaches the memory side), 2-B stores
// otherwise.
// STP (TX): 0 = the launcher's nt_store flag (nontemporal or plain stores,
// lab A/B); 2-6 = fr_store16_pol's cache policies; the product's TX fill
// stores `nt sc0 sc1` (6).
template <int MODE, int SEC = 0, int STP = 0>
struct FrameSrc {
    static_assert(SEC == 0 || SEC == 32 || SEC == 64, "field block size");
    static_assert(STP == 0 || (STP >= 2 && STP <= 6) || (MODE == FR_ECHO && STP == 7), "field store policy");
    const uint8_t* base;             // the frames' bytes
    uint8_t* wbase;                  // the same, writable (TX)
    const lvlip_frame_desc* frames;  // this launch's first frame
    uint8_t* out8;                   // RX: verdict[], TX: status[] (may be null)
    bool nt_store = false;           // TX: nontemporal field stores (the launcher's default)
    uint64_t* rec = nullptr;         // FR_TX_REC: one record per frame
    static constexpr uint32_t SLOTS = (MODE == FR_RX || MODE == FR_ECHO) ? 1u : 2u;
    // the frame descriptor of entry i (k_flat2's PFA prefetch: 16 B, like a
    // batch descriptor)
    __device__ __forceinline__ const lvlip_frame_desc* desc_ptr(uint32_t i) const { return frames + i / SLOTS; }
    // The parse window's chunks are in registers after get(): k_flat2 sums
    // each entry's bytes inside the window there and sweeps only the rest, so
    // no frame byte is read from HBM twice.
    static constexpr bool WIN_SUM = true;

    // ip_rcv's decisions (src/ip_input.c:17-60) -> entries {header, L4} and the
    // plan word (verdict so far | flags)
    __device__ __forceinline__ void parse_rx(const lvlip_frame_desc& fd, const FrWin& x,
                                             lvlip_csum_desc& d0, lvlip_csum_desc& d1,
                                             uint32_t& w) const {
        uint32_t v = 0;
        if (fd.len < FR_ETH + 20u) {
            v = LVLIP_RX_SHORT;
        } else if (x.be16(12) != 0x0800u) {  // netdev_receive, src/netdev.c:67-80
            v = LVLIP_RX_NOT_IP;
        } else {
            const uint32_t ver = x.b(14) >> 4, ihl = x.b(14) & 0x0fu;
            if (ver != 4u) {  // src/ip_input.c:22
                v = LVLIP_RX_BAD_VERSION;
            } else if (ihl < 5u) {  // src/ip_input.c:27
                v = LVLIP_RX_BAD_IHL;
            } else if (x.b(22) == 0u) {  // src/ip_input.c:32
                v = LVLIP_RX_TTL0;
            } else if (fd.len < FR_ETH + ihl * 4u) {
                v = LVLIP_RX_SHORT;
            } else {
                d0 = fr_mk(fd.offset + FR_ETH, ihl * 4u, 0);  // src/ip_input.c:38
                w |= FR_HAS_HDR;
                const uint32_t proto = x.b(23);
                if (proto != 6u && proto != 1u) {  // src/ip_input.c:51-60
                    v = FR_PENDING | LVLIP_RX_UNKNOWN_PROTO;
                } else if (MODE == FR_RX_L4) {
                    const uint32_t iplen = x.be16(16);
                    if (iplen < ihl * 4u || fd.len < FR_ETH + iplen) {
                        v = FR_PENDING | LVLIP_RX_SHORT;
                    } else {
                        const uint32_t l4len = iplen - ihl * 4u;
                        const uint32_t seed = proto == 6u ? fr_pseudo_rfc(x.le32(26), x.le32(30), 6u, l4len) : 0u;
                        d1 = fr_mk(fd.offset + FR_ETH + ihl * 4u, l4len, seed);
                        w |= FR_HAS_L4;
                    }
                }
            }
        }
        w |= v;
    }

    // the TX decisions of lvlip_tx_plan -> entries {header, L4} (address order,
    // as the sweep wants its entries); plan word =
    // filled | L4 flag | the L4 checksum field's offset in the L4 entry << 16
    __device__ __forceinline__ void parse_tx(const lvlip_frame_desc& fd, const uint8_t* h, const FrWin& x,
                                             lvlip_csum_desc& d0, lvlip_csum_desc& d1,
                                             uint32_t& w) const {
        if (fd.len < FR_ETH + 20u) return;
        const uint32_t ihl = x.b(14) & 0x0fu, iplen = x.be16(16), proto = x.b(23);
        if ((x.b(14) >> 4) != 4u || ihl < 5u || iplen < ihl * 4u || fd.len < FR_ETH + iplen) return;
        const uint32_t l4 = FR_ETH + ihl * 4u, l4len = iplen - ihl * 4u;
        // each field's current u16 is taken out of the seed (skb_batch.c): the
        // same sum as the reference's zero-then-checksum, mod 2^32.  The L4
        // field is in the window for ihl 5-6, else one more (dependent) read.
        if (proto == 6u && l4len >= 20u) {  // src/tcp_output.c:110,126
            const uint32_t cur = ihl == 5u ? x.le16(50) : ihl == 6u ? x.le16(54) : fr_le16(h + l4 + 16);
            d1 = fr_mk(fd.offset + l4, l4len, fr_pseudo_lossy(x.le32(26), x.le32(30), 6u, l4len) - cur);
            w = FR_HAS_L4 | (16u << 16);
        } else if (proto == 1u && l4len >= 4u) {  // src/icmpv4.c:46-47
            const uint32_t cur = ihl == 5u ? x.le16(36) : ihl == 6u ? x.le16(40) : fr_le16(h + l4 + 2);
            d1 = fr_mk(fd.offset + l4, l4len, 0u - cur);
            w = FR_HAS_L4 | (2u << 16);
        }
        d0 = fr_mk(fd.offset + FR_ETH, ihl * 4u, 0u - x.le16(24));  // src/ip_output.c:42,53
        w |= 1u;
        if constexpr (MODE == FR_TX_REC) w |= l4 << 24;  // the L4 entry's offset in the frame (<= 74)
        if constexpr (SEC > 0) {
            // which fields' SEC-byte blocks lie wholly inside [frame, frame + len).
            // A field at the last byte of a block straddles two blocks: then
            // neither field of the frame is block-stored (a whole-block
            // rewrite must never hold a byte another lane stores separately).
            const uint64_t fs = reinterpret_cast<uint64_t>(h), fe = fs + fd.len;
            const uint64_t fh = fs + FR_ETH + 10u, bh = fh & ~(uint64_t)(SEC - 1);
            const bool has_l4 = (w & FR_HAS_L4) != 0u;
            const uint64_t fl = fs + l4 + ((w >> 16) & 0xffu), bl = fl & ~(uint64_t)(SEC - 1);
            const bool straddle = (fh & (SEC - 1)) == SEC - 1 || (has_l4 && (fl & (SEC - 1)) == SEC - 1);
            if (!straddle) {
                if (bh >= fs && bh + SEC <= fe) w |= FR_SEC_HDR;
                if (has_l4) {
                    if (bl >= fs && bl + SEC <= fe) w |= FR_SEC_L4;
                    if (bl == bh && (w & FR_SEC_HDR)) w |= FR_SEC_SHARED;
                    w |= (uint32_t)(fl - fh) << 24;  // <= 60 + 16 - 10
                }
            }
        }
    }

    // the checks of lvlip_icmp_echo_reply_fill (skb_batch.c): an IPv4 ICMP echo
    // request (type 8, code 0) whose message lies inside the frame -> its
    // message as the entry, seeded with -(0x0008 + HC): the reply's message is
    // the request's with word 0 (type 8, code 0: LE 0x0008) and word 1 (the
    // field HC) zeroed, so its u32 word sum is W - 0x0008 - HC, and the
    // entry's result is icmpv4_reply's field (src/icmpv4.c:45-47) for any
    // request, verified or not.  Plan word: 1 = a request.
    __device__ __forceinline__ void parse_echo(const lvlip_frame_desc& fd, const uint8_t* h, const FrWin& x,
                                               lvlip_csum_desc& d0, uint32_t& w) const {
        if (fd.len < FR_ETH + 20u) return;
        const uint32_t ver = x.b(14) >> 4, ihl = x.b(14) & 0x0fu, iplen = x.be16(16);
        const uint32_t l4 = FR_ETH + ihl * 4u;
        if (ver != 4u || ihl < 5u || x.b(23) != 1u || iplen < ihl * 4u + 4u || fd.len < FR_ETH + iplen) return;
        // type, code and checksum from the window when it holds them (ihl <= 9)
        uint32_t type, code, hc;
        if (l4 + 4u <= 56u) {
            const uint32_t q = (ihl == 5u) ? x.le32(34) : (ihl == 6u) ? x.le32(38) : (ihl == 7u) ? x.le32(42)
                             : (ihl == 8u) ? x.le32(46) : x.le32(50);
            type = q & 0xffu;
            code = (q >> 8) & 0xffu;
            hc = q >> 16;
        } else {
            type = h[l4];
            code = h[l4 + 1u];
            hc = fr_le16(h + l4 + 2u);
        }
        if (type != 8u || code != 0u) return;
        d0 = fr_mk(fd.offset + l4, iplen - ihl * 4u, 0u - 0x0008u - hc);
        w = 1u;
    }

    __device__ __forceinline__ lvlip_csum_desc get(uint32_t i, uint32_t& w, uint4* win = nullptr,
                                                   uint64_t* wa = nullptr) const {
        // the descriptor's two words in flight together (the compiler would
        // load len, branch on it, then load offset)
        typedef uint32_t v2u __attribute__((ext_vector_type(2)));
        v2u fo, fl;
        asm volatile(
            "global_load_dwordx2 %0, %2, off\n\t"
            "global_load_dwordx2 %1, %2, off offset:8\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(fo), "=&v"(fl)
            : "v"(reinterpret_cast<uint64_t>(frames + i / SLOTS))
            : "memory");
        lvlip_frame_desc fd;
        fd.offset = (uint64_t)fo.x | ((uint64_t)fo.y << 32);
        fd.len = fl.x;
        fd.reserved = 0;
        const uint8_t* h = base + fd.offset;
        FrWin x;
        x.load(h, fd.len, reinterpret_cast<uint64_t>(frames + i / SLOTS) & ~15ull);
        lvlip_csum_desc d0 = fr_mk(0, 0, 0), d1 = fr_mk(0, 0, 0);
        w = 0;
        if (fr_is_tx(MODE))
            parse_tx(fd, h, x, d0, d1, w);
        else if (MODE == FR_ECHO)
            parse_echo(fd, h, x, d0, w);
        else
            parse_rx(fd, x, d0, d1, w);
        if (win) {
#pragma unroll
            for (int k = 0; k < 4; ++k) win[k] = x.raw[k];
            *wa = x.abase;
        }
        return (SLOTS == 2u && (i & 1u)) ? d1 : d0;
    }

    // TX writes the two checksum fields after the workgroup's sweep.  A
    // neighbouring workgroup that reads those bytes as part of an edge chunk
    // adds and then subtracts the same value it read, so a concurrent write
    // cannot change its sums.
    // The field is addressed from the entry's own first byte (no second read of
    // the frame descriptor): L4 field at entry + (w >> 16), IPv4 header
    // checksum at entry + 10.
    __device__ __forceinline__ void put(uint32_t i, uint16_t c, uint32_t w, bool valid,
                                        uint64_t addr) const {
        const uint32_t f = i / SLOTS;
        if constexpr (MODE == FR_ECHO) {
            // the reply: ICMP type 0 (ICMP_V4_REPLY, src/icmpv4.c:45) and the
            // field, stored raw, at the message's first bytes (inside the
            // entry: a neighbouring tile reads them only in an edge chunk,
            // whose out-of-entry bytes it subtracts as loaded)
            if (!valid) return;
            uint32_t st = 0;
            if (w & 1u) {
                fr_store_echo_reply<STP>(wbase + (addr - reinterpret_cast<uint64_t>(base)), c);
                st = 2u;
            }
            if (out8) out8[f] = (uint8_t)st;
            return;
        }
        if constexpr (MODE == FR_TX_REC) {
            // the header lane (slot 2f) writes the frame's record with the L4
            // lane's result (every lane runs the shuffle)
            const uint32_t cl4 = (uint32_t)__shfl_xor((int)c, 1, 64) & 0xffffu;
            if (!valid || (i & 1u)) return;
            uint64_t r = 0;
            if (w & 1u) {
                r = (uint64_t)c | (1ull << 40);
                if (w & FR_HAS_L4)
                    r |= ((uint64_t)cl4 << 16) | ((uint64_t)((w >> 24) + ((w >> 16) & 0xffu)) << 32);
            }
            rec[f] = r;
            return;
        }
        if (MODE == FR_TX) {
            // SEC: the header lane writes a block both fields share, so it
            // takes the L4 lane's result (every lane runs the shuffle)
            const uint32_t cl4 = SEC > 0 ? ((uint32_t)__shfl_xor((int)c, 1, 64) & 0xffffu) : 0u;
            if (!valid) return;
            if ((i & 1u) == 0u && out8) out8[f] = (uint8_t)(w & 1u);
            if (!(w & 1u)) return;
            const bool l4 = (i & 1u) != 0u;
            if (l4 && !(w & FR_HAS_L4)) return;
            // raw store (no htons) of the two bytes; one u16 store when aligned
            const uint64_t fa = addr + (l4 ? ((w >> 16) & 0xffu) : 10u);
            if constexpr (SEC > 0) {
                if (w & (l4 ? FR_SEC_L4 : FR_SEC_HDR)) {
                    if (l4 && (w & FR_SEC_SHARED)) return;  // written by the header lane
                    const uint64_t sa = fa & ~(uint64_t)(SEC - 1);
                    const bool two = !l4 && (w & FR_SEC_SHARED);
                    fr_block_put<SEC>(sa, (uint32_t)(fa - sa), c, two, (uint32_t)(fa - sa) + (w >> 24), cl4);
                    return;
                }
            }
            if constexpr (STP > 0) {
                fr_store16_pol<STP>(fa, c);
                return;
            }
            uint8_t* p = wbase + (fa - reinterpret_cast<uint64_t>(base));
            if (nt_store) {
                if (fa & 1ull) {
                    __builtin_nontemporal_store((uint8_t)c, p);
                    __builtin_nontemporal_store((uint8_t)(c >> 8), p + 1);
                } else {
                    __builtin_nontemporal_store(c, reinterpret_cast<uint16_t*>(p));
                }
            } else if (fa & 1ull) {
                p[0] = (uint8_t)c;
                p[1] = (uint8_t)(c >> 8);
            } else {
                *reinterpret_cast<uint16_t*>(p) = c;
            }
            return;
        }
        // RX: slot 2f (or f) holds the header result, 2f+1 the L4 result
        const uint32_t c1 = SLOTS == 2u ? ((uint32_t)__shfl_xor((int)c, 1, 64) & 0xffffu) : 0u;
        if (!valid || (SLOTS == 2u && (i & 1u))) return;
        uint32_t v = w & 0xffu;
        if (w & FR_HAS_HDR) {  // lvlip_rx_apply
            if (c != 0u)
                v = LVLIP_RX_BAD_CSUM;
            else if ((w & FR_HAS_L4) && c1 != 0u && v == 0u)
                v = LVLIP_RX_BAD_L4;
            v = v == 0u ? (uint32_t)LVLIP_RX_OK : (v & ~FR_PENDING);
        }
        out8[f] = (uint8_t)v;
    }
};

}  // namespace lvlip
