// flat_src.h — where k_flat2 (csum_kernels.hip) takes its entries from and
// where its results go.
//
//   get(i, ctx): entry i as {offset, len, start_sum}; ctx is a word the source
//       wants back in put
//   put(i, c, ctx, valid): called by every thread of the workgroup (valid =
//       i < n), so a source may exchange results between neighbouring lanes
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
    const lvlip_csum_desc* descs;
    uint16_t* out;
    __device__ __forceinline__ lvlip_csum_desc get(uint32_t i, uint32_t& ctx) const {
        ctx = 0;
        return descs[i];
    }
    __device__ __forceinline__ void put(uint32_t i, uint16_t c, uint32_t, bool valid) const {
        if (valid) out[i] = c;
    }
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
enum { FR_TX = 0, FR_RX = 1, FR_RX_L4 = 2 };

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

// The decisions are those of skb_batch.c (host), which cites the reference line
// of each.  Entry slots: RX with L4 and TX use two per frame (lanes 2f, 2f+1 of
// one wave, so the pair exchanges results by shuffle), RX header-only one.  An
// entry the frame does not have is empty (len 0).  Frame bytes are read with
// byte loads (any alignment), never past the frame's len.
template <int MODE>
struct FrameSrc {
    const uint8_t* base;             // the frames' bytes
    uint8_t* wbase;                  // the same, writable (TX)
    const lvlip_frame_desc* frames;  // this launch's first frame
    uint8_t* out8;                   // RX: verdict[], TX: status[] (may be null)
    static constexpr uint32_t SLOTS = MODE == FR_RX ? 1u : 2u;

    // ip_rcv's decisions (src/ip_input.c:17-60) -> entries {header, L4} and the
    // plan word (verdict so far | flags)
    __device__ __forceinline__ void parse_rx(const lvlip_frame_desc& fd, const uint8_t* h,
                                             lvlip_csum_desc& d0, lvlip_csum_desc& d1,
                                             uint32_t& w) const {
        uint32_t v = 0;
        if (fd.len < FR_ETH + 20u) {
            v = LVLIP_RX_SHORT;
        } else if (fr_be16(h + 12) != 0x0800u) {  // netdev_receive, src/netdev.c:67-80
            v = LVLIP_RX_NOT_IP;
        } else {
            const uint32_t ver = h[14] >> 4, ihl = h[14] & 0x0fu;
            if (ver != 4u) {  // src/ip_input.c:22
                v = LVLIP_RX_BAD_VERSION;
            } else if (ihl < 5u) {  // src/ip_input.c:27
                v = LVLIP_RX_BAD_IHL;
            } else if (h[22] == 0u) {  // src/ip_input.c:32
                v = LVLIP_RX_TTL0;
            } else if (fd.len < FR_ETH + ihl * 4u) {
                v = LVLIP_RX_SHORT;
            } else {
                d0 = fr_mk(fd.offset + FR_ETH, ihl * 4u, 0);  // src/ip_input.c:38
                w |= FR_HAS_HDR;
                const uint32_t proto = h[23];
                if (proto != 6u && proto != 1u) {  // src/ip_input.c:51-60
                    v = FR_PENDING | LVLIP_RX_UNKNOWN_PROTO;
                } else if (MODE == FR_RX_L4) {
                    const uint32_t iplen = fr_be16(h + 16);
                    if (iplen < ihl * 4u || fd.len < FR_ETH + iplen) {
                        v = FR_PENDING | LVLIP_RX_SHORT;
                    } else {
                        const uint32_t l4len = iplen - ihl * 4u;
                        const uint32_t seed =
                            proto == 6u ? fr_pseudo_rfc(fr_le32(h + 26), fr_le32(h + 30), 6u, l4len) : 0u;
                        d1 = fr_mk(fd.offset + FR_ETH + ihl * 4u, l4len, seed);
                        w |= FR_HAS_L4;
                    }
                }
            }
        }
        w |= v;
    }

    // the TX decisions of lvlip_tx_plan -> entries {L4, header}; plan word =
    // filled | L4 flag | the L4 checksum field's offset in the frame << 16
    __device__ __forceinline__ void parse_tx(const lvlip_frame_desc& fd, const uint8_t* h,
                                             lvlip_csum_desc& d0, lvlip_csum_desc& d1,
                                             uint32_t& w) const {
        if (fd.len < FR_ETH + 20u) return;
        const uint32_t ihl = h[14] & 0x0fu, iplen = fr_be16(h + 16), proto = h[23];
        if ((h[14] >> 4) != 4u || ihl < 5u || iplen < ihl * 4u || fd.len < FR_ETH + iplen) return;
        const uint32_t l4 = FR_ETH + ihl * 4u, l4len = iplen - ihl * 4u;
        // each field's current u16 is taken out of the seed (skb_batch.c): the
        // same sum as the reference's zero-then-checksum, mod 2^32
        if (proto == 6u && l4len >= 20u) {  // src/tcp_output.c:110,126
            d0 = fr_mk(fd.offset + l4, l4len,
                       fr_pseudo_lossy(fr_le32(h + 26), fr_le32(h + 30), 6u, l4len) - fr_le16(h + l4 + 16));
            w = FR_HAS_L4 | ((l4 + 16u) << 16);
        } else if (proto == 1u && l4len >= 4u) {  // src/icmpv4.c:46-47
            d0 = fr_mk(fd.offset + l4, l4len, 0u - fr_le16(h + l4 + 2));
            w = FR_HAS_L4 | ((l4 + 2u) << 16);
        }
        d1 = fr_mk(fd.offset + FR_ETH, ihl * 4u, 0u - fr_le16(h + 24));  // src/ip_output.c:42,53
        w |= 1u;
    }

    __device__ __forceinline__ lvlip_csum_desc get(uint32_t i, uint32_t& w) const {
        const lvlip_frame_desc fd = frames[i / SLOTS];
        const uint8_t* h = base + fd.offset;
        lvlip_csum_desc d0 = fr_mk(0, 0, 0), d1 = fr_mk(0, 0, 0);
        w = 0;
        if (MODE == FR_TX)
            parse_tx(fd, h, d0, d1, w);
        else
            parse_rx(fd, h, d0, d1, w);
        return (SLOTS == 2u && (i & 1u)) ? d1 : d0;
    }

    // TX writes the two checksum fields after the workgroup's sweep.  A
    // neighbouring workgroup that reads those bytes as part of an edge chunk
    // adds and then subtracts the same value it read, so a concurrent write
    // cannot change its sums.
    __device__ __forceinline__ void put(uint32_t i, uint16_t c, uint32_t w, bool valid) const {
        const uint32_t f = i / SLOTS;
        if (MODE == FR_TX) {
            if (!valid) return;
            if ((i & 1u) == 0u && out8) out8[f] = (uint8_t)(w & 1u);
            if (!(w & 1u)) return;
            uint8_t* h = wbase + frames[f].offset;
            if ((i & 1u) == 0u) {
                if (w & FR_HAS_L4) {  // raw store (no htons), byte by byte: any alignment
                    const uint32_t fo = w >> 16;
                    h[fo] = (uint8_t)c;
                    h[fo + 1] = (uint8_t)(c >> 8);
                }
            } else {
                h[24] = (uint8_t)c;
                h[25] = (uint8_t)(c >> 8);
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
