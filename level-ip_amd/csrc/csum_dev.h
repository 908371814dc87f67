// csum_dev.h — device code shared by the product library (csum_kernels.hip)
// and the A/B lab library (lab_kernels.hip): the word-sum helpers, the ring of
// k_window (ring_sweep), the chunk sweep k_flat2 and the launch helpers.
//
// What is computed (bit-exact with src/utils.c:22-55 of level-ip):
//   W   = sum of the packet's native little-endian u16 words, mod 2^32, plus
//         the odd trailing byte as a low byte (utils.c:27-35);
//   T   = (u32)start_sum + W (mod 2^32) (utils.c:46-48; the TCP seed of
//         src/tcp.c:92-95 already carries the reference's lost carry);
//   T   = fold(fold(T)) == while (T >> 16) T = (T & 0xffff) + (T >> 16);
//   out = (u16)~T, stored raw (src/ip_output.c:11, src/tcp_output.c:126).
// Every partial sum below is a u32 add with wrap-around, so any grouping of the
// adds is exact (mod-2^32 addition is associative); end-around-carry folding is
// applied once, after the seed, exactly as the reference does.
//
// Byte alignment (the flat kernels; the ring kernels read through a per-packet
// buffer resource whose base is the packet's first byte instead, so their words
// are packet-relative, see below): the GPU reads whole 16-byte aligned chunks
// covering [offset, offset+len) and zeroes the bytes outside the packet.  When
// offset is odd, each aligned u16 holds (odd-relative byte, even-relative byte),
// so the two bytes of every half-dword are swapped before summing; the
// reference's tail byte (even relative index) then lands in the low byte as it
// should.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include <atomic>
#include <type_traits>

#include "flat_src.h"
#include "lvlip_csum.h"
#include "lvlip_skb.h"

namespace lvlip {

// ---------------------------------------------------------------- helpers --

// One u16-word sum of a dword (two words).  `odd` swaps bytes within each half
// first (packets that start at an odd address, see header comment).
template <bool ODD>
__device__ __forceinline__ uint32_t dword_words(uint32_t x) {
    if (ODD) x = ((x & 0x00ff00ffu) << 8) | ((x >> 8) & 0x00ff00ffu);
    return (x & 0xffffu) + (x >> 16);
}

template <bool ODD>
__device__ __forceinline__ uint32_t chunk_words(const uint4 v) {
    return dword_words<ODD>(v.x) + dword_words<ODD>(v.y) + dword_words<ODD>(v.z) +
           dword_words<ODD>(v.w);
}

// Mask of bytes [b0, b1) (0 <= b0, b1 <= 16 relative to the chunk) within
// dword k of the chunk.
__device__ __forceinline__ uint32_t dword_mask(int b0, int b1, int k) {
    int s = min(max(b0 - 4 * k, 0), 4);
    int e = min(max(b1 - 4 * k, 0), 4);
    uint64_t hi = (1ull << (8 * e)) - 1ull;
    uint64_t lo = (1ull << (8 * s)) - 1ull;
    return (uint32_t)(hi & ~lo);  // zero when e <= s
}

__device__ __forceinline__ uint4 mask_chunk(uint4 v, int b0, int b1) {
    v.x &= dword_mask(b0, b1, 0);
    v.y &= dword_mask(b0, b1, 1);
    v.z &= dword_mask(b0, b1, 2);
    v.w &= dword_mask(b0, b1, 3);
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// 64-lane u32 sum with DPP (no LDS traffic); the total is returned uniform
// (SGPR) from lane 63.  quad_perm(1,0,3,2), quad_perm(2,3,0,1), row_ror:4,
// row_ror:8 leave every lane holding its 16-lane row sum; row_bcast:15 (rows 1,3)
// and row_bcast:31 (rows 2,3) accumulate the four rows into lane 63.  Lanes of
// rows a row_mask leaves out keep `old` = 0, so the adds there are no-ops.
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Streaming (read-once) 16-B load: `global_load_dwordx4 ... nt`.  The batch is
// read exactly once, so keeping it out of the caches' retained set is worth
// ~+8 % read bandwidth on MI355X (scripts/lab_read.py).
__device__ __forceinline__ uint4 load_nt(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Nontemporal 16-B load from a 64-bit global address held as an integer (the
// cast to address space 1 keeps it a global_load; a generic pointer would make
// it a flat_load, which counts on lgkmcnt too and serialises the waits).
__device__ __forceinline__ uint4 load_nt_global(uint64_t a) {
    typedef __attribute__((address_space(1))) const u32x4 gvec;
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<gvec*>(a));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint4 load_global(uint64_t a) {
    typedef __attribute__((address_space(1))) const u32x4 gvec;
    const u32x4 v = *reinterpret_cast<gvec*>(a);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// utils.c:46-54.  Two unconditional folds equal the reference's while loop:
// after the first T <= 0x1fffe, after the second T <= 0xffff, and a fold of a
// value <= 0xffff is the identity.
__device__ __forceinline__ uint16_t finish(uint32_t start_sum, uint32_t w) {
    uint32_t t = start_sum + w;
    t = (t & 0xffffu) + (t >> 16);
    t = (t & 0xffffu) + (t >> 16);
    return (uint16_t)~t;
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) {
    return __builtin_amdgcn_readfirstlane(x);
}

// ------------------------------------------------------- k_wave (VGPR path) --

// Partial word sum of one packet for this lane; the wave reduces afterwards.
template <int U, bool ODD>
__device__ __forceinline__ uint32_t wave_packet_sum(const uint4* __restrict__ src,
                                                    uint32_t nch, int lo, uint32_t last_valid,
                                                    uint32_t lane) {
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64u * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * 64u + lane;
            v[u] = (c < nch) ? src[c] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * 64u + lane;
            if (c == 0u || c == nch - 1u) {  // the only chunks that can be partial
                const int b0 = (c == 0u) ? lo : 0;
                const int b1 = (c == nch - 1u) ? (int)last_valid : 16;
                v[u] = mask_chunk(v[u], b0, b1);
            }
            acc += chunk_words<ODD>(v[u]);
        }
    }
    return acc;
}

// ---------------------------------- the ring (k_stream, k_window): building blocks --
//
// One wavefront per packet, persistent.  Each wave streams through its packets
// (which ones: the deal, below) with a ring of R outstanding pieces; a piece is
// up to 2 KiB of one packet, read as two 1 KiB wave-loads (64 lanes x 16 B,
// nontemporal).  The next packet's loads are issued before the current packet
// is reduced.  The packet's last piece triggers the DPP reduction and the fold;
// results gather in lane (k - gc) of a register and leave as one store per 64
// packets.  A piece keeps all per-piece bookkeeping amortised over 2 KiB, so a
// 1500-B segment is one piece (r01 profile of a per-1KiB-slot ring: ~130 SALU
// per packet, the CU's scalar unit ~80 % busy and the kernel SALU-bound; this
// layout cuts that ~3x).
//
// Addressing: a buffer resource per packet whose base is the packet's first
// byte (any byte alignment; gfx950 buffer loads accept it) and whose
// num_records is len rounded up to 4.  gfx950 range-checks raw buffer loads per
// dword (dword k is returned iff 4k+4 <= num_records, else 0; scripts/lab_oob.py),
// so lanes past the packet read zeros with no select and no memory access, the
// u16 words are packet-relative (no odd-address byte swap), and the only fix-up
// is the 1-3 byte tail of a length that is not a multiple of 4, in one lane.
//
// Wait-count discipline (what keeps the ring in flight): ring loads are issued
// from inline asm, exactly two per piece (pieces past the range use
// num_records = 0), and retired by piece_wait<2(R-1)>; hipcc's own wait-count
// pass cannot follow a ring across the loop back edge and would drain it.
// Descriptors arrive 64 at a time in per-wave LDS windows by LDS-DMA (also asm,
// so hipcc does not drain the ring before each LDS read); a window is refilled
// 64 packets (>= 64 ring loads) before it is read, so the ring's waits retire it.

constexpr int SW_WAVES = 4;  // waves per 256-thread workgroup
constexpr uint32_t SRD_WORD3 = 0x00020000u;  // raw 32-bit buffer, as make_buffer_rsrc

// POL (A/B knob): 0 nt (default), 1 default policy, 2 nt sc1,
// 3 nt sc0 sc1, 4 sc1
template <int POL = 0>
__device__ __forceinline__ u32x4 buffer_load_nt_asm(uint32_t voff, const u32x4 srd) {
    // The resource must sit in SGPRs; it is wave-uniform by construction, which
    // readfirstlane makes explicit to the compiler (cdna_hip_programming.md T20).
    u32x4 s;
    s.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)srd.x);
    s.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)srd.y);
    s.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)srd.z);
    s.w = (uint32_t)__builtin_amdgcn_readfirstlane((int)srd.w);
    // s_nop 4: the resource words may have just been written by v_readfirstlane
    // (a VALU write of SGPRs); a VMEM read of such SGPRs needs 5 wait states on
    // gfx9-family parts, and hipcc inserts no hazard padding around inline asm.
    u32x4 r;
    if (POL == 0)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen nt"
                     : "=v"(r)
                     : "v"(voff), "s"(s));
    else if (POL == 1)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen"
                     : "=v"(r)
                     : "v"(voff), "s"(s));
    else if (POL == 2)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen nt sc1"
                     : "=v"(r)
                     : "v"(voff), "s"(s));
    else if (POL == 3)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen sc0 sc1 nt"
                     : "=v"(r)
                     : "v"(voff), "s"(s));
    else
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen sc1"
                     : "=v"(r)
                     : "v"(voff), "s"(s));
    return r;
}

// Sum of the two u16 halves of x, added to acc (v_dot2_u32_u16 with {1,1}).
__device__ __forceinline__ uint32_t dot2_acc(uint32_t x, uint32_t acc) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), one, acc, false);
}

struct PacketMeta {
    u32x4 srd;        // buffer resource: base = first byte, num_records = round_up(len, 4)
    uint32_t tinfo;   // lc << 4 | tk << 2 | (len & 3): lc = chunk holding the last byte
                      // (0 for empty packets, which still take one slot), tk = its dword
    uint32_t start;   // start_sum
};

// d = {offset_lo, offset_hi, len, start_sum} (struct lvlip_csum_desc as dwords)
__device__ __forceinline__ PacketMeta packet_meta(const uint8_t* base, const u32x4 d) {
    PacketMeta m;
    const uint64_t a = reinterpret_cast<uint64_t>(base) + (((uint64_t)d.y << 32) | d.x);
    const int32_t len = (int32_t)d.z;
    const uint32_t l = len > 0 ? (uint32_t)len : 0u;
    const uint32_t lm1 = l ? l - 1u : 0u;
    m.srd.x = (uint32_t)a;
    m.srd.y = (uint32_t)(a >> 32) & 0xffffu;  // stride 0
    m.srd.z = (l + 3u) & ~3u;                 // 0 for empty packets: all dwords zero
    m.srd.w = SRD_WORD3;
    m.tinfo = ((lm1 >> 4) << 4) | (((lm1 >> 2) & 3u) << 2) | (l & 3u);
    m.start = d.w;
    return m;
}

// Retire the two loads of a ring piece (both operands are in/out, so nothing
// that reads them can be scheduled above the wait).
template <int N>
__device__ __forceinline__ void piece_wait(u32x4& a, u32x4& b) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}

// ------------------------------------------ the ring: k_stream and k_window --
//
// One body, two deals of packets to the nw = 4 x grid waves:
//
//   k_stream (G = 0)  wave r owns the contiguous range [r p, r p + p), p = ceil(n/nw):
//                     the nw waves in flight read nw streams spread over the batch;
//   k_window (G > 0)  the packets are dealt in groups of G round robin over the
//                     grid: wave r owns groups r, r + nw, r + 2 nw, ... (group j =
//                     packets [jG, jG + G)), and its k-th packet is
//
//                       gidx(k) = ((k / G) * nw + r) * G + k % G,
//
//                     so the waves in flight read one narrow window of the batch
//                     (nw x G packets) that slides through it.  Plain streaming
//                     reads in that order run 3-6 % faster on MI355X than in nw
//                     far-apart streams (scripts/lab_window.py).
//
// Everything else is local to the wave's packet sequence k = 0 .. cnt-1: the
// descriptor windows hold the wave's packets 64k .. 64k+63 (the LDS-DMA takes a
// per-lane address, so the interleaved gather costs nothing extra), and each
// window's 64 results leave as one store with per-lane addresses (one 128-B
// store for a contiguous range).
//
// k_window's ranks are XCD-major when the grid is a multiple of 8 blocks (block
// b runs on XCD b % 8 as observed; placement is a speed matter only, every rank
// is owned by exactly one wave whatever the placement): neighbouring groups then
// belong to waves of one XCD, so the partial 32-B sectors of their 2-B results
// merge in that XCD's L2 before they are written back.
template <int G, int WPB = SW_WAVES>  // WPB: waves per workgroup
struct Deal {
    uint64_t nw, rank, p_lo;
    uint32_t cnt;  // the wave's packets

    // false when this wave has no packet
    __device__ __forceinline__ bool init(uint32_t n, uint32_t wid) {
        nw = (uint64_t)gridDim.x * WPB;
        if (G == 0) {
            rank = (uint64_t)blockIdx.x * WPB + wid;
            const uint64_t per = ((uint64_t)n + nw - 1) / nw;
            p_lo = rank * per;
            if (p_lo >= n) return false;
            cnt = (uint32_t)min<uint64_t>(per, (uint64_t)n - p_lo);
            return true;
        }
        rank = (gridDim.x & 7u) == 0u
                   ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * WPB + wid
                   : (uint64_t)blockIdx.x * WPB + wid;
        p_lo = 0;
        // gcount groups, the last one short when it is the batch's last
        const uint64_t ng = ((uint64_t)n + G - 1) / G;
        if (rank >= ng) return false;
        const uint64_t gcount = (ng - 1 - rank) / nw + 1;
        const uint64_t glast = rank + (gcount - 1) * nw;
        const uint64_t last_size = min<uint64_t>((uint64_t)(G > 0 ? G : 1), (uint64_t)n - glast * G);
        cnt = (uint32_t)((gcount - 1) * G + last_size);
        return true;
    }
    __device__ __forceinline__ uint64_t gidx(uint32_t k) const {
        if (G == 0) return p_lo + k;
        return ((uint64_t)(k / (G > 0 ? G : 1)) * nw + rank) * G + (k % (G > 0 ? G : 1));
    }
};

// Descriptors of the wave's packets [first, first + 64) into an LDS window by
// LDS-DMA, one per lane; issued from asm so hipcc does not see it in flight.
template <int G, int WPB>
__device__ __forceinline__ void fetch_window(const lvlip_csum_desc* __restrict__ descs,
                                             const Deal<G, WPB>& dl, uint32_t first, uint32_t lane,
                                             uint4* win /* LDS, 64 entries */) {
    uint32_t k = first + lane;
    k = k < dl.cnt ? k : dl.cnt - 1u;  // lanes past the wave's packets re-read a valid descriptor
    const lvlip_csum_desc* g = descs + dl.gidx(k);
    const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)win);
    // m0 is reserved to the compiler, which warns on the clobber; nothing else in
    // these kernels reads m0 (tests/test_isa.py checks every m0 write is ours).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    // s_nop 4: `lds` comes from v_readfirstlane (VALU->SGPR->use hazard) and an
    // M0 write needs a wait state before an LDS-DMA reads it.
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(g), "s"(lds)
                 : "memory", "m0");
#pragma clang diagnostic pop
}

template <int R, int G, int POL, int WPB = SW_WAVES>
__device__ __forceinline__ void ring_sweep(const uint8_t* __restrict__ base,
                                           const lvlip_csum_desc* __restrict__ descs, uint32_t n,
                                           uint16_t* __restrict__ out, uint4 (*s_win)[64]) {
    constexpr uint32_t END = 0xffffffffu;
    constexpr uint32_t PIECE = 2048u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lane16 = lane * 16u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    Deal<G, WPB> dl;
    if (!dl.init(n, wid)) return;
    const uint32_t cnt = dl.cnt;

    // descriptor windows: the wave's packets [64w, 64w + 64) live in s_win[w & 1]
    fetch_window<G, WPB>(descs, dl, 0u, lane, s_win[0]);
    fetch_window<G, WPB>(descs, dl, 64u, lane, s_win[1]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // Packet metadata for the issue cursor's window, one packet per lane (VALU,
    // 64 packets at a time); the issue side pulls its packet's fields with
    // v_readlane.  (Computing them per packet on the scalar unit made the
    // kernel SALU-bound: r01 profile.)
    uint32_t m_x, m_y, m_z, m_t, m_s;  // srd.x, srd.y, srd.z, tinfo, start of packet (window + lane)
    auto load_window_meta = [&](uint32_t w) {
        const uint4 d = s_win[w & 1u][lane];
        const PacketMeta pm = packet_meta(base, u32x4{d.x, d.y, d.z, d.w});
        m_x = pm.srd.x;
        m_y = pm.srd.y;
        m_z = pm.srd.z;
        m_t = pm.tinfo;
        m_s = pm.start;
    };
    load_window_meta(0);

    uint32_t ip = 0, io = 0;  // issue cursor: the wave's packet ip, byte offset io in it
    u32x4 srd;
    uint32_t tinfo, start;
    auto pull = [&](uint32_t k) {  // k = packet index within its window
        srd.x = (uint32_t)__builtin_amdgcn_readlane((int)m_x, (int)k);
        srd.y = (uint32_t)__builtin_amdgcn_readlane((int)m_y, (int)k);
        srd.z = (uint32_t)__builtin_amdgcn_readlane((int)m_z, (int)k);
        srd.w = SRD_WORD3;
        tinfo = (uint32_t)__builtin_amdgcn_readlane((int)m_t, (int)k);
        start = (uint32_t)__builtin_amdgcn_readlane((int)m_s, (int)k);
    };
    pull(0);

    uint32_t gc = 0;  // consume side: results of the wave's packets [gc, gc+64) gather in lanes
    uint32_t res_w = 0, res_s = 0;
    uint32_t acc = 0;
    u32x4 va[R], vb[R];
    // per piece: the wave's packet index (END past its packets), start_sum, and
    // meta = last | (len & 3) << 1 | (byte offset of the last dword in the piece) << 3
    uint32_t s_pkt[R], s_start[R], s_meta[R];

    auto issue = [&](int r) {
        const bool live = ip < cnt;  // uniform
        u32x4 sr = srd;
        if (!live) sr.z = 0;  // past the range: every dword out of range -> zeros
        const uint32_t off = lane16 + io;
        va[r] = buffer_load_nt_asm<POL>(off, sr);
        vb[r] = buffer_load_nt_asm<POL>(off + 1024u, sr);
        // srd.z = round_up(len, 4): the piece is the packet's last when it reaches
        // that (or the packet is empty)
        const bool last = io + PIECE >= srd.z;
        s_pkt[r] = live ? ip : END;
        s_start[r] = start;
        s_meta[r] = (uint32_t)last | ((tinfo & 3u) << 1) | (((srd.z - 4u) - io) << 3);
        if (live) {
            if (!last) {
                io += PIECE;
            } else {
                ++ip;
                io = 0;
                if (ip < cnt) {
                    if ((ip & 63u) == 0u) {  // entered window ip/64
                        load_window_meta(ip >> 6);
                        fetch_window<G, WPB>(descs, dl, ip + 64u, lane, s_win[((ip >> 6) + 1u) & 1u]);
                    }
                    pull(ip & 63u);
                }
            }
        }
    };

    auto consume = [&](int r) {
        // Piece r's two loads are the oldest in flight: 2*(R-1) ring loads (and
        // possibly result stores / window DMAs, which only make this stricter)
        // were issued after them.
        piece_wait<2 * (R - 1)>(va[r], vb[r]);
        u32x4 x = va[r], y = vb[r];
        const uint32_t meta = s_meta[r];
        const uint32_t len3 = (meta >> 1) & 3u;
        if ((meta & 1u) && len3) {  // uniform: keep bytes [0, len & 3) of the last dword
            const uint32_t pos = meta >> 3;  // byte offset of that dword in the piece
            const uint32_t m = (1u << (8u * len3)) - 1u;
            const bool me = lane == ((pos >> 4) & 63u);
            const uint32_t tk = (pos >> 2) & 3u;
            const bool in_b = pos >= 1024u;
            const uint32_t m0 = (me && tk == 0u) ? m : ~0u, m1 = (me && tk == 1u) ? m : ~0u;
            const uint32_t m2 = (me && tk == 2u) ? m : ~0u, m3 = (me && tk == 3u) ? m : ~0u;
            if (in_b) {
                y.x &= m0; y.y &= m1; y.z &= m2; y.w &= m3;
            } else {
                x.x &= m0; x.y &= m1; x.z &= m2; x.w &= m3;
            }
        }
        acc = dot2_acc(x.x, acc);
        acc = dot2_acc(x.y, acc);
        acc = dot2_acc(x.z, acc);
        acc = dot2_acc(x.w, acc);
        acc = dot2_acc(y.x, acc);
        acc = dot2_acc(y.y, acc);
        acc = dot2_acc(y.z, acc);
        acc = dot2_acc(y.w, acc);
        if (meta & 1u) {
            const uint32_t w = wave_sum_dpp(acc);
            acc = 0;
            const uint32_t k = s_pkt[r] - gc;
            if (lane == k) {
                res_w = w;
                res_s = s_start[r];
            }
            if (k == 63u || s_pkt[r] + 1u == cnt) {
                // fold 64 results at once (src/utils.c:46-54, per lane)
                uint32_t tt = res_s + res_w;
                tt = (tt & 0xffffu) + (tt >> 16);
                tt = (tt & 0xffffu) + (tt >> 16);
                if (lane <= k) out[dl.gidx(gc + lane)] = (uint16_t)~tt;
                gc += 64u;
            }
        }
    };

#pragma unroll
    for (int r = 0; r < R; ++r) issue(r);
    bool done = false;
    while (!done) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (s_pkt[r] == END) {
                done = true;
                break;
            }
            consume(r);
            issue(r);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of this wave left in flight
}

// ------------------------------------------------- k_flat2 (ragged batches) --
//
// Chunk-balanced tile sweep, for batches of many small or mixed-size packets
// (20-B IPv4 headers next to 64-1460-B payloads, configs[3]).  A 256-thread
// workgroup owns 256 descriptors.  Phase 1 lays their 16-B aligned chunks end to
// end in a virtual chunk space (exclusive prefix of chunk counts) and marks each
// packet's first chunk in a head bitmap, kept per 64-chunk group with the
// number of heads before the group.  Phase 2 sweeps the chunk space, one group
// of 64 chunks per wave-load, U groups in flight per wave:
//   rank   = heads before the group + heads at or below this lane - 1
//            (no search: the packet of every lane in two mbcnt instructions),
//   bytes  = whole 16-B aligned chunks from the packet's own address
//            (coalesced across packet boundaries), odd-address packets
//            byte-swapped within u16 halves (v_perm); no per-lane masking:
//            a packet's first and last chunk, when they hold bytes outside
//            it, are also stashed raw in LDS, and phase 4 subtracts those
//            bytes once per packet (mod 2^32) — every byte is read from HBM
//            once, by the sweep,
//   reduce = inclusive DPP prefix sum P over the wave; a packet's first-chunk
//            lane adds val - P and its last-chunk lane (or lane 63) adds P to
//            the packet's u32 accumulator in LDS (mod-2^32 adds: exact in any
//            order), which leaves each segment's sum there.
// Packets longer than FCAP chunks go to a whole-wave loop instead.
constexpr int FT = 256;                  // descriptors per tile = threads
constexpr uint32_t FCAP = 128;           // chunks of the largest swept packet (2 KiB)

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_row_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// inclusive prefix sum over the 64 lanes (u32, wrap-around)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += dpp_row_shr<0x111>(v);  // row_shr:1
    v += dpp_row_shr<0x112>(v);  // row_shr:2
    v += dpp_row_shr<0x114>(v);  // row_shr:4
    v += dpp_row_shr<0x118>(v);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// A ring's 16-B group load, `global_load_dwordx4 ... nt` from asm (k_flat2's
// pipelined sweep, lab k_rflat): the compiler's wait-count pass does not see
// it, so the ring's own counted waits retire it.
__device__ __forceinline__ u32x4 group_load_nt(uint64_t a) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(a) : "memory");
    return r;
}

template <int N>
__device__ __forceinline__ void group_wait(u32x4& a) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
}

// two exclusive prefixes over the 256 threads for one barrier pair; *ta, *tb
// get the totals
__device__ __forceinline__ void block_excl_scan2(uint32_t a, uint32_t b, uint32_t* s_tmp /* >= 8 */,
                                                 uint32_t* ea, uint32_t* eb, uint32_t* ta,
                                                 uint32_t* tb) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
    if (lane == 63u) {
        s_tmp[wid] = ia;
        s_tmp[4u + wid] = ib;
    }
    __syncthreads();
    uint32_t ba = 0, bb = 0, aa = 0, ab = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t x = s_tmp[k], y = s_tmp[4u + k];
        ba += (k < wid) ? x : 0u;
        bb += (k < wid) ? y : 0u;
        aa += x;
        ab += y;
    }
    __syncthreads();
    *ea = ba + ia - a;
    *eb = bb + ib - b;
    *ta = aa;
    *tb = ab;
}

// Orders this wave's LDS traffic across lanes (a lane reading what another
// lane wrote): LDS ops of one wave execute in order, so the compiler only has
// to be kept from moving them, and the counter drained.  No vmcnt: global
// loads in flight stay in flight.
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// byte mask of bytes [b0, b1) of a 16-B chunk that fall in dword j
__device__ __forceinline__ uint32_t byte_range_mask(int b0, int b1, int j) {
    const int s = min(max(b0 - 4 * j, 0), 4);
    const int e = min(max(b1 - 4 * j, 0), 4);
    const int w = (e - s) * 8;
    if (w <= 0) return 0u;
    if (w >= 32) return 0xffffffffu;
    return ((1u << w) - 1u) << (8 * s);
}

// D descriptors per thread (a tile of FT * D): D = 2 halves the per-tile
// plan's share of the launch (A/B, batch calls only; unroll bit 10).  Thread t
// owns the tile's descriptors t*D .. t*D + D - 1, so its ranks, chunk starts
// and big-packet slots follow from one exclusive scan of its D counts.
// FIN_LDS (A/B, lab): phase 4's per-descriptor words go through LDS instead of
// staying in registers across the sweep (fewer VGPRs live in phase 2).
// PFA (the product's batch calls use kFlatPrefetchTiles; frame sources A/B): each
// thread also loads the descriptor PFA tiles ahead of its own, issued after
// its own (loads return in order, so its own descriptor's wait does not cover
// it).  Block b runs on XCD b % 8 (as observed), so with PFA a multiple of 8
// the workgroup that runs that tile later finds its descriptors in its own
// XCD's L2: phase 1's first round trip becomes an L2 hit, and HBM traffic is
// unchanged (PMC: FETCH_SIZE and L2 misses equal, L2 hits + the prefetch).
// VAR (A/B bits, lab id 13): bit 0 raises the instruction-issue priority
// (s_setprio 2) for the load-issuing part of each sweep round, bit 1 for phase
// 1; bit 2 (block order) spreads a tile's last, partial round over the four
// waves instead of leaving it to the first ones; bit 3 waits for every load
// of a round (no early exit at the first group past the wave's); bit 5 is an
// ablation (wrong results): the sweep's loads with one xor per dword instead
// of the reduction.
template <int U, bool NT, int GORD, class Src, int D = 1, bool PIPE = false, bool FIN_LDS = false,
          int PFA = 0, int VAR = 0>
__device__ __forceinline__ void flat2_body(const uint8_t* __restrict__ base, const Src src, uint32_t n) {
    static_assert(D == 1 || D == 2, "descriptors per thread");
    static_assert(!PIPE || (NT && U <= 8), "the pipelined sweep: nontemporal, at most 8 loads per round");
    constexpr uint32_t TD = (uint32_t)FT * D;   // descriptors per tile
    constexpr uint32_t FG = TD * FCAP / 64;     // most 64-chunk groups a tile can have
    __shared__ uint4 s_rec[TD];        // by rank: {a0 lo, a0 hi, cstart, meta}
    __shared__ uint2 s_grp[FG];        // by 64-chunk group: head bitmap {lo, hi}
    __shared__ uint16_t s_hb[FG];      // by 64-chunk group: heads before it (<= TD)
    __shared__ uint32_t s_acc[TD];     // by descriptor
    __shared__ uint32_t s_big[TD];     // descriptors longer than FCAP chunks
    __shared__ uint4 s_edge[2 * TD];   // by descriptor: raw first / last chunk
    __shared__ uint32_t s_tmp[8];
    __shared__ uint2 s_fin[FIN_LDS ? TD : 1];  // by descriptor: {start_sum, phase-4 word}

    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t tile0 = blockIdx.x * TD;
    const uint32_t t = tid;

    // ---- phase 1: descriptors -> chunk counts, ranks, records, head bitmap
    if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(2);
    uint4 pf = make_uint4(0u, 0u, 0u, 0u);  // PFA's prefetch, consumed at the end
    uint32_t start_sum[D], nch[D], meta[D], lo[D], lastv[D], ctx[D];
    uint64_t a0[D];  // the swept part's first chunk; its first byte is a0 + lo
    uint64_t ent[D];  // the entry's first byte (the frame calls' put)
    bool big[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t j = t * D + d, i = tile0 + j;
        start_sum[d] = 0, nch[d] = 0, meta[d] = 0, lo[d] = 0, lastv[d] = 16, ctx[d] = 0;
        a0[d] = 0;
        ent[d] = 0;
        big[d] = false;
        uint32_t wsum = 0;  // the entry's bytes inside the parse window (frame calls)
        if (i < n) {
            uint4 win[4];
            uint64_t wa = 0;
            lvlip_csum_desc ds;
            if constexpr (Src::WIN_SUM)
                ds = src.get(i, ctx[d], win, &wa);
            else
                ds = src.get(i, ctx[d]);
            if constexpr (PFA > 0) {
                if (d == 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    const uint64_t ip = (uint64_t)i + (uint64_t)PFA * TD;
                    pf = load_global(reinterpret_cast<uint64_t>(src.desc_ptr(ip < n ? (uint32_t)ip : i)));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            start_sum[d] = ds.start_sum;
            if (ds.len > 0) {
                uint64_t abs = reinterpret_cast<uint64_t>(base) + ds.offset;
                const uint64_t eend = abs + (uint32_t)ds.len;
                ent[d] = abs;
                const bool odd = abs & 1ull;
                big[d] = (((abs & 15ull) + (uint32_t)ds.len + 15u) >> 4) > FCAP;
                if constexpr (Src::WIN_SUM) {
                    // Frame calls: the parse already holds the frame's chunks
                    // [wa, wa + 64) in registers.  Sum the entry's bytes there
                    // (same masking and parity as the sweep plus the edge
                    // corrections) and sweep only the rest, from wa + 64: the
                    // header entry then needs no sweep at all, and no frame
                    // byte is read from HBM twice.  Big entries keep the
                    // whole-wave loop over all their bytes.
                    const uint64_t we = wa + 64u;
                    if (!big[d] && abs >= wa && abs < we) {
                        const uint64_t pe = eend < we ? eend : we;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint64_t ck = wa + 16u * k;
                            const int b0 = abs > ck ? (int)(abs - ck < 16u ? abs - ck : 16u) : 0;
                            const int b1 = pe > ck ? (int)(pe - ck < 16u ? pe - ck : 16u) : 0;
                            const uint4 v = mask_chunk(win[k], b0, b1);
                            wsum += odd ? chunk_words<true>(v) : chunk_words<false>(v);
                        }
                        abs = pe;
                    }
                }
                if (abs < eend) {
                    a0[d] = abs & ~15ull;
                    lo[d] = (uint32_t)(abs & 15ull);
                    const uint64_t span = (uint64_t)lo[d] + (eend - abs);
                    const uint64_t c64 = (span + 15u) >> 4;
                    lastv[d] = (uint32_t)(span - 16ull * (c64 - 1u));
                    nch[d] = big[d] ? 0u : (uint32_t)c64;
                    // edge flags: the sweep stashes the packet's first (bit 10)
                    // and last (bit 11) chunk in LDS when they hold bytes
                    // outside it
                    const bool ef = !big[d] && (lo[d] != 0u || (c64 == 1u && lastv[d] != 16u));
                    const bool el = !big[d] && c64 > 1u && lastv[d] != 16u;
                    meta[d] = nch[d] | ((uint32_t)odd << 9) | ((uint32_t)ef << 10) |
                              ((uint32_t)el << 11) | (j << 18);
                }
            }
        }
        s_acc[j] = wsum;
        if constexpr (FIN_LDS)
            s_fin[j] = make_uint2(start_sum[d], nch[d] | (meta[d] & (7u << 9)) | (lo[d] << 12) | (lastv[d] << 16));
    }
    for (uint32_t g = t; g < FG; g += FT) s_grp[g] = make_uint2(0u, 0u);
    // one scan pass for three prefixes: big packets (high half) and swept
    // packets (low half, both <= TD) packed in one word, chunks in the other
    uint32_t sa = 0, sb = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        sa += (big[d] ? 0x10000u : 0u) | (nch[d] ? 1u : 0u);
        sb += nch[d];
    }
    uint32_t e1 = 0, cs = 0, t1 = 0, C = 0;
    block_excl_scan2(sa, sb, s_tmp, &e1, &cs, &t1, &C);
    const uint32_t nbig = t1 >> 16;
    const uint32_t G = (C + 63u) >> 6;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t j = t * D + d;
        const uint32_t big_pos = e1 >> 16, rank = e1 & 0xffffu, cstart = cs;
        if (big[d]) s_big[big_pos] = j;
        if (nch[d]) {
            s_rec[rank] = make_uint4((uint32_t)a0[d], (uint32_t)(a0[d] >> 32), cstart, meta[d]);
            const uint32_t g = cstart >> 6, b = cstart & 63u;
            if (b < 32u) atomicOr(&s_grp[g].x, 1u << b);
            else atomicOr(&s_grp[g].y, 1u << (b - 32u));
            // heads before group g = swept packets that start before chunk 64 g.
            // The packets' chunk ranges tile [0, C) in rank order, so for every
            // group that starts inside (cstart, cstart + nch] that count is this
            // packet's rank + 1 (at most 3 groups: nch <= FCAP = 128)
            for (uint32_t gg = g + 1u; gg < G && (gg << 6) <= cstart + nch[d]; ++gg)
                s_hb[gg] = (uint16_t)(rank + 1u);
        }
        // the next descriptor of this thread follows in rank and chunk order
        e1 += (big[d] ? 0x10000u : 0u) | (nch[d] ? 1u : 0u);
        cs += nch[d];
    }
    if (t == 0u) s_hb[0] = 0;
    __syncthreads();
    if constexpr ((VAR & 2) != 0) __builtin_amdgcn_s_setprio(0);

    // ---- phase 2: sweep the chunk space, groups wid, wid+4, ... ; U per round.
    // Every round issues exactly U loads, unconditionally (lanes past the chunk
    // space read a valid chunk of the tile's last packet and are zeroed), after
    // all U group headers and all U records are in registers: hipcc then retires
    // them with counted vmcnt waits instead of draining.
    //
    // Segment sums without locating heads: with P the inclusive prefix over the
    // wave, a packet's segment in a group is P(last lane) - (P(first lane) -
    // val(first lane)).  So the lane holding the packet's first chunk adds
    // val - P, the lane holding its last chunk (or lane 63) adds P, and a
    // segment that starts at lane 0 as a continuation needs nothing (exclusive
    // prefix 0).  One LDS atomic per group carries both.
    //
    // Group order (GORD).  2 (default) = blocks: a round of the workgroup is 4U
    // consecutive groups, U per wave, so the tile is read as one stream and
    // only every U-th group boundary (a 128-B line two groups can share) falls
    // between two waves, which request it at about the same time.  1 = quarters:
    // wave w takes groups [w*G/4, (w+1)*G/4), four streams per tile.  0 =
    // interleaved, groups w, w+4, ...: every shared line is requested by two
    // waves at different times (PMC: 4.4 % re-fetched lines).  Blocks against
    // quarters on mixed: +0.5-1.6 % (U 8 / U 4) and 0.9 % less HBM traffic.
    const uint32_t gstep = GORD == 0 ? 4u : 1u;             // between a round's groups
    const uint32_t rstep = GORD == 1 ? (uint32_t)U : 4u * U;  // between rounds
    const uint32_t gper = (G + 3u) / 4u;
    const uint32_t g_lo = GORD == 1 ? wid * gper : (GORD == 2 ? wid * (uint32_t)U : wid);
    const uint32_t g_end = GORD == 1 ? (g_lo + gper < G ? g_lo + gper : G) : G;
    if (PIPE && C > 0) {
        // Pipelined sweep (A/B, lab): two rounds' loads (two register banks)
        // are issued before the first is reduced, so the second round's loads
        // are in flight during the first's reduction instead of being issued
        // after it.  The loads are asm (group_load_nt) and retired by counted
        // waits: a load of the first bank has its bank's later loads and the
        // second bank's U behind it, a load of the second only its own bank's
        // (a round past the wave's groups is a placeholder round of valid
        // loads, so the counts hold).
        u32x4 xa[U], xb[U];
        uint32_t mta[U], mtb[U], kka[U], kkb[U];
        bool vla[U], vlb[U], gva[U], gvb[U];
        auto prep = [&](uint32_t gr, u32x4* x, uint32_t* mt, uint32_t* kk, bool* vl, bool* gv) {
            uint32_t hlo[U], hhi[U], hb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t g = gr + gstep * u;
                gv[u] = g < g_end;
                const uint32_t gc = gv[u] ? g : G - 1u;
                const uint2 gg = s_grp[gc];
                hlo[u] = uniform(gg.x);
                hhi[u] = uniform(gg.y);
                hb[u] = uniform((uint32_t)s_hb[gc]);
            }
            uint4 rec[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t H = ((uint64_t)hhi[u] << 32) | hlo[u];
                const uint64_t Hs = H >> 1;
                const uint32_t cnt = __builtin_amdgcn_mbcnt_hi((uint32_t)(Hs >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)Hs, 0u));
                rec[u] = s_rec[(hb[u] + (uint32_t)(H & 1ull) - 1u) + cnt];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = (gr + gstep * u) * 64u + lane;
                vl[u] = gv[u] && j < C;
                kk[u] = vl[u] ? j - rec[u].z : 0u;
                x[u] = group_load_nt((((uint64_t)rec[u].y << 32) | rec[u].x) + 16ull * kk[u]);
                mt[u] = rec[u].w;
            }
        };
        auto reduce = [&](auto depth, u32x4* x, const uint32_t* mt, const uint32_t* kk, const bool* vl,
                          const bool* gv) {
            constexpr int B = decltype(depth)::value;  // loads issued after a bank's first
#pragma unroll
            for (int u = 0; u < U; ++u) {
                switch (u) {
                    case 0: group_wait<(B > 1 ? B - 1 : 0)>(x[u]); break;
                    case 1: group_wait<(B > 2 ? B - 2 : 0)>(x[u]); break;
                    case 2: group_wait<(B > 3 ? B - 3 : 0)>(x[u]); break;
                    case 3: group_wait<(B > 4 ? B - 4 : 0)>(x[u]); break;
                    case 4: group_wait<(B > 5 ? B - 5 : 0)>(x[u]); break;
                    case 5: group_wait<(B > 6 ? B - 6 : 0)>(x[u]); break;
                    case 6: group_wait<(B > 7 ? B - 7 : 0)>(x[u]); break;
                    default: group_wait<(B > 8 ? B - 8 : 0)>(x[u]); break;
                }
                if (!gv[u]) continue;  // uniform: past the wave's groups (waited all the same)
                const u32x4 raw = x[u];
                uint4 v = make_uint4(raw.x, raw.y, raw.z, raw.w);
                const uint32_t m = mt[u];
                if (__builtin_amdgcn_ballot_w64((m & (1u << 9)) != 0u)) {
                    const uint32_t sel = (m & (1u << 9)) ? 0x02030001u : 0x03020100u;
                    v.x = __builtin_amdgcn_perm(v.x, v.x, sel);
                    v.y = __builtin_amdgcn_perm(v.y, v.y, sel);
                    v.z = __builtin_amdgcn_perm(v.z, v.z, sel);
                    v.w = __builtin_amdgcn_perm(v.w, v.w, sel);
                }
                uint32_t val = 0;
                val = dot2_acc(v.x, val);
                val = dot2_acc(v.y, val);
                val = dot2_acc(v.z, val);
                val = dot2_acc(v.w, val);
                val = vl[u] ? val : 0u;
                const uint32_t P = wave_incl_scan(val);
                const bool first = kk[u] == 0u;
                const bool last = kk[u] + 1u == (m & 0xFFu);
                const uint32_t add = (first ? val - P : 0u) + ((last || lane == 63u) ? P : 0u);
                if (vl[u] && (first || last || lane == 63u)) atomicAdd(&s_acc[m >> 18], add);
                if (vl[u] && first && (m & (1u << 10)))
                    s_edge[2u * (m >> 18)] = make_uint4(raw.x, raw.y, raw.z, raw.w);
                if (vl[u] && last && (m & (1u << 11)))
                    s_edge[2u * (m >> 18) + 1u] = make_uint4(raw.x, raw.y, raw.z, raw.w);
            }
        };
        // Rounds in pairs: the second round's loads are in flight while the
        // first is reduced, and nothing is in flight across the loop's back
        // edge.  (A version that carried a bank in flight across the back edge
        // let the register allocator copy a bank's registers at the loop head
        // before their loads had landed: wrong sums, caught by the parity tests
        // and by tests/test_isa.py's in-flight register check.)
        using Two = std::integral_constant<int, 2 * U>;
        using One = std::integral_constant<int, U>;
        for (uint32_t gr = g_lo; gr < g_end; gr += 2u * rstep) {
            prep(gr, xa, mta, kka, vla, gva);
            prep(gr + rstep, xb, mtb, kkb, vlb, gvb);  // placeholders past g_end
            reduce(Two{}, xa, mta, kka, vla, gva);
            reduce(One{}, xb, mtb, kkb, vlb, gvb);
        }
    } else if (C > 0) {
        uint32_t abl = 0;  // VAR bit 5's ablation
        constexpr bool TAILB = (VAR & 4) != 0 && GORD == 2;
        // TAILB: rr walks the workgroup's rounds; the last, partial one is
        // dealt to the four waves in equal parts
        for (uint32_t rr = TAILB ? 0u : g_lo; rr < g_end; rr += rstep) {
            uint32_t gr = rr, ge = g_end;
            if constexpr (TAILB) {
                gr = rr + wid * (uint32_t)U;
                if (rr + rstep > G) {
                    const uint32_t R = G - rr;
                    gr = rr + (R * wid) / 4u;
                    ge = rr + (R * (wid + 1u)) / 4u;
                }
            }
            if constexpr ((VAR & 1) != 0) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(2);
                __builtin_amdgcn_sched_barrier(0);
            }
            uint4 x[U];
            uint32_t mt[U], kk[U];
            bool vl[U];
            uint32_t hlo[U], hhi[U], hb[U];
            bool gv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t g = gr + gstep * u;
                gv[u] = g < ge;
                const uint32_t gc = gv[u] ? g : G - 1u;
                const uint2 gg = s_grp[gc];
                hlo[u] = uniform(gg.x);
                hhi[u] = uniform(gg.y);
                hb[u] = uniform((uint32_t)s_hb[gc]);
            }
            uint32_t r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // heads at or below this lane = bit 0 + heads of bits 1..lane
                // = bit 0 + mbcnt(H >> 1); the scalar part folds into one add
                const uint64_t H = ((uint64_t)hhi[u] << 32) | hlo[u];
                const uint64_t Hs = H >> 1;
                const uint32_t cnt = __builtin_amdgcn_mbcnt_hi((uint32_t)(Hs >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)Hs, 0u));
                r[u] = (hb[u] + (uint32_t)(H & 1ull) - 1u) + cnt;  // always a valid rank
            }
            uint4 rec[U];
#pragma unroll
            for (int u = 0; u < U; ++u) rec[u] = s_rec[r[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = (gr + gstep * u) * 64u + lane;
                vl[u] = gv[u] && j < C;
                kk[u] = vl[u] ? j - rec[u].z : 0u;
                const uint64_t ca = (((uint64_t)rec[u].y << 32) | rec[u].x) + 16ull * kk[u];
                x[u] = NT ? load_nt_global(ca) : load_global(ca);
                mt[u] = rec[u].w;
            }
            if constexpr ((VAR & 1) != 0) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr ((VAR & 32) != 0) {
                    // ablation (A/B only, wrong results): the loads, every one
                    // used unconditionally, without the reduction
                    abl ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
                    continue;
                }
                // uniform.  VAR bit 3: no early exit, so no load of this round
                // is left in flight into the next round's loop head (whose
                // conservative wait would then also cover PFA's prefetch)
                if (!gv[u]) {
                    if constexpr ((VAR & 8) != 0) {
                        asm volatile("" ::"v"(x[u].x));  // retire it here (vmcnt)
                        continue;
                    } else {
                        break;
                    }
                }
                uint4 v = x[u];
                const uint32_t m = mt[u];
                if (__builtin_amdgcn_ballot_w64((m & (1u << 9)) != 0u)) {
                    const uint32_t sel = (m & (1u << 9)) ? 0x02030001u : 0x03020100u;
                    v.x = __builtin_amdgcn_perm(v.x, v.x, sel);
                    v.y = __builtin_amdgcn_perm(v.y, v.y, sel);
                    v.z = __builtin_amdgcn_perm(v.z, v.z, sel);
                    v.w = __builtin_amdgcn_perm(v.w, v.w, sel);
                }
                uint32_t val = 0;
                val = dot2_acc(v.x, val);
                val = dot2_acc(v.y, val);
                val = dot2_acc(v.z, val);
                val = dot2_acc(v.w, val);
                val = vl[u] ? val : 0u;
                const uint32_t P = wave_incl_scan(val);
                const bool first = kk[u] == 0u;
                const bool last = kk[u] + 1u == (m & 0xFFu);
                const uint32_t add = (first ? val - P : 0u) + ((last || lane == 63u) ? P : 0u);
                if (vl[u] && (first || last || lane == 63u)) atomicAdd(&s_acc[m >> 18], add);
                // edge chunks, raw, for the corrections of phase 4 (no second read)
                if (vl[u] && first && (m & (1u << 10))) s_edge[2u * (m >> 18)] = x[u];
                if (vl[u] && last && (m & (1u << 11))) s_edge[2u * (m >> 18) + 1u] = x[u];
            }
        }
        if constexpr ((VAR & 32) != 0) atomicAdd(&s_acc[t], abl);
    }

    // ---- phase 3: packets longer than FCAP chunks, one wave each
    for (uint32_t q = wid; q < nbig; q += 4u) {
        const uint32_t tq = s_big[q];
        uint32_t cq;
        const lvlip_csum_desc d = src.get(tile0 + tq, cq);
        const uint64_t abs = reinterpret_cast<uint64_t>(base) + d.offset;
        const int lo = (int)(abs & 15ull);
        const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
        const uint32_t nchq = (uint32_t)((span + 15u) >> 4);
        const uint32_t lastv = (uint32_t)(span - 16ull * (nchq - 1u));
        const uint4* src = reinterpret_cast<const uint4*>(abs & ~15ull);
        uint32_t w = (abs & 1ull) ? wave_packet_sum<4, true>(src, nchq, lo, lastv, lane)
                                  : wave_packet_sum<4, false>(src, nchq, lo, lastv, lane);
        w = wave_sum_dpp(w);
        if (lane == 0) s_acc[tq] = w;
    }
    __syncthreads();

    // ---- phase 4: edge corrections, fold and store (coalesced 2-B stores).
    // The sweep summed whole 16-B chunks; subtract, once per packet, the bytes
    // of its first and last chunk that lie outside it (same parity convention,
    // mod 2^32 — exact).
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t j = t * D + d, i = tile0 + j;
        uint16_t res = 0;
        if constexpr (FIN_LDS) {
            const uint2 f = s_fin[j];
            start_sum[d] = f.x;
            nch[d] = f.y & 0xFFu;
            meta[d] = f.y & 0xFFFu;
            lo[d] = (f.y >> 12) & 15u;
            lastv[d] = f.y >> 16;
        }
        if (i < n) {
            uint32_t acc = s_acc[j];
            if (meta[d] & (3u << 10)) {
                const bool odd = meta[d] & (1u << 9);
                uint32_t c = 0;
                if (meta[d] & (1u << 10)) {
                    uint4 f = s_edge[2u * j];
                    const int fb1 = (nch[d] == 1u) ? (int)lastv[d] : 16;
                    f.x &= ~byte_range_mask((int)lo[d], fb1, 0);
                    f.y &= ~byte_range_mask((int)lo[d], fb1, 1);
                    f.z &= ~byte_range_mask((int)lo[d], fb1, 2);
                    f.w &= ~byte_range_mask((int)lo[d], fb1, 3);
                    c += odd ? chunk_words<true>(f) : chunk_words<false>(f);
                }
                if (meta[d] & (1u << 11)) {
                    uint4 l = s_edge[2u * j + 1u];
                    l.x &= ~byte_range_mask(0, (int)lastv[d], 0);
                    l.y &= ~byte_range_mask(0, (int)lastv[d], 1);
                    l.z &= ~byte_range_mask(0, (int)lastv[d], 2);
                    l.w &= ~byte_range_mask(0, (int)lastv[d], 3);
                    c += odd ? chunk_words<true>(l) : chunk_words<false>(l);
                }
                acc -= c;
            }
            res = finish(start_sum[d], acc);
        }
        src.put(i, res, ctx[d], i < n, ent[d]);
    }
    if constexpr (PFA > 0) {
        // never true (n > 0): keeps the load and all four of its registers live
        if ((pf.x ^ pf.y ^ pf.z ^ pf.w) == 0x5A5A5A5Au && n == 0u) s_tmp[0] = pf.y;
    }
}

// The prefetch distance of the product's batch calls: the resident tiles of a
// 256-CU MI355X (5 workgroups per CU at U 8).  Mixed, one process, 11 rounds:
// 640 ahead +0.6 %, 1 280 +1.2 %, 2 560 +1.0 %, 4 480 +0.2 % over none
// (profiles/r03_ab_flat_prefetch_mixed.json).
constexpr int kFlatPrefetchTiles = 1280;

template <int U, bool NT, int GORD, class Src, int D = 1, bool PIPE = false, int PFA = 0>
__global__ __launch_bounds__(FT) void k_flat2(const uint8_t* __restrict__ base, const Src src,
                                              uint32_t n) {
    flat2_body<U, NT, GORD, Src, D, PIPE, false, PFA>(base, src, n);
}

// --------------------------------------------- k_rx_hdr (RX header verify) --
//
// f1's header-only RX call (lvlip_rx_verify_dev without LVLIP_RX_VERIFY_L4) as
// one lane per frame.  The parse window FrWin, here its first three chunks,
// holds frame bytes [12, 45) at least: the whole IPv4 header for ihl 5-7, so
// the lane sums it from registers (header dword m = window bytes 14+4m ..
// 17+4m, one alignbyte each) and no entry, tile plan or second read of the
// header exists.  Header words past the window (options) come from byte
// loads.  The decisions are FrameSrc<FR_RX>'s (parse_rx) and the verdict
// rule its put's.
//
// PFA > 0: each lane also loads the frame descriptor PFA blocks ahead, after
// its own (as k_flat2's PFA), so that block's first round trip hits its XCD's
// L2 (A/B in the lab, mode 3 of lvlip_lab_frames_dev).
template <int PFA>
__global__ __launch_bounds__(256) void k_rx_hdr(const uint8_t* __restrict__ base,
                                                const lvlip_frame_desc* __restrict__ frames,
                                                uint32_t n, uint8_t* __restrict__ verdict) {
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f >= n) return;  // no cross-lane step below
    const FrameSrc<FR_RX> src{base, nullptr, frames, verdict};
    const uint4 raw = load_global(reinterpret_cast<uint64_t>(frames + f));
    uint4 pf = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (PFA > 0) {
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t fp = (uint64_t)f + (uint64_t)PFA * 256u;
        pf = load_global(reinterpret_cast<uint64_t>(frames + (fp < n ? fp : (uint64_t)f)));
        __builtin_amdgcn_sched_barrier(0);
    }
    lvlip_frame_desc fd;
    fd.offset = ((uint64_t)raw.y << 32) | raw.x;
    fd.len = raw.z;
    fd.reserved = 0;
    const uint8_t* h = base + fd.offset;
    // three chunks: frame bytes [12, cov), cov >= 45 (FrWin::load<3>), which
    // hold every field parse_rx reads in this mode and the header of ihl 5-7
    FrWin x;
    x.load<3>(h, fd.len, reinterpret_cast<uint64_t>(frames + f) & ~15ull);
    const uint32_t cov = 60u - (uint32_t)((reinterpret_cast<uint64_t>(h) + 12u) & 15u);
    lvlip_csum_desc d0 = fr_mk(0, 0, 0), d1 = fr_mk(0, 0, 0);
    uint32_t w = 0;
    src.parse_rx(fd, x, d0, d1, w);
    uint32_t v = w & 0xffu;
    if (w & FR_HAS_HDR) {
        const uint32_t ihl = x.b(14) & 0x0fu;
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t m = 0; m < 10u; ++m) {
            // header dword m = frame bytes 14+4m .. 17+4m: from the window when
            // it holds them, else from memory (options past the window)
            const bool inw = 18u + 4u * m <= cov;
            uint32_t hd = __builtin_amdgcn_alignbyte(x.A[m + 1u], x.A[m], 2u);
            if (m < ihl && !inw) hd = fr_le16(h + 14u + 4u * m) | (fr_le16(h + 16u + 4u * m) << 16);
            acc = dot2_acc(m < ihl ? hd : 0u, acc);
        }
        for (uint32_t k = 54u; k < FR_ETH + 4u * ihl; k += 2u) acc += fr_le16(h + k);
        // src/ip_input.c:38-43, as FrameSrc<FR_RX>::put
        if (finish(0u, acc) != 0u) v = LVLIP_RX_BAD_CSUM;
        v = v == 0u ? (uint32_t)LVLIP_RX_OK : (v & ~FR_PENDING);
    }
    verdict[f] = (uint8_t)v;
    if constexpr (PFA > 0) {
        // never true (n > f): keeps the prefetch and its four registers live
        if ((pf.x ^ pf.y ^ pf.z ^ pf.w) == 0x5A5A5A5Au && n == 0u) verdict[f] = (uint8_t)pf.y;
    }
}

}  // namespace lvlip

// ------------------------------------------------------------ host helpers --
namespace lvlip_host {

// CUs of HIP device `dev`, cached per device (256 on MI355X).
inline int cu_count(int dev) {
    static std::atomic<int> cache[64];
    if (dev < 0 || dev >= 64) return 256;
    int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
    cache[dev].store(c, std::memory_order_relaxed);
    return c;
}

inline int current_cus() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return cu_count(dev);
}

// A dispatch's grid is at most 2^32 - 1 work-items on this runtime, and the
// flat kernel runs one thread per descriptor: batches beyond kLaunchMax
// descriptors go out as several launches on the same stream (offsets stay
// relative to the same base, so nothing else changes).
constexpr uint32_t kLaunchMax = 1u << 30;

}  // namespace lvlip_host

namespace lvlip {

// ------------------------------------------ k_echo_reply (f4, RFC 1624) --
//
// icmpv4_reply (src/icmpv4.c:31-54) turns an echo request into the reply by
// setting type 8 -> 0 and recomputing the ICMP checksum over the whole message
// with the field zeroed (:45-47).  For a request whose checksum verified, the
// reply's field follows from the request's field alone (RFC 1624 eqn. 3,
// lvlip_icmp_echo_reply_csum in skb_batch.c): S = ~HC (0xffff
// when HC = 0xffff, the other zero), S' = S + ~0x0008 with end-around carry,
// field = ~S'.  S' = 0xffff cannot tell a zero-sum reply (field 0x0000) from
// an all-zero one (field 0xffff); that frame's lane sums the message itself.
// One lane per frame: the parse window (the product's: three chunks, frame
// bytes [12, 45) at least) holds the IPv4 header fields the checks read and,
// for ihl <= 6, the ICMP type, code and checksum (longer headers: byte
// loads); nothing else of the message is read except in the undecidable
// case.  Three chunks against four: 119.8 against 126.7 us per 2M mixed
// frames.
__device__ __forceinline__ uint32_t oc_add16(uint32_t a, uint32_t b) {
    const uint32_t t = a + b;
    return (t & 0xffffu) + (t >> 16);
}

// LVLIP_ECHO_FULL (icmpv4_reply's full sum for any request) is not this
// kernel: it runs on the flat sweep with a frame source (FrameSrc<FR_ECHO>,
// flat_src.h; round 5: 0.23 against 0.51 ms for one lane per frame summing
// its message alone, 1M requests).
// STP: the reply's store form (fr_store_echo_reply).  NCH: the parse window's
// chunks, 4 (frame bytes [12, 56): ihl <= 9 from registers) or 3 ([12, 45)
// at least: ihl <= 6, FrWin::load).
template <int STP, int NCH = 4>
__global__ __launch_bounds__(256) void k_echo_reply(uint8_t* __restrict__ base,
                                                    const lvlip_frame_desc* __restrict__ frames,
                                                    uint32_t n, uint8_t* __restrict__ status) {
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f >= n) return;  // no cross-lane step below
    const uint4 raw = load_global(reinterpret_cast<uint64_t>(frames + f));
    const uint64_t off = ((uint64_t)raw.y << 32) | raw.x;
    const uint32_t len = raw.z;
    uint8_t* h = base + off;
    FrWin x;
    x.load<NCH>(h, len, reinterpret_cast<uint64_t>(frames + f) & ~15ull);
    constexpr uint32_t kWinEnd = NCH == 4 ? 56u : 45u;  // window bytes valid below this
    uint32_t st = 0;
    // the checks of lvlip_icmp_echo_reply_fill (skb_batch.c): an IPv4 ICMP echo
    // request (type 8, code 0) whose message lies inside the frame
    if (len >= FR_ETH + 20u) {
        const uint32_t ver = x.b(14) >> 4, ihl = x.b(14) & 0x0fu, iplen = x.be16(16);
        const uint32_t l4 = FR_ETH + ihl * 4u;
        if (ver == 4u && ihl >= 5u && x.b(23) == 1u && iplen >= ihl * 4u + 4u && len >= FR_ETH + iplen) {
            // type, code and checksum from the window when it holds them
            // (ihl <= 9, or <= 6 with three chunks), else from memory
            uint32_t type, code, hc;
            if (l4 + 4u <= kWinEnd) {
                const uint32_t w = (ihl == 5u) ? x.le32(34) : (ihl == 6u) ? x.le32(38) : (ihl == 7u) ? x.le32(42)
                                 : (ihl == 8u) ? x.le32(46) : x.le32(50);
                type = w & 0xffu;
                code = (w >> 8) & 0xffu;
                hc = w >> 16;
            } else {
                type = h[l4];
                code = h[l4 + 1u];
                hc = fr_le16(h + l4 + 2u);
            }
            if (type == 8u && code == 0u) {
                const uint32_t icmp_len = iplen - ihl * 4u;
                const uint32_t S = hc == 0xffffu ? 0xffffu : (~hc & 0xffffu);
                const uint32_t S1 = oc_add16(S, 0xffffu - 0x0008u);
                uint32_t field;
                if (S1 != 0xffffu) {
                    field = ~S1 & 0xffffu;
                    st = 1u;
                } else {
                    // src/icmpv4.c:45-47: type 0, field 0, checksum over icmp_len
                    // bytes (words 0 and 1 are then zero)
                    const uint8_t* m = h + l4;
                    uint32_t acc = 0;
                    uint32_t k = 4u;
                    for (; k + 1u < icmp_len; k += 2u) acc += fr_le16(m + k);
                    if (k < icmp_len) acc += m[k];
                    field = finish(0u, acc);
                    st = 2u;
                }
                fr_store_echo_reply<STP>(h + l4, field);
            }
        }
    }
    if (status) status[f] = (uint8_t)st;
}

// f1/f2 on frames in HBM (include/lvlip_skb.h): one k_flat2 launch with a
// frame source (flat_src.h) per at most kLaunchMax entries, whole frames per
// launch.  out8 is the verdict / status array, or for FR_TX_REC the u64
// record array.  Returns LVLIP_EHIP when a launch fails (the error stays
// readable by hipGetLastError).
template <int MODE, int U, int GORD, int PFA = 0, int SEC = 0, int STP = 0>
int launch_frames_flat(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* out8,
                       hipStream_t s, bool nt_store) {
    using Src = FrameSrc<MODE, SEC, STP>;
    const uint32_t per = lvlip_host::kLaunchMax / Src::SLOTS;
    for (uint32_t f0 = 0; f0 < n;) {
        const uint32_t m = n - f0 < per ? n - f0 : per;
        const uint32_t entries = m * Src::SLOTS;
        const uint32_t grid = (uint32_t)(((uint64_t)entries + FT - 1) / FT);
        Src src{(const uint8_t*)base, (uint8_t*)base, frames + f0, out8 ? out8 + f0 : nullptr};
        if constexpr (MODE == FR_TX_REC) {
            src.out8 = nullptr;
            src.rec = reinterpret_cast<uint64_t*>(out8) + f0;
        }
        src.nt_store = nt_store;
        hipLaunchKernelGGL((k_flat2<U, true, GORD, Src, 1, false, PFA>), dim3(grid), dim3(FT), 0, s,
                           (const uint8_t*)base, src, entries);
        if (hipPeekAtLastError() != hipSuccess) return LVLIP_EHIP;
        f0 += m;
    }
    return LVLIP_OK;
}

}  // namespace lvlip
