// csum_kernels.hip — gfx950 (CDNA4) kernels for level-ip's Internet checksum,
// and Group 2 (device-resident batches) of include/lvlip_csum.h.
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
// Byte alignment (the flat and round-1 kernels; the ring kernels read through a
// per-packet buffer resource whose base is the packet's first byte instead, so
// their words are packet-relative, see below): the GPU reads whole 16-byte aligned chunks covering
// [offset, offset+len) and zeroes the bytes outside the packet.  When offset is
// odd, each aligned u16 holds (odd-relative byte, even-relative byte), so the
// two bytes of every half-dword are swapped before summing; the reference's
// tail byte (even relative index) then lands in the low byte as it should.
//
// Kernels (roofline: HBM read bandwidth; ~1 VALU op per loaded dword, no MFMA;
// DESIGN.md §4):
//   k_window  : the default from 896 B.  One wavefront per packet, persistent, a
//               ring of 2-KiB pieces in flight per wave; packets dealt to the
//               waves in small groups round robin over the grid, so the waves in
//               flight read one narrow window of the batch.
//   k_stream  : the same ring with contiguous per-wave ranges (A/B).
//   k_flat2   : the default below 896 B (ragged batches: 20-B headers next to
//               payloads).  A chunk-balanced tile sweep over 16-B chunks that
//               crosses packet boundaries; segment sums by a DPP prefix scan.
//               Also the frame calls' kernel (flat_src.h, skb_dev.hip).
//   k_wflat   : k_flat2's sweep one wave per tile, tiles dealt round robin (A/B).
//   k_wave_simple, k_wave_lds, k_flat : round-1 variants kept for A/B.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

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

template <int U>
__global__ __launch_bounds__(256) void k_wave_simple(const uint8_t* __restrict__ base,
                                              const lvlip_csum_desc* __restrict__ descs,
                                              uint32_t n, uint16_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * wpb;
    // 64-bit cursor: with n near LVLIP_MAX_BATCH a u32 p + stride would wrap
    for (uint64_t p = uniform(blockIdx.x * wpb + (threadIdx.x >> 6)); p < n; p += stride) {
        const lvlip_csum_desc d = descs[p];
        uint32_t w = 0;
        if (d.len > 0) {
            const uint64_t a0 = d.offset & ~15ull;
            const int lo = (int)(d.offset & 15ull);
            const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
            const uint32_t nch = (uint32_t)((span + 15u) >> 4);
            const uint32_t last_valid = (uint32_t)(span - 16ull * (nch - 1u));  // 1..16
            const uint4* src = reinterpret_cast<const uint4*>(base + a0);
            w = (d.offset & 1ull) ? wave_packet_sum<U, true>(src, nch, lo, last_valid, lane)
                                  : wave_packet_sum<U, false>(src, nch, lo, last_valid, lane);
        }
        w = wave_sum(w);
        if (lane == 0) out[p] = finish(d.start_sum, w);
    }
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
template <int G>
struct Deal {
    uint64_t nw, rank, p_lo;
    uint32_t cnt;  // the wave's packets

    // false when this wave has no packet
    __device__ __forceinline__ bool init(uint32_t n, uint32_t wid) {
        nw = (uint64_t)gridDim.x * SW_WAVES;
        if (G == 0) {
            rank = (uint64_t)blockIdx.x * SW_WAVES + wid;
            const uint64_t per = ((uint64_t)n + nw - 1) / nw;
            p_lo = rank * per;
            if (p_lo >= n) return false;
            cnt = (uint32_t)min<uint64_t>(per, (uint64_t)n - p_lo);
            return true;
        }
        rank = (gridDim.x & 7u) == 0u
                   ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * SW_WAVES + wid
                   : (uint64_t)blockIdx.x * SW_WAVES + wid;
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
template <int G>
__device__ __forceinline__ void fetch_window(const lvlip_csum_desc* __restrict__ descs,
                                             const Deal<G>& dl, uint32_t first, uint32_t lane,
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

template <int R, int G, int POL>
__device__ __forceinline__ void ring_sweep(const uint8_t* __restrict__ base,
                                           const lvlip_csum_desc* __restrict__ descs, uint32_t n,
                                           uint16_t* __restrict__ out, uint4 (*s_win)[64]) {
    constexpr uint32_t END = 0xffffffffu;
    constexpr uint32_t PIECE = 2048u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lane16 = lane * 16u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    Deal<G> dl;
    if (!dl.init(n, wid)) return;
    const uint32_t cnt = dl.cnt;

    // descriptor windows: the wave's packets [64w, 64w + 64) live in s_win[w & 1]
    fetch_window<G>(descs, dl, 0u, lane, s_win[0]);
    fetch_window<G>(descs, dl, 64u, lane, s_win[1]);
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
                        fetch_window<G>(descs, dl, ip + 64u, lane, s_win[((ip >> 6) + 1u) & 1u]);
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

// POL: the data loads' cache policy (A/B, LVLIP_LOAD_POLICY)
template <int R, int POL = 0>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ base,
                                                const lvlip_csum_desc* __restrict__ descs,
                                                uint32_t n, uint16_t* __restrict__ out) {
    __shared__ uint4 s_win[SW_WAVES][2][64];
    ring_sweep<R, 0, POL>(base, descs, n, out, s_win[uniform(threadIdx.x >> 6)]);
}

template <int R, int G>
__global__ __launch_bounds__(256) void k_window(const uint8_t* __restrict__ base,
                                                const lvlip_csum_desc* __restrict__ descs,
                                                uint32_t n, uint16_t* __restrict__ out) {
    static_assert(G > 0, "k_window deals groups of G >= 1 packets");
    __shared__ uint4 s_win[SW_WAVES][2][64];
    ring_sweep<R, G, 0>(base, descs, n, out, s_win[uniform(threadIdx.x >> 6)]);
}

// ------------------------------------------------- k_wave_lds (LDS-DMA path) --

template <int U, bool ODD>
__device__ __forceinline__ uint32_t wave_packet_sum_lds(const uint8_t* __restrict__ src,
                                                        uint32_t nch, int lo,
                                                        uint32_t last_valid, uint32_t lane,
                                                        uint4* slab /* U*64 chunks */) {
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64u * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * 64u + lane;
            // LDS destination is wave-uniform base + lane*16; the global source is
            // per lane.  Lanes past the packet re-read its first chunk (harmless,
            // in range) and are zeroed below.
            const uint8_t* g = src + 16ull * (c < nch ? c : 0u);
            __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(slab + u * 64), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * 64u + lane;
            uint4 v = slab[u * 64 + lane];
            if (c >= nch) v = make_uint4(0u, 0u, 0u, 0u);
            if (c == 0u || c == nch - 1u) {
                const int b0 = (c == 0u) ? lo : 0;
                const int b1 = (c == nch - 1u) ? (int)last_valid : 16;
                v = mask_chunk(v, b0, b1);
            }
            acc += chunk_words<ODD>(v);
        }
        // WAR: every lane's ds_read of this round must land before the next
        // round's DMA overwrites the slab.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return acc;
}

template <int U>
__global__ __launch_bounds__(256) void k_wave_lds(const uint8_t* __restrict__ base,
                                                  const lvlip_csum_desc* __restrict__ descs,
                                                  uint32_t n, uint16_t* __restrict__ out) {
    __shared__ uint4 slabs[4 * U * 64];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    uint4* slab = slabs + wid * (U * 64);
    const uint64_t stride = (uint64_t)gridDim.x * 4u;
    for (uint64_t p = uniform(blockIdx.x * 4u + wid); p < n; p += stride) {
        const lvlip_csum_desc d = descs[p];
        uint32_t w = 0;
        if (d.len > 0) {
            const uint64_t a0 = d.offset & ~15ull;
            const int lo = (int)(d.offset & 15ull);
            const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
            const uint32_t nch = (uint32_t)((span + 15u) >> 4);
            const uint32_t last_valid = (uint32_t)(span - 16ull * (nch - 1u));
            w = (d.offset & 1ull)
                    ? wave_packet_sum_lds<U, true>(base + a0, nch, lo, last_valid, lane, slab)
                    : wave_packet_sum_lds<U, false>(base + a0, nch, lo, last_valid, lane, slab);
        }
        w = wave_sum(w);
        if (lane == 0) out[p] = finish(d.start_sum, w);
    }
}

// ------------------------------------------------------ k_flat (ragged path) --

constexpr int FLAT_T = 256;                 // threads = descriptors per tile
constexpr uint32_t FLAT_MAX_CHUNKS = 1u << 16;  // bigger packets: whole-wave path

template <bool ODD>
__device__ __forceinline__ uint32_t words_of(uint4 v) { return chunk_words<ODD>(v); }

__global__ __launch_bounds__(FLAT_T) void k_flat(const uint8_t* __restrict__ base,
                                                 const lvlip_csum_desc* __restrict__ descs,
                                                 uint32_t n, uint16_t* __restrict__ out) {
    __shared__ uint32_t s_cstart[FLAT_T + 1];  // chunk prefix (exclusive), [T] = total
    __shared__ uint64_t s_a0[FLAT_T];          // 16-B aligned start offset
    __shared__ uint32_t s_meta[FLAT_T];        // lo | last_valid<<4 | odd<<9 | big<<10
    __shared__ uint32_t s_acc[FLAT_T];
    __shared__ uint32_t s_wsum[FLAT_T / 64];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wid = tid >> 6;
    const uint32_t tile0 = blockIdx.x * (uint32_t)FLAT_T;
    const uint32_t i_me = tile0 + tid;

    // 1. descriptor metadata + chunk counts
    uint32_t nch = 0, meta = 0;
    uint64_t a0 = 0;
    uint32_t start_sum = 0;
    bool big = false;
    if (i_me < n) {
        const lvlip_csum_desc d = descs[i_me];
        start_sum = d.start_sum;
        if (d.len > 0) {
            a0 = d.offset & ~15ull;
            const uint32_t lo = (uint32_t)(d.offset & 15ull);
            const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
            const uint64_t nch64 = (span + 15u) >> 4;
            const uint32_t last_valid = (uint32_t)(span - 16ull * (nch64 - 1u));
            big = nch64 > FLAT_MAX_CHUNKS;
            nch = big ? 0u : (uint32_t)nch64;
            meta = lo | (last_valid << 4) | ((uint32_t)(d.offset & 1ull) << 9) |
                   ((uint32_t)big << 10);
        }
    }
    s_a0[tid] = a0;
    s_meta[tid] = meta;
    s_acc[tid] = 0;

    // 2. exclusive prefix sum of nch over the tile (wave scan + wave totals)
    uint32_t incl = nch;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += t;
    }
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t k = 0; k < wid; ++k) wbase += s_wsum[k];
    s_cstart[tid] = wbase + incl - nch;
    if (tid == FLAT_T - 1) s_cstart[FLAT_T] = wbase + incl;
    __syncthreads();

    // 3. sweep the tile's chunks: lane j takes chunk j (coalesced across packets)
    const uint32_t total = s_cstart[FLAT_T];
    for (uint32_t j0 = wid * 64u; j0 < total; j0 += FLAT_T) {
        const uint32_t j = j0 + lane;
        uint32_t i = FLAT_T;  // sentinel for lanes past the end
        uint32_t val = 0;
        if (j < total) {
            // largest i with cstart[i] <= j (skips empty descriptors)
            i = 0;
#pragma unroll
            for (uint32_t step = FLAT_T / 2; step > 0; step >>= 1)
                if (s_cstart[i + step] <= j) i += step;
            const uint32_t k = j - s_cstart[i];
            const uint32_t m = s_meta[i];
            const uint32_t ni = s_cstart[i + 1] - s_cstart[i];
            uint4 v = *reinterpret_cast<const uint4*>(base + s_a0[i] + 16ull * k);
            if (k == 0u || k == ni - 1u) {
                const int b0 = (k == 0u) ? (int)(m & 15u) : 0;
                const int b1 = (k == ni - 1u) ? (int)((m >> 4) & 31u) : 16;
                v = mask_chunk(v, b0, b1);
            }
            val = (m & (1u << 9)) ? chunk_words<true>(v) : chunk_words<false>(v);
        }
        // segmented reduction keyed by i (non-decreasing across lanes)
        const uint32_t i_first = __shfl(i, 0, 64);
        const uint32_t i_last = __shfl(i, 63, 64);
        if (i_first == i_last) {
            val = wave_sum(val);
            if (lane == 0 && i_first < (uint32_t)FLAT_T) atomicAdd(&s_acc[i_first], val);
        } else {
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t v2 = __shfl_up(val, off, 64);
                const uint32_t i2 = __shfl_up(i, off, 64);
                if (lane >= (uint32_t)off && i2 == i) val += v2;
            }
            const uint32_t i_next = __shfl_down(i, 1, 64);
            const bool tail = (lane == 63u) || (i_next != i);
            if (tail && i < (uint32_t)FLAT_T) atomicAdd(&s_acc[i], val);
        }
    }

    // 4. packets too big for the tile sweep: one wave each
    __syncthreads();
    for (uint32_t q = 0; q < (uint32_t)FLAT_T; ++q) {
        if (!(s_meta[q] & (1u << 10))) continue;  // uniform: LDS broadcast
        if ((q & 3u) != wid) continue;
        const uint32_t m = s_meta[q];
        const lvlip_csum_desc d = descs[tile0 + q];
        const uint64_t span = (uint64_t)(m & 15u) + (uint64_t)(uint32_t)d.len;
        const uint32_t nchq = (uint32_t)((span + 15u) >> 4);
        const uint4* src = reinterpret_cast<const uint4*>(base + s_a0[q]);
        uint32_t w = (m & (1u << 9))
                         ? wave_packet_sum<2, true>(src, nchq, (int)(m & 15u), (m >> 4) & 31u, lane)
                         : wave_packet_sum<2, false>(src, nchq, (int)(m & 15u), (m >> 4) & 31u, lane);
        w = wave_sum(w);
        if (lane == 0) s_acc[q] = w;
    }
    __syncthreads();

    // 5. fold and store (coalesced 2-B stores)
    if (i_me < n) out[i_me] = finish(start_sum, s_acc[tid]);
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
template <int U, bool NT, int GORD, class Src, int D = 1>
__global__ __launch_bounds__(FT) void k_flat2(const uint8_t* __restrict__ base, const Src src,
                                              uint32_t n) {
    static_assert(D == 1 || D == 2, "descriptors per thread");
    constexpr uint32_t TD = (uint32_t)FT * D;   // descriptors per tile
    constexpr uint32_t FG = TD * FCAP / 64;     // most 64-chunk groups a tile can have
    __shared__ uint4 s_rec[TD];        // by rank: {a0 lo, a0 hi, cstart, meta}
    __shared__ uint2 s_grp[FG];        // by 64-chunk group: head bitmap {lo, hi}
    __shared__ uint16_t s_hb[FG];      // by 64-chunk group: heads before it (<= TD)
    __shared__ uint32_t s_acc[TD];     // by descriptor
    __shared__ uint32_t s_big[TD];     // descriptors longer than FCAP chunks
    __shared__ uint4 s_edge[2 * TD];   // by descriptor: raw first / last chunk
    __shared__ uint32_t s_tmp[8];

    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t tile0 = blockIdx.x * TD;
    const uint32_t t = tid;

    // ---- phase 1: descriptors -> chunk counts, ranks, records, head bitmap
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
    if (C > 0) {
        for (uint32_t gr = g_lo; gr < g_end; gr += rstep) {
            uint4 x[U];
            uint32_t mt[U], kk[U];
            bool vl[U];
            uint32_t hlo[U], hhi[U], hb[U];
            bool gv[U];
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
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!gv[u]) break;  // uniform
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
}

// ------------------------------------------- k_wflat (ragged, window deal) --
//
// k_flat2's chunk sweep, one wave per tile of D descriptors, with the tiles
// dealt round robin over the grid as k_window deals its packet groups: wave
// rank r (XCD-major) sweeps tiles r, r + nw, r + 2 nw, ...  A k_flat2 workgroup
// owns 256 descriptors (~100 KB of a mixed batch) and its four waves sweep
// contiguous quarters of them, so the waves in flight read ~8 000 streams over
// ~200 MB; here the waves in flight read one window of nw x D descriptors
// (~13-25 MB of a mixed batch) that slides through the batch.  The read probes
// on the mixed buffer measure that order 4.7 % faster (scripts/lab_window.py,
// DESIGN.md §4).
//
// Per tile, all in one wave (no workgroup barrier):
//   1. lane i < D reads descriptor i; chunk counts, an exclusive wave scan of
//      them (the tile's virtual chunk space), a rank among the non-empty small
//      descriptors (mbcnt of a ballot), records by rank and a head bitmap per
//      64-chunk load in the wave's LDS;
//   2. the sweep: U loads of 64 chunks per round, every lane's packet found as
//      in k_flat2 (heads before the load + mbcnt), bytes outside the packet
//      masked in the lane (its first and last chunk), odd-address packets
//      byte-swapped, and segment sums by the inclusive-scan trick into the
//      descriptor's LDS accumulator;
//   3. descriptors longer than WCAP chunks: one wave-per-packet loop each;
//   4. fold, ~, one store of the tile's D results.
constexpr uint32_t WCAP = 128;  // chunks of the largest swept descriptor (2 KiB)

template <int D>
struct WflatLds {
    uint4 rec[SW_WAVES][D];                 // by rank: {a0 lo, a0 hi, cstart, meta}
    uint2 msk[SW_WAVES][D * WCAP / 64];     // head bitmap per 64-chunk load
    uint32_t acc[SW_WAVES][D];              // by descriptor
    uint4 edge[SW_WAVES][2 * D];            // by descriptor: raw first / last chunk
};

// Orders this wave's LDS traffic across lanes (a lane reading what another
// lane wrote): LDS ops of one wave execute in order, so the compiler only has
// to be kept from moving them, and the counter drained.  No vmcnt: global
// loads in flight stay in flight.
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

template <int U, int D>
__global__ __launch_bounds__(256) void k_wflat(const uint8_t* __restrict__ base,
                                               const lvlip_csum_desc* __restrict__ descs,
                                               uint32_t n, uint16_t* __restrict__ out) {
    static_assert(D >= 1 && D <= 64, "one descriptor per lane");
    __shared__ WflatLds<D> L;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * SW_WAVES;
    const uint64_t rank =
        (gridDim.x & 7u) == 0u
            ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * SW_WAVES + wid
            : (uint64_t)blockIdx.x * SW_WAVES + wid;
    const uint64_t ntiles = ((uint64_t)n + D - 1) / D;
    uint4* s_rec = L.rec[wid];
    uint2* s_msk = L.msk[wid];
    uint32_t* s_acc = L.acc[wid];
    uint4* s_edge = L.edge[wid];

    // descriptors of the wave's next tile, one 16-B load per lane issued a tile
    // ahead (lanes past the batch re-read its last descriptor)
    // Issued from asm, so hipcc's wait-count pass does not see it in flight and
    // drain it before the sweep's first loads; the sweep's own waits retire it
    // (vector memory ops retire in issue order), and the loop head waits for it
    // explicitly, which costs nothing after a tile that had a sweep round.
    auto fetch = [&](uint64_t t, u32x4& d) {
        uint64_t i = t * D + (lane < (uint32_t)D ? lane : 0u);
        i = i < n ? i : n - 1u;
        const lvlip_csum_desc* g = descs + i;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(g) : "memory");
    };
    u32x4 dnext;
    fetch(rank < ntiles ? rank : 0u, dnext);
    // the previous tile's results, stored once the next prefetch is retired
    uint64_t i_prev = 0;
    bool st_prev = false;
    uint16_t res_prev = 0;
    for (uint64_t t = rank; t < ntiles; t += nw) {
        const uint64_t i = t * D + lane;
        const bool mine = lane < (uint32_t)D && i < n;
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(dnext) : : "memory");
        const u32x4 dv = dnext;  // {offset lo, offset hi, len, start_sum}
        // the previous tile's store and the next tile's prefetch go out behind
        // this tile's first sweep loads, so they share their round trip (the
        // store's data register is reused soon after, and the wait hipcc puts
        // before that reuse drains everything in flight)
        bool side_done = false;
        auto side = [&]() {
            if (st_prev) out[i_prev] = res_prev;
            st_prev = false;
            if (t + nw < ntiles) fetch(t + nw, dnext);
            side_done = true;
        };
        // ---- 1. descriptors -> chunk space, records, head bitmap
        uint32_t start_sum = 0, nch = 0, meta = 0;
        uint64_t a0 = 0;
        bool big = false;
        if (mine) {
            lvlip_csum_desc d;
            d.offset = ((uint64_t)dv.y << 32) | dv.x;
            d.len = (int32_t)dv.z;
            d.start_sum = dv.w;
            start_sum = d.start_sum;
            if (d.len > 0) {
                const uint64_t abs = reinterpret_cast<uint64_t>(base) + d.offset;
                a0 = abs & ~15ull;
                const uint32_t lo = (uint32_t)(abs & 15ull);
                const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
                const uint64_t c64 = (span + 15u) >> 4;
                const uint32_t lastv = (uint32_t)(span - 16ull * (c64 - 1u));  // 1..16
                big = c64 > WCAP;
                nch = big ? 0u : (uint32_t)c64;
                // edge flags: the sweep stashes the first (bit 24) and last (bit
                // 25) chunk in LDS when they hold bytes outside the descriptor,
                // and step 4 subtracts those bytes (as k_flat2)
                const bool ef = !big && (lo != 0u || (c64 == 1u && lastv != 16u));
                const bool el = !big && c64 > 1u && lastv != 16u;
                // meta: nch (8 bits) | lo << 8 | lastv << 12 | odd << 17 | lane << 18 | ef, el
                meta = nch | (lo << 8) | (lastv << 12) | ((uint32_t)(abs & 1ull) << 17) | (lane << 18) |
                       ((uint32_t)ef << 24) | ((uint32_t)el << 25);
            }
        }
        const uint32_t incl = wave_incl_scan(nch);
        const uint32_t C = uniform((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
        const uint32_t cstart = incl - nch;
        const uint64_t nz = __builtin_amdgcn_ballot_w64(nch != 0u);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u));
        const uint32_t nloads = (C + 63u) >> 6;
        for (uint32_t q = lane; q < nloads; q += 64u) s_msk[q] = make_uint2(0u, 0u);
        if (lane < (uint32_t)D) s_acc[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
        if (nch) {
            s_rec[r] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), cstart, meta);
            const uint32_t q = cstart >> 6, b = cstart & 63u;
            if (b < 32u) atomicOr(&s_msk[q].x, 1u << b);
            else atomicOr(&s_msk[q].y, 1u << (b - 32u));
        }
        lds_sync();

        // ---- 2. sweep the tile's chunk space, U loads of 64 chunks per round
        uint32_t heads = 0;  // heads in the loads before this round
        for (uint32_t u0 = 0; u0 < nloads; u0 += U) {
            uint32_t hb[U], hlo[U], hhi[U];
            bool gv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                gv[u] = u0 + u < nloads;
                const uint2 m = s_msk[gv[u] ? u0 + u : nloads - 1u];
                hlo[u] = uniform(m.x);
                hhi[u] = uniform(m.y);
                hb[u] = heads;
                heads += gv[u] ? (uint32_t)__popcll(((uint64_t)hhi[u] << 32) | hlo[u]) : 0u;
            }
            uint4 x[U], rec[U];
            uint32_t kk[U];
            bool vl[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = (u0 + u) * 64u + lane;
                vl[u] = gv[u] && c < C;
                const uint64_t H = ((uint64_t)hhi[u] << 32) | hlo[u];
                const uint64_t Hs = H >> 1;
                const uint32_t cnt = __builtin_amdgcn_mbcnt_hi((uint32_t)(Hs >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)Hs, 0u));
                // a valid chunk's packet: heads at or below it - 1 (chunk 0 is a
                // head); lanes past the chunk space read record 0's first chunk,
                // a valid address, and are zeroed
                const uint32_t rk = hb[u] + (uint32_t)(H & 1ull) + cnt - 1u;
                rec[u] = s_rec[vl[u] ? rk : 0u];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = (u0 + u) * 64u + lane;
                kk[u] = vl[u] ? c - rec[u].z : 0u;
                const uint64_t ca = (((uint64_t)rec[u].y << 32) | rec[u].x) + 16ull * kk[u];
                x[u] = load_nt_global(ca);
            }
            if (!side_done) side();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!gv[u]) break;  // uniform
                uint4 v = x[u];
                const uint32_t m = rec[u].w;
                const uint32_t pn = m & 0xFFu;
                const bool first = kk[u] == 0u;
                const bool last = kk[u] + 1u == pn;
                const uint32_t q = (m >> 18) & 63u;
                if (vl[u] && first && (m & (1u << 24))) s_edge[2u * q] = x[u];
                if (vl[u] && last && (m & (1u << 25))) s_edge[2u * q + 1u] = x[u];
                if (__builtin_amdgcn_ballot_w64((m & (1u << 17)) != 0u)) {
                    const uint32_t sel = (m & (1u << 17)) ? 0x02030001u : 0x03020100u;
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
                const uint32_t add = (first ? val - P : 0u) + ((last || lane == 63u) ? P : 0u);
                if (vl[u] && (first || last || lane == 63u)) atomicAdd(&s_acc[q], add);
            }
        }

        if (!side_done) side();  // a tile with nothing to sweep

        // ---- 3. descriptors longer than WCAP chunks, one wave each
        uint64_t bigm = __builtin_amdgcn_ballot_w64(big);
        while (bigm) {
            const uint32_t q = (uint32_t)__builtin_ctzll(bigm);
            bigm &= bigm - 1ull;
            const lvlip_csum_desc d = descs[t * D + q];
            const uint64_t abs = reinterpret_cast<uint64_t>(base) + d.offset;
            const int lo = (int)(abs & 15ull);
            const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
            const uint32_t nchq = (uint32_t)((span + 15u) >> 4);
            const uint32_t lastv = (uint32_t)(span - 16ull * (nchq - 1u));
            const uint4* src = reinterpret_cast<const uint4*>(abs & ~15ull);
            uint32_t w = (abs & 1ull) ? wave_packet_sum<4, true>(src, nchq, lo, lastv, lane)
                                      : wave_packet_sum<4, false>(src, nchq, lo, lastv, lane);
            w = wave_sum_dpp(w);
            if (lane == 0) s_acc[q] = w;
        }
        lds_sync();

        // ---- 4. edge corrections (bytes of the first / last chunk outside the
        // descriptor, once per descriptor, mod 2^32), fold; the store goes out
        // behind the next tile's first sweep loads
        uint32_t acc = s_acc[lane < (uint32_t)D ? lane : 0u];
        if (meta & (3u << 24)) {
            const bool odd = meta & (1u << 17);
            const int lo = (int)((meta >> 8) & 15u), lastv = (int)((meta >> 12) & 31u);
            uint32_t c = 0;
            if (meta & (1u << 24)) {
                uint4 f = s_edge[2u * lane];
                const int fb1 = (nch == 1u) ? lastv : 16;
                f.x &= ~byte_range_mask(lo, fb1, 0);
                f.y &= ~byte_range_mask(lo, fb1, 1);
                f.z &= ~byte_range_mask(lo, fb1, 2);
                f.w &= ~byte_range_mask(lo, fb1, 3);
                c += odd ? chunk_words<true>(f) : chunk_words<false>(f);
            }
            if (meta & (1u << 25)) {
                uint4 l = s_edge[2u * lane + 1u];
                l.x &= ~byte_range_mask(0, lastv, 0);
                l.y &= ~byte_range_mask(0, lastv, 1);
                l.z &= ~byte_range_mask(0, lastv, 2);
                l.w &= ~byte_range_mask(0, lastv, 3);
                c += odd ? chunk_words<true>(l) : chunk_words<false>(l);
            }
            acc -= c;
        }
        res_prev = finish(start_sum, acc);
        i_prev = i;
        st_prev = mine;
        __builtin_amdgcn_wave_barrier();
    }
    if (st_prev) out[i_prev] = res_prev;
}

// ------------------------------------------------ k_lane (small packets) --
//
// S lanes per packet (S = 1, 2, 4 or 8), for batches of packets a few 16-B
// chunks long (20-B IPv4 headers alone, 40-64-B headers and echo payloads).
// The flat sweep's per-tile plan (three block scans, the head bitmaps, the
// records, two LDS round trips per group) costs about as much as sweeping a
// tile of such packets: a 256-descriptor tile of 20-B headers is 8 KB of
// bytes.  Here a group of S lanes reads its packet's descriptor (every lane
// of the group the same one: one coalesced wave load per P), then lane s of
// the group reads the packet's aligned chunks s, s + S, ..., up to K of them,
// straight from the packet's address, and sums them in registers; an xor
// butterfly over the group adds the S partial sums.  No LDS and no barrier.
// With S chunks per packet slot (20-B headers in 32-B slots: S = 2) one wave
// load covers 64 consecutive chunks, so every load instruction is one
// contiguous 1-KiB read; with S = 1 the lanes of one load are a slot apart
// and a load touches 64 slots' lines (measured: 64-B packets 2.6 TB/s at
// S = 1).  Bytes outside the packet (the first chunk's lead-in, the last
// chunk's tail) are masked in the lane; odd-address packets are byte-swapped
// within u16 halves (see the file header).  A packet longer than S x K
// chunks is summed by the whole wave after the group phase
// (wave_packet_sum), one packet at a time.
template <int S, int P, int K, int M>
__global__ __launch_bounds__(256) void k_lane(const uint8_t* __restrict__ base,
                                              const lvlip_csum_desc* __restrict__ descs,
                                              uint32_t n, uint16_t* __restrict__ out) {
    static_assert(S == 1 || S == 2 || S == 4 || S == 8, "lanes per packet");
    constexpr uint32_t PB = 256 / S;  // packets per block and p
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t sub = threadIdx.x & (uint32_t)(S - 1);
    const uint32_t i0 = blockIdx.x * (PB * (uint32_t)P) + threadIdx.x / (uint32_t)S;
    uint4 dd[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const uint32_t i = i0 + PB * p;
        if (M == 0) {
            dd[p] = i < n ? load_global(reinterpret_cast<uint64_t>(descs + i)) : make_uint4(0u, 0u, 0u, 0u);
        } else {
            const uint4 v = load_global(reinterpret_cast<uint64_t>(descs + (i < n ? i : n - 1u)));
            dd[p] = i < n ? v : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    // Chunk loads, M = 0 (default): only the lanes with a chunk to read load
    // (exec-masked).  hipcc turns each conditional load into a branch and
    // retires each packet's K loads at the join, so a lane has K chunks in
    // flight at a time.  M = 1 (A/B): every lane loads unconditionally, a lane
    // with nothing to read from one wave-uniform address (the descriptor
    // array's first 16 B), and all P x K loads are issued before any is used
    // (sched_barrier).  Measured, M = 0 is faster: the masked lanes cost the
    // address unit nothing, and enough waves cover the latency.
    const uint64_t safe = reinterpret_cast<uint64_t>(descs);
    uint64_t a0[P];
    uint32_t lo[P], nch[P], lastv[P];
    uint4 x[P][K];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const uint64_t abs = reinterpret_cast<uint64_t>(base) + (((uint64_t)dd[p].y << 32) | dd[p].x);
        const int32_t len = (int32_t)dd[p].z;
        a0[p] = abs & ~15ull;
        lo[p] = (uint32_t)(abs & 15ull);
        const uint64_t span = (uint64_t)lo[p] + (uint64_t)(uint32_t)(len > 0 ? len : 0);
        nch[p] = len > 0 ? (uint32_t)((span + 15u) >> 4) : 0u;
        lastv[p] = len > 0 ? (uint32_t)(span - 16ull * (nch[p] - 1u)) : 16u;
        const bool in_group = nch[p] <= (uint32_t)(S * K);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = sub + (uint32_t)(S * k);
            const bool want = in_group && c < nch[p];
            if (M == 0)
                x[p][k] = want ? load_nt_global(a0[p] + 16ull * c) : make_uint4(0u, 0u, 0u, 0u);
            else
                x[p][k] = load_nt_global(want ? a0[p] + 16ull * c : safe);
        }
    }
    if (M == 1) __builtin_amdgcn_sched_barrier(0);
    uint32_t acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const uint32_t sel = (lo[p] & 1u) ? 0x02030001u : 0x03020100u;
        const bool in_group = nch[p] <= (uint32_t)(S * K);
        uint32_t a = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t c = sub + (uint32_t)(S * k);
            uint4 v = M == 0 || (in_group && c < nch[p]) ? x[p][k] : make_uint4(0u, 0u, 0u, 0u);
            const int b0 = c == 0u ? (int)lo[p] : 0;
            const int b1 = c + 1u == nch[p] ? (int)lastv[p] : 16;
            // M = 1: unconditional (no branch), all-ones masks for the middle chunks
            if (M == 1 || c == 0u || c + 1u == nch[p]) v = mask_chunk(v, b0, b1);
            a = dot2_acc(__builtin_amdgcn_perm(v.x, v.x, sel), a);
            a = dot2_acc(__builtin_amdgcn_perm(v.y, v.y, sel), a);
            a = dot2_acc(__builtin_amdgcn_perm(v.z, v.z, sel), a);
            a = dot2_acc(__builtin_amdgcn_perm(v.w, v.w, sel), a);
        }
#pragma unroll
        for (int off = 1; off < S; off <<= 1) a += __shfl_xor(a, off, 64);
        acc[p] = a;
    }
    // packets longer than S x K chunks: the whole wave, one packet at a time
#pragma unroll
    for (int p = 0; p < P; ++p) {
        uint64_t big = __builtin_amdgcn_ballot_w64(sub == 0u && nch[p] > (uint32_t)(S * K));
        while (big) {
            const uint32_t q = (uint32_t)__builtin_ctzll(big);
            big &= big - 1ull;
            const uint64_t qa0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(a0[p] >> 32), (int)q) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0[p], (int)q);
            const uint32_t qlo = (uint32_t)__builtin_amdgcn_readlane((int)lo[p], (int)q);
            const uint32_t qn = (uint32_t)__builtin_amdgcn_readlane((int)nch[p], (int)q);
            const uint32_t qlv = (uint32_t)__builtin_amdgcn_readlane((int)lastv[p], (int)q);
            const uint4* src = reinterpret_cast<const uint4*>(qa0);
            uint32_t w = (qlo & 1u) ? wave_packet_sum<4, true>(src, qn, (int)qlo, qlv, lane)
                                    : wave_packet_sum<4, false>(src, qn, (int)qlo, qlv, lane);
            w = wave_sum_dpp(w);
            if (lane == q) acc[p] = w;
        }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const uint32_t i = i0 + PB * p;
        if (sub == 0u && i < n) out[i] = finish(dd[p].w, acc[p]);
    }
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
__global__ __launch_bounds__(256) void k_rx_hdr(const uint8_t* __restrict__ base,
                                                const lvlip_frame_desc* __restrict__ frames,
                                                uint32_t n, uint8_t* __restrict__ verdict) {
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f >= n) return;  // no cross-lane step below
    const FrameSrc<FR_RX> src{base, nullptr, frames, verdict};
    const uint4 raw = load_global(reinterpret_cast<uint64_t>(frames + f));
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
}
}  // namespace lvlip

// ======================================================== host side (C ABI) ==

namespace {

thread_local char g_last_err[256] = "";

int hip_fail(hipError_t e, const char* what) {
    snprintf(g_last_err, sizeof g_last_err, "%s: %s", what, hipGetErrorString(e));
    return LVLIP_EHIP;
}

}  // namespace

// Shared with skb_dev.hip (hidden: -fvisibility=hidden keeps it internal).
int lvlip_internal_hip_fail(hipError_t e, const char* what) { return hip_fail(e, what); }

namespace {

struct DevInfo {
    std::atomic<int> cus{0};
};
DevInfo g_dev[64];

int cu_count(int dev) {
    if (dev < 0 || dev >= 64) return 256;
    int c = g_dev[dev].cus.load(std::memory_order_relaxed);
    if (c > 0) return c;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        c <= 0)
        c = 256;
    g_dev[dev].cus.store(c, std::memory_order_relaxed);
    return c;
}

uint32_t grid_for(uint32_t n, uint32_t packets_per_block, int waves_per_cu, int waves_per_block) {
    uint64_t blocks = ((uint64_t)n + packets_per_block - 1) / packets_per_block;
    if (waves_per_cu > 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        const uint64_t cap = (uint64_t)cu_count(dev) * (uint64_t)waves_per_cu / waves_per_block;
        if (cap > 0 && blocks > cap) blocks = cap;
    }
    if (blocks == 0) blocks = 1;
    return (uint32_t)blocks;
}

template <int U>
void launch_wave_simple(uint32_t grid, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                        uint32_t n, uint16_t* out) {
    hipLaunchKernelGGL(lvlip::k_wave_simple<U>, dim3(grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

// Persistent streaming launch: waves_per_cu waves on every CU, each owning a
// contiguous range of ceil(n / waves) packets.
// LVLIP_LOAD_POLICY (A/B knob, read once): the data loads' cache
// policy.  nt (default) | temporal | nt_sc1 | nt_sc0sc1 | sc1; the flat kernel
// knows nt and temporal only (anything else is nt there).
int load_policy() {
    static const int pol = [] {
        const char* e = getenv("LVLIP_LOAD_POLICY");
        if (!e) return 0;
        if (!strcmp(e, "temporal")) return 1;
        if (!strcmp(e, "nt_sc1")) return 2;
        if (!strcmp(e, "nt_sc0sc1")) return 3;
        if (!strcmp(e, "sc1")) return 4;
        return 0;
    }();
    return pol;
}
bool load_nt() { return load_policy() != 1; }

// LVLIP_FLAT_GROUPS (A/B knob, read once): k_flat2's group order.
// block (default, 2: rounds of 4U consecutive groups, U per wave) | quarters
// (1: contiguous quarters of the tile per wave, round 1's order) | interleaved
// (0: groups w, w+4, ...; batch calls only).
int flat_group_order() {
    static const int c = [] {
        const char* e = getenv("LVLIP_FLAT_GROUPS");
        if (e && strcmp(e, "interleaved") == 0) return 0;
        if (e && strcmp(e, "quarters") == 0) return 1;
        return 2;
    }();
    return c;
}

// LVLIP_FLAT_LDS_PAD (A/B knob, read once): bytes of unused dynamic LDS per
// k_flat2 workgroup, which caps the resident workgroups per CU (160 KiB / (19 KiB
// + pad)); 0 = none.
size_t flat_lds_pad() {
    static const size_t v = [] {
        const char* e = getenv("LVLIP_FLAT_LDS_PAD");
        const long x = e ? atol(e) : 0;
        return (size_t)(x < 0 ? 0 : (x > 131072 ? 131072 : x));
    }();
    return v;
}

// k_stream: waves_per_cu waves on every CU (fewer when the batch has fewer
// packets), whole 256-thread blocks; each wave owns a contiguous range of
// ceil(n / waves) packets.
template <int U>
void launch_stream(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                   uint32_t n, uint16_t* out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint64_t waves = (uint64_t)cu_count(dev) * (uint64_t)waves_per_cu;
    if (waves > n) waves = n;
    waves = (waves + 3) & ~3ull;  // whole 256-thread blocks
    const uint32_t grid = (uint32_t)(waves / 4);
    switch (load_policy()) {
#define LVLIP_STREAM_POL(P)                                                              \
    case P:                                                                              \
        hipLaunchKernelGGL((lvlip::k_stream<U, P>), dim3(grid), dim3(256), 0, s,         \
                           (const uint8_t*)base, d, n, out);                             \
        break;
        LVLIP_STREAM_POL(1)
        LVLIP_STREAM_POL(2)
        LVLIP_STREAM_POL(3)
        LVLIP_STREAM_POL(4)
#undef LVLIP_STREAM_POL
        default:
            hipLaunchKernelGGL((lvlip::k_stream<U, 0>), dim3(grid), dim3(256), 0, s,
                               (const uint8_t*)base, d, n, out);
    }
}

// k_window: waves_per_cu waves on every CU (fewer when the batch has fewer
// groups), R pieces in flight per wave, groups of G packets.  The grid stays a
// multiple of 8 blocks when it can, so the ranks are XCD-major.
template <int R, int G>
void launch_window_g(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint64_t waves = (uint64_t)cu_count(dev) * (uint64_t)waves_per_cu;
    const uint64_t ng = ((uint64_t)n + G - 1) / G;
    if (waves > ng) waves = ng;
    uint64_t grid = (waves + lvlip::SW_WAVES - 1) / lvlip::SW_WAVES;
    if (grid > 8) grid = grid & ~7ull;
    hipLaunchKernelGGL((lvlip::k_window<R, G>), dim3((uint32_t)grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

// Packets per group: the caller's (cfg->unroll >> 8), else LVLIP_WINDOW_GROUP
// (A/B knob, read once), else by the length hint.
int window_group(int requested, int len_hint) {
    static const int v = [] {
        const char* e = getenv("LVLIP_WINDOW_GROUP");
        return e ? atoi(e) : 0;
    }();
    if (requested == 1 || requested == 2 || requested == 3 || requested == 4 || requested == 8)
        return requested;
    if (v == 1 || v == 2 || v == 3 || v == 4 || v == 8) return v;
    // no group in the request: as AUTO (dispatch_one) picks for this hint
    if (len_hint >= 4096) return 3;
    if (len_hint >= 1792) return 2;
    return 4;
}

template <int R>
void launch_window(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                   uint32_t n, uint16_t* out, int group, int len_hint) {
    switch (window_group(group, len_hint)) {
        case 1: launch_window_g<R, 1>(waves_per_cu, s, base, d, n, out); break;
        case 3: launch_window_g<R, 3>(waves_per_cu, s, base, d, n, out); break;
        case 4: launch_window_g<R, 4>(waves_per_cu, s, base, d, n, out); break;
        case 8: launch_window_g<R, 8>(waves_per_cu, s, base, d, n, out); break;
        default: launch_window_g<R, 2>(waves_per_cu, s, base, d, n, out); break;
    }
}

// k_wflat: waves_per_cu waves on every CU (fewer when the batch has fewer
// tiles); the grid stays a multiple of 8 blocks when it can (XCD-major ranks).
template <int U, int D>
void launch_wflat_ud(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint64_t waves = (uint64_t)cu_count(dev) * (uint64_t)waves_per_cu;
    const uint64_t nt = ((uint64_t)n + D - 1) / D;
    if (waves > nt) waves = nt;
    uint64_t grid = (waves + lvlip::SW_WAVES - 1) / lvlip::SW_WAVES;
    if (grid > 8) grid = grid & ~7ull;
    hipLaunchKernelGGL((lvlip::k_wflat<U, D>), dim3((uint32_t)grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

template <int U>
bool launch_wflat(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                  uint32_t n, uint16_t* out, int tile) {
    switch (tile) {
        case 16: launch_wflat_ud<U, 16>(waves_per_cu, s, base, d, n, out); return true;
        case 32: launch_wflat_ud<U, 32>(waves_per_cu, s, base, d, n, out); return true;
        case 64: launch_wflat_ud<U, 64>(waves_per_cu, s, base, d, n, out); return true;
        default: return false;
    }
}

// k_lane: S lanes per packet, P packets per lane group, K chunks per lane;
// one launch wave.
template <int S, int P, int K>
void launch_lane_spk(int mode, hipStream_t s, const void* base, const lvlip_csum_desc* d, uint32_t n,
                     uint16_t* out) {
    constexpr uint64_t per_block = 256 / S * P;
    const uint32_t grid = (uint32_t)(((uint64_t)n + per_block - 1) / per_block);
    if (mode)
        hipLaunchKernelGGL((lvlip::k_lane<S, P, K, 1>), dim3(grid), dim3(256), 0, s,
                           (const uint8_t*)base, d, n, out);
    else
        hipLaunchKernelGGL((lvlip::k_lane<S, P, K, 0>), dim3(grid), dim3(256), 0, s,
                           (const uint8_t*)base, d, n, out);
}

bool launch_lane(int lanes, int per_group, int chunks, int mode, hipStream_t s, const void* base,
                 const lvlip_csum_desc* d, uint32_t n, uint16_t* out) {
    switch ((lanes << 16) | (chunks << 8) | per_group) {
#define LVLIP_LANE(SS, PP, KK) \
    case (SS << 16) | (KK << 8) | PP: launch_lane_spk<SS, PP, KK>(mode, s, base, d, n, out); return true;
        LVLIP_LANE(1, 2, 4) LVLIP_LANE(1, 4, 4) LVLIP_LANE(1, 2, 6)
        LVLIP_LANE(2, 2, 2) LVLIP_LANE(2, 4, 2) LVLIP_LANE(2, 4, 1) LVLIP_LANE(2, 8, 1)
        LVLIP_LANE(2, 2, 4)
        LVLIP_LANE(4, 2, 1) LVLIP_LANE(4, 4, 1) LVLIP_LANE(4, 8, 1) LVLIP_LANE(4, 2, 2)
        LVLIP_LANE(4, 4, 2)
        LVLIP_LANE(8, 4, 1) LVLIP_LANE(8, 2, 2) LVLIP_LANE(8, 4, 2)
#undef LVLIP_LANE
        default: return false;
    }
}

template <int U>
void launch_wave_lds(uint32_t grid, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    hipLaunchKernelGGL(lvlip::k_wave_lds<U>, dim3(grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

}  // namespace

extern "C" {

const char* lvlip_strerror(int err) {
    switch (err) {
        case LVLIP_OK: return "ok";
        case LVLIP_EINVAL: return "invalid argument";
        case LVLIP_ENODEV: return "no HIP device";
        case LVLIP_EHIP: return "HIP runtime error";
        case LVLIP_ENOMEM: return "out of memory";
        case LVLIP_ERANGE: return "batch exceeds context arena";
        default: return "unknown error";
    }
}

int lvlip_abi_version(void) { return LVLIP_CSUM_ABI_VERSION; }

const char* lvlip_last_hip_error(void) { return g_last_err; }

int lvlip_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

}  // extern "C"

namespace {

// AUTO's k_lane range: hints below this many bytes (scripts/shape_sweep.py,
// DESIGN.md §4).  LVLIP_LANE_HINT_MAX overrides it (A/B knob, read once).
int lane_hint_max() {
    static const int v = [] {
        const char* e = getenv("LVLIP_LANE_HINT_MAX");
        return e ? atoi(e) : 33;
    }();
    return v;
}

// One launch of the selected kernel over n <= kLaunchMax descriptors.
int dispatch_one(const void* base, const lvlip_csum_desc* descs, uint32_t n, uint16_t* out,
                 hipStream_t s, const lvlip_launch_cfg* cfg) {
    int kernel = cfg ? cfg->kernel : LVLIP_KERNEL_AUTO;
    int unroll = cfg ? cfg->unroll : 0;
    int wpc = cfg ? cfg->waves_per_cu : 0;
    if (kernel == LVLIP_KERNEL_AUTO) {
        // Measured on MI355X: the interleaved stream (k_window)
        // leads on uniform MTU/jumbo segments, the flat sweep on mixed
        // header/payload batches and stays within ~10 % elsewhere, so it is the
        // choice when sizes are unknown.
        const int hint = cfg ? cfg->len_hint : 0;
        if (hint >= 896) {
            // the interleaved stream, shapes from scripts/shape_sweep.py
            // (DESIGN.md §4): 2 pieces in flight per wave; more waves per CU for
            // smaller packets (per-packet work); groups of 4 packets below
            // 1792 B, 2 up to 4 KiB, 3 for jumbo packets (power-of-two group
            // bytes such as 2 x 4096 measured 3 % slow)
            kernel = LVLIP_KERNEL_WINDOW;
            if (wpc <= 0) wpc = hint < 1280 ? 16 : (hint < 1792 ? 12 : 8);
            if (unroll <= 0) {
                // ... but at least 16 groups per wave, or the last round of
                // groups leaves most waves idle (45 776 packets of 64 KiB: G 3
                // 6 698, G 1 6 974 GB/s)
                int dev = 0;
                (void)hipGetDevice(&dev);
                const uint64_t nw = (uint64_t)cu_count(dev) * (uint64_t)wpc;
                int g = hint < 1792 ? 4 : (hint < 4096 ? 2 : 3);
                while (g > 1 && (uint64_t)n < 16ull * (uint64_t)g * nw) --g;
                unroll = 2 | (g << 8);
            }
        } else {
            // below ~900 B the flat sweep leads (uniform 512 / 768 B: 6 442 /
            // 6 482 vs 3 973 / 5 916 GB/s for the stream), 4 loads per round
            // below 320 B (64 / 128 B: 4 973 / 6 114 vs 3 825 / 5 448 with 8),
            // 2 below 40 B (IPv4 headers alone, 20 B: 2 356 vs 2 251 with 4)
            kernel = LVLIP_KERNEL_FLAT;
            if (unroll <= 0 && hint > 0 && hint < 320) unroll = hint < 40 ? 2 : 4;
            // up to 32 B (IPv4 headers alone, 20-32 B in 32-B slots): two
            // lanes per packet read every slot pair as one contiguous wave
            // load, no tile plan (20 / 32 B: 2 819 / 4 356 vs 2 474 / 4 121
            // GB/s for the flat sweep; 36 B: 3 108 vs 3 469)
            if (hint > 0 && hint < lane_hint_max()) {
                kernel = LVLIP_KERNEL_LANE;
                unroll = 0;
            }
        }
    }

    switch (kernel) {
        case LVLIP_KERNEL_WAVE:
        case LVLIP_KERNEL_WAVE_STATIC:
        case LVLIP_KERNEL_WAVE_DYN: {
            // k_stream: contiguous ranges (A/B against the window deal); unroll =
            // 2-KiB pieces in flight per wave.  WAVE_STATIC and WAVE_DYN are the
            // ids of round 1's split and dynamic-tail variants;
            // both run the contiguous split now.
            if (unroll <= 0) unroll = 2;
            const int w = wpc > 0 ? wpc : 16;
            switch (unroll) {
                case 2: launch_stream<2>(w, s, base, descs, n, out); break;
                case 3: launch_stream<3>(w, s, base, descs, n, out); break;
                case 4: launch_stream<4>(w, s, base, descs, n, out); break;
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case LVLIP_KERNEL_WINDOW: {
            // unroll = 2-KiB pieces in flight per wave (low byte, default 3) |
            // packets per group << 8 (0 = by len_hint); 8 waves/CU by default
            if (unroll < 0) unroll = 0;
            const int group = (unroll >> 8) & 0xff;
            if ((unroll >> 16) != 0 ||
                (group != 0 && group != 1 && group != 2 && group != 3 && group != 4 && group != 8))
                return LVLIP_EINVAL;
            int r = unroll & 0xff;
            if (r == 0) r = 3;
            const int w = wpc > 0 ? wpc : 8;
            const int hint = cfg ? cfg->len_hint : 0;
            switch (r) {
                case 2: launch_window<2>(w, s, base, descs, n, out, group, hint); break;
                case 3: launch_window<3>(w, s, base, descs, n, out, group, hint); break;
                case 4: launch_window<4>(w, s, base, descs, n, out, group, hint); break;
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case LVLIP_KERNEL_WFLAT: {
            // unroll = 64-chunk loads per round (low byte, default 4) | descriptors
            // per tile << 8 (16, 32 or 64; 0 = 32); 8 waves/CU by default
            int u = unroll > 0 ? unroll & 0xff : 0;
            int tile = unroll > 0 ? (unroll >> 8) & 0xff : 0;
            if (u == 0) u = 4;
            if (tile == 0) tile = 32;
            const int w = wpc > 0 ? wpc : 8;
            bool ok = false;
            switch (u) {
                case 2: ok = launch_wflat<2>(w, s, base, descs, n, out, tile); break;
                case 4: ok = launch_wflat<4>(w, s, base, descs, n, out, tile); break;
                case 8: ok = launch_wflat<8>(w, s, base, descs, n, out, tile); break;
                default: break;
            }
            if (!ok) return LVLIP_EINVAL;
            break;
        }
        case LVLIP_KERNEL_LANE: {
            // unroll = packets per lane group (low byte, default 4) | chunks per
            // lane << 8 (default 2) | lanes per packet << 16 (1, 2, 4 or 8;
            // default 2) | load mode << 24 (0 masked, 1 unconditional: A/B):
            // the default sums any packet of <= 49 B in its group (20-B
            // headers at any alignment)
            if (unroll < 0 || (unroll >> 25) != 0) return LVLIP_EINVAL;
            int pg = unroll & 0xff, ch = (unroll >> 8) & 0xff, sl = (unroll >> 16) & 0xff;
            const int mode = (unroll >> 24) & 1;
            if (pg == 0) pg = 4;
            if (ch == 0) ch = 2;
            if (sl == 0) sl = 2;
            if (!launch_lane(sl, pg, ch, mode, s, base, descs, n, out)) return LVLIP_EINVAL;
            break;
        }
        case LVLIP_KERNEL_WAVE_SIMPLE: {
            if (unroll <= 0) unroll = 2;
            const uint32_t grid = grid_for(n, 4, wpc, 4);
            switch (unroll) {
                case 1: launch_wave_simple<1>(grid, s, base, descs, n, out); break;
                case 2: launch_wave_simple<2>(grid, s, base, descs, n, out); break;
                case 4: launch_wave_simple<4>(grid, s, base, descs, n, out); break;
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case LVLIP_KERNEL_WAVE_LDS: {
            if (unroll <= 0) unroll = 2;
            const uint32_t grid = grid_for(n, 4, wpc, 4);
            switch (unroll) {
                case 1: launch_wave_lds<1>(grid, s, base, descs, n, out); break;
                case 2: launch_wave_lds<2>(grid, s, base, descs, n, out); break;
                case 4: launch_wave_lds<4>(grid, s, base, descs, n, out); break;
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case LVLIP_KERNEL_FLAT: {
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
            // 8 loads of 64 chunks per round: 94 VGPRs, 5 workgroups per CU with
            // 8 KiB in flight per wave; 2-3 % ahead of 4 (8 workgroups, 4 KiB)
            // on mixed in 3 of 4 same-process A/B runs
            if (unroll < 0) unroll = 0;
            if ((unroll >> 11) != 0) return LVLIP_EINVAL;
            const int uo = (unroll >> 8) & 3;  // group order + 1 (A/B), 0 = the knob's
            const bool d2 = (unroll >> 10) & 1;  // 2 descriptors per thread (A/B)
            unroll &= 0xFF;
            if (unroll <= 0) unroll = 8;
            const bool nt = load_nt();
            const int gord = uo ? uo - 1 : flat_group_order();
            if (d2) {
                // tiles of 512 descriptors (nontemporal loads only)
                const uint32_t grid2 = (uint32_t)(((uint64_t)n + 2 * lvlip::FT - 1) / (2 * lvlip::FT));
                switch (unroll * 8 + gord) {
#define LVLIP_FLAT_D2(UU, CG)                                                                  \
    case UU * 8 + CG:                                                                         \
        hipLaunchKernelGGL((lvlip::k_flat2<UU, true, CG, lvlip::DescSrc, 2>), dim3(grid2),     \
                           dim3(lvlip::FT), flat_lds_pad(), s, (const uint8_t*)base,         \
                           lvlip::DescSrc{descs, out}, n);                                  \
        break;
                    LVLIP_FLAT_D2(4, 1) LVLIP_FLAT_D2(4, 2) LVLIP_FLAT_D2(8, 1) LVLIP_FLAT_D2(8, 2)
#undef LVLIP_FLAT_D2
                    default: return LVLIP_EINVAL;
                }
                break;
            }
            switch (unroll * 8 + (nt ? 4 : 0) + gord) {
#define LVLIP_FLAT(UU, NTV, CG)                                                               \
    case UU * 8 + (NTV ? 4 : 0) + CG:                                                        \
        hipLaunchKernelGGL((lvlip::k_flat2<UU, NTV, CG, lvlip::DescSrc>), dim3(grid),         \
                           dim3(lvlip::FT), flat_lds_pad(), s, (const uint8_t*)base,         \
                           lvlip::DescSrc{descs, out}, n);                                  \
        break;
                LVLIP_FLAT(2, true, 1) LVLIP_FLAT(2, true, 0) LVLIP_FLAT(2, true, 2)
                LVLIP_FLAT(2, false, 1) LVLIP_FLAT(2, false, 0) LVLIP_FLAT(2, false, 2)
                LVLIP_FLAT(4, true, 1) LVLIP_FLAT(4, true, 0) LVLIP_FLAT(4, true, 2)
                LVLIP_FLAT(4, false, 1) LVLIP_FLAT(4, false, 0) LVLIP_FLAT(4, false, 2)
                LVLIP_FLAT(8, true, 1) LVLIP_FLAT(8, true, 0) LVLIP_FLAT(8, true, 2)
                LVLIP_FLAT(8, false, 1) LVLIP_FLAT(8, false, 0) LVLIP_FLAT(8, false, 2)
                LVLIP_FLAT(6, true, 1) LVLIP_FLAT(6, true, 2) LVLIP_FLAT(12, true, 1) LVLIP_FLAT(12, true, 2)
#undef LVLIP_FLAT
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case 5: {  // first-generation flat kernel, kept for A/B measurement
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FLAT_T - 1) / lvlip::FLAT_T);
            hipLaunchKernelGGL(lvlip::k_flat, dim3(grid), dim3(lvlip::FLAT_T), 0, s,
                               (const uint8_t*)base, descs, n, out);
            break;
        }
        default: return LVLIP_EINVAL;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    return LVLIP_OK;
}

// A dispatch's grid is at most 2^32 - 1 work-items on this runtime, and the
// flat kernel runs one thread per descriptor: batches beyond kLaunchMax
// descriptors go out as several launches on the same stream (offsets stay
// relative to the same base, so nothing else changes).
constexpr uint32_t kLaunchMax = 1u << 30;

}  // namespace

extern "C" {

int lvlip_csum_batch_dev_ex(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                            uint16_t* out, void* stream, const lvlip_launch_cfg* cfg) {
    if (n == 0) return LVLIP_OK;
    if (!base || !descs || !out || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    if (((uintptr_t)base & 15u) != 0) return LVLIP_EINVAL;
    for (uint32_t lo = 0; lo < n;) {
        const uint32_t m = n - lo < kLaunchMax ? n - lo : kLaunchMax;
        const int rc = dispatch_one(base, descs + lo, m, out + lo, (hipStream_t)stream, cfg);
        if (rc != LVLIP_OK) return rc;
        lo += m;
    }
    return LVLIP_OK;
}

int lvlip_csum_batch_dev(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                         uint16_t* out, void* stream) {
    return lvlip_csum_batch_dev_ex(base, descs, n, out, stream, nullptr);
}

}  // extern "C"

namespace {

// LVLIP_FRAMES_UNROLL (A/B knob, read once): loads per round of the frame
// calls' sweep, 4 (default) or 8.
int frames_unroll() {
    static const int v = [] {
        const char* e = getenv("LVLIP_FRAMES_UNROLL");
        return e && atoi(e) == 8 ? 8 : 4;
    }();
    return v;
}

// LVLIP_FRAMES_GROUPS (A/B knob, read once): the frame calls' k_flat2 group
// order, quarters (default) | block.  Blocks measured 7-9 % slower on the RX
// header call (20-B pieces, 0.090 vs 0.084 ms) and within 1 % on TX fill and
// RX + L4, so the frame calls keep quarters.
bool frames_quarters() {
    static const bool q = [] {
        const char* e = getenv("LVLIP_FRAMES_GROUPS");
        return !(e && strcmp(e, "block") == 0);
    }();
    return q;
}

// LVLIP_FRAMES_RX_HDR (A/B knob, read per call so one process can time and
// test both): the header-only RX call's kernel, lane (default: k_rx_hdr, one
// lane per frame) | flat (k_flat2 with a frame source, as the other frame
// calls).
bool frames_rx_lane() {
    const char* e = getenv("LVLIP_FRAMES_RX_HDR");
    return !(e && strcmp(e, "flat") == 0);
}

// LVLIP_FRAMES_TX_STORE (A/B knob, read per call): the TX call's field stores,
// nt (default: nontemporal, 0.382 vs 0.414 ms on 2M frames) |
// plain.
bool frames_tx_nt() {
    const char* e = getenv("LVLIP_FRAMES_TX_STORE");
    return !(e && strcmp(e, "plain") == 0);
}

int launch_rx_hdr(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* out8,
                  hipStream_t s) {
    for (uint32_t f0 = 0; f0 < n;) {
        const uint32_t m = n - f0 < kLaunchMax ? n - f0 : kLaunchMax;
        hipLaunchKernelGGL(lvlip::k_rx_hdr, dim3((m + 255u) / 256u), dim3(256), 0, s,
                           (const uint8_t*)base, frames + f0, m, out8 + f0);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_rx_hdr");
        f0 += m;
    }
    return LVLIP_OK;
}

template <int MODE>
int launch_frames(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* out8,
                  hipStream_t s) {
    if (MODE == lvlip::FR_RX && frames_rx_lane()) return launch_rx_hdr(base, frames, n, out8, s);
    using Src = lvlip::FrameSrc<MODE>;
    // a dispatch holds at most 2^30 entries (kLaunchMax): whole frames per launch
    const uint32_t per = kLaunchMax / Src::SLOTS;
    for (uint32_t f0 = 0; f0 < n;) {
        const uint32_t m = n - f0 < per ? n - f0 : per;
        const uint32_t entries = m * Src::SLOTS;
        const uint32_t grid = (uint32_t)(((uint64_t)entries + lvlip::FT - 1) / lvlip::FT);
        Src src{(const uint8_t*)base, (uint8_t*)base, frames + f0, out8 ? out8 + f0 : nullptr};
        src.nt_store = frames_tx_nt();
        const bool quarters = frames_quarters();
#define LVLIP_FRAMES_K(UU, GO)                                                              \
    hipLaunchKernelGGL((lvlip::k_flat2<UU, true, GO, Src>), dim3(grid), dim3(lvlip::FT), 0, s, \
                       (const uint8_t*)base, src, entries)
        if (frames_unroll() == 8) {
            if (quarters) LVLIP_FRAMES_K(8, 1); else LVLIP_FRAMES_K(8, 2);
        } else {
            if (quarters) LVLIP_FRAMES_K(4, 1); else LVLIP_FRAMES_K(4, 2);
        }
#undef LVLIP_FRAMES_K
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_flat2 (frames)");
        f0 += m;
    }
    return LVLIP_OK;
}

}  // namespace

// Shared with skb_dev.hip (hidden: -fvisibility=hidden keeps it internal): f1/f2
// on device-resident frames as one fused flat-sweep launch (flat_src.h).
// mode: 0 TX fill (out8 = status, may be null), 1 RX header verify, 2 RX with
// L4 (out8 = verdict).
int lvlip_internal_frames(int mode, const void* base, const lvlip_frame_desc* frames, uint32_t n,
                          uint8_t* out8, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
        case lvlip::FR_TX: return launch_frames<lvlip::FR_TX>(base, frames, n, out8, s);
        case lvlip::FR_RX: return launch_frames<lvlip::FR_RX>(base, frames, n, out8, s);
        case lvlip::FR_RX_L4: return launch_frames<lvlip::FR_RX_L4>(base, frames, n, out8, s);
        default: return LVLIP_EINVAL;
    }
}
