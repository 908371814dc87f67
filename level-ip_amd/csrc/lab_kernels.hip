// lab_kernels.hip — the A/B kernels of DESIGN.md §4, §8, §9 (liblvlip_lab.so,
// diagnostics; the product library does not contain them).
//
//   k_stream       the ring of k_window with contiguous per-wave ranges
//                  (LVLIP_KERNEL_WAVE = 1), in five load policies
//   k_wave_simple  one wave per packet, one launch wave each (4)
//   k_wave_lds     the same with LDS-DMA staging (2)
//   k_flat         the first flat kernel: binary search, ds_bpermute
//                  segmented scan (5)
//   k_wflat        k_flat2's sweep one wave per tile, tiles dealt round robin (9)
//   k_rflat        the same with a ring of group loads across tiles (11;
//                  round 3, DESIGN.md §4: instruction-bound, 4.0 vs 6.2 TB/s)
//   k_wsflat       k_flat2's sweep in persistent workgroups of 4 sweeper
//                  waves + 1 planner wave, tiles double-buffered (12)
//   k_flat2_occ    k_flat2 compiled for a set number of waves per SIMD (13)
//   k_flat2        its other shapes (3): group orders, tiles of 512, temporal
//                  loads, U 6 / 12, an LDS pad; and the frame calls' variants
//                  (8 loads per round, block order, plain field stores, the
//                  flat sweep for the header-only RX call)
//
// Entry points (C ABI, used by bench.py --sweep and scripts/ through
// lvlip.py): lvlip_lab_batch_dev_ex takes the kernel ids above with
// lvlip_launch_cfg's encodings; lvlip_lab_frames_dev the frame-call variants.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "csum_dev.h"

namespace lvlip {

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

// POL: the data loads' cache policy (A/B, LVLIP_LOAD_POLICY)
template <int R, int POL = 0>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ base,
                                                const lvlip_csum_desc* __restrict__ descs,
                                                uint32_t n, uint16_t* __restrict__ out) {
    __shared__ uint4 s_win[SW_WAVES][2][64];
    ring_sweep<R, 0, POL>(base, descs, n, out, s_win[uniform(threadIdx.x >> 6)]);
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
    // ahead (lanes past the batch re-read its last descriptor).  A
    // compiler-visible load (an asm load here left the compiler
    // free to copy its destination register before the data arrived); the
    // compiler's own wait retires it before the next tile's plan.
    auto fetch = [&](uint64_t t, u32x4& d) {
        uint64_t i = t * D + (lane < (uint32_t)D ? lane : 0u);
        i = i < n ? i : n - 1u;
        const uint4 v = load_global(reinterpret_cast<uint64_t>(descs + i));
        d = u32x4{v.x, v.y, v.z, v.w};
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

// ------------------------------------------------ k_rflat (ragged, ring) --
//
// k_flat2's chunk sweep (csum_dev.h) with k_window's two remedies for the
// mixed config's gap to the memory system:
//   * a narrow window: tiles of D descriptors (~6 KB of a mixed batch at
//     D = 16) dealt round robin over the persistent waves (XCD-major ranks),
//     so the waves in flight read one window of nw x D descriptors that slides
//     through the batch, instead of ~1 300 resident workgroups each sweeping
//     its own ~100 KB tile;
//   * a ring across tiles: every wave keeps two rounds of U 1-KiB group loads
//     in flight (round k+1 is issued before round k is reduced), and a tile's
//     plan (one wave-level scan, records and head bitmaps in the wave's LDS)
//     is made while the previous tile's loads are in flight.  k_wflat, the
//     window deal without the ring, drained every round and every tile (8
//     waves/CU read 3.5 TB/s there).
// One wave owns its tiles end to end: no workgroup barrier anywhere.
//
// Per wave, RF_NB tile buffers in LDS (a tile is planned into buffer s % NB,
// s = the wave's tile sequence number) hold records by rank {a0 lo, a0 hi,
// cstart, meta}, the head bitmap per 64-chunk group, the per-descriptor
// accumulators and edge chunks (as k_flat2) and the phase-4 words; a tile is
// finished (edge corrections, fold, one 2-B store per descriptor) when the
// consume side reduces its last group.  The issue side never runs more than
// NB tiles ahead of the finished ones (it issues placeholder loads instead).
// Descriptors come two tiles ahead by LDS-DMA (no VGPR is written behind the
// compiler's back, cf. k_wflat).
//
// Wait-count discipline (as k_window's ring, tests/test_isa.py): the group
// loads, the descriptor DMA are inline asm, one vm operation each, counted in
// `nvm`; group (k, u) is retired by vmcnt(2U - 1 - u), the U - 1 - u later
// loads of its round plus the U of the next round being issued after it (the
// DMAs and result stores in between only make the wait stricter); a plan
// retires its DMA with vmcnt(vm operations issued since it), exact.
constexpr uint32_t RF_NB = 4;             // tile buffers per wave
constexpr uint32_t RF_INV = 0xffffffffu;  // kk of a lane with no chunk

template <int D>
struct RflatTile {
    uint4 rec[D];              // by rank: {a0 lo, a0 hi, cstart, meta}
    uint2 msk[D * FCAP / 64];  // head bitmap per 64-chunk group
    uint32_t acc[D];           // by descriptor
    uint4 edge[2 * D];         // by descriptor: raw first / last chunk
    uint2 fin[D];              // by descriptor: {start_sum, phase-4 word}
    uint2 info;                // {groups, chunks} of the tile
};

template <int D>
struct RflatLds {
    RflatTile<D> t[SW_WAVES][RF_NB];
    uint4 pfd[SW_WAVES][2][64];  // descriptors of the next tiles (LDS-DMA)
};

// s_waitcnt vmcnt(n) for a run-time n (0..23; larger n waits for 23, which
// is stricter): the plan's wait for its descriptor DMA.
__device__ __forceinline__ void wait_vm_dyn(uint32_t n) {
    switch (n < 23u ? n : 23u) {
#define LVLIP_VMW(K) \
    case K: asm volatile("s_waitcnt vmcnt(" #K ")" ::: "memory"); break;
        LVLIP_VMW(0) LVLIP_VMW(1) LVLIP_VMW(2) LVLIP_VMW(3) LVLIP_VMW(4) LVLIP_VMW(5)
        LVLIP_VMW(6) LVLIP_VMW(7) LVLIP_VMW(8) LVLIP_VMW(9) LVLIP_VMW(10) LVLIP_VMW(11)
        LVLIP_VMW(12) LVLIP_VMW(13) LVLIP_VMW(14) LVLIP_VMW(15) LVLIP_VMW(16) LVLIP_VMW(17)
        LVLIP_VMW(18) LVLIP_VMW(19) LVLIP_VMW(20) LVLIP_VMW(21) LVLIP_VMW(22)
        default: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
#undef LVLIP_VMW
    }
}

template <int U, int D>
__global__ __launch_bounds__(256) void k_rflat(const uint8_t* __restrict__ base,
                                               const lvlip_csum_desc* __restrict__ descs, uint32_t n,
                                               uint16_t* __restrict__ out) {
    static_assert(D == 16 || D == 32 || D == 64, "descriptors per tile");
    static_assert(U >= 2 && 2 * U + 2 <= 23, "group loads per round");
    __shared__ RflatLds<D> L;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * SW_WAVES;
    const uint64_t rank =
        (gridDim.x & 7u) == 0u
            ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * SW_WAVES + wid
            : (uint64_t)blockIdx.x * SW_WAVES + wid;
    const uint64_t ntiles = ((uint64_t)n + D - 1) / D;
    if (rank >= ntiles) return;  // uniform: this wave has no tile
    // the wave's tiles: rank, rank + nw, ...; count
    const uint32_t my_tiles = (uint32_t)((ntiles - 1 - rank) / nw + 1);
    RflatTile<D>* T = L.t[wid];
    const uint64_t safe = reinterpret_cast<uint64_t>(descs);  // a readable 16-B address

    uint32_t nvm = 0;     // vm operations this wave issued from asm (loads, DMAs)
    uint32_t pf_at[2];    // nvm when the DMA for the tile of parity p was issued

    // descriptors of the wave's tile s into pfd[s & 1], one per lane (lanes
    // past the tile or the batch re-read a valid descriptor)
    auto prefetch = [&](uint32_t s) {
        const uint64_t t = rank + (uint64_t)s * nw;
        uint64_t i = t * D + (lane < (uint32_t)D ? lane : 0u);
        i = i < n ? i : n - 1u;
        const lvlip_csum_desc* g = descs + i;
        const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)L.pfd[wid][s & 1u]);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     :
                     : "v"(g), "s"(lds)
                     : "memory", "m0");
#pragma clang diagnostic pop
        pf_at[s & 1u] = nvm;
        ++nvm;
    };

    // ---- issue side.  Tiles are planned ahead of the group loads so that a
    // round's U groups never wait for a plan: s_plan = next tile to plan,
    // s_iss = the tile whose groups are being issued (cur_g of cur_ng issued),
    // ahead = planned groups not issued yet.
    uint32_t s_plan = 0, s_iss = 0;
    uint32_t cur_b = 0, cur_g = 0, cur_ng = 0, cur_C = 0;
    uint32_t ahead = 0;
    uint32_t heads = 0;     // heads in the issue tile's earlier groups
    uint32_t fin_count = 0; // tiles finished (consume side)

    // plan of tile s into buffer s % NB: records, head bitmaps, accumulators,
    // phase-4 words, {groups, chunks}; the DMA for tile s + 2 goes out behind it
    auto plan = [&](uint32_t s) {
        wait_vm_dyn(nvm - pf_at[s & 1u] - 1u);  // vm ops issued after this tile's DMA
        const uint4 dv = L.pfd[wid][s & 1u][lane];
        RflatTile<D>& B = T[s % RF_NB];
        const uint64_t t = rank + (uint64_t)s * nw;
        const uint64_t i = t * D + lane;
        const bool mine = lane < (uint32_t)D && i < n;
        uint32_t start_sum = 0, nch = 0, meta = 0, fw = 0;
        uint64_t a0 = 0;
        if (mine) {
            const int32_t len = (int32_t)dv.z;
            start_sum = dv.w;
            fw = 1u << 21;
            if (len > 0) {
                const uint64_t abs = reinterpret_cast<uint64_t>(base) + (((uint64_t)dv.y << 32) | dv.x);
                a0 = abs & ~15ull;
                const uint32_t lo = (uint32_t)(abs & 15ull);
                const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)len;
                const uint64_t c64 = (span + 15u) >> 4;
                const uint32_t lastv = (uint32_t)(span - 16ull * (c64 - 1u));  // 1..16
                const bool big = c64 > FCAP;
                nch = big ? 0u : (uint32_t)c64;
                const bool odd = abs & 1ull;
                const bool ef = !big && (lo != 0u || (c64 == 1u && lastv != 16u));
                const bool el = !big && c64 > 1u && lastv != 16u;
                meta = nch | ((uint32_t)odd << 9) | ((uint32_t)ef << 10) | ((uint32_t)el << 11) | (lane << 18);
                fw |= lo | (lastv << 4) | (nch << 9) | ((uint32_t)odd << 17) | ((uint32_t)ef << 18) |
                      ((uint32_t)el << 19) | ((uint32_t)big << 20);
            }
        }
        const uint32_t incl = wave_incl_scan(nch);
        const uint32_t C = uniform((uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
        const uint32_t cstart = incl - nch;
        const uint64_t nz = __builtin_amdgcn_ballot_w64(nch != 0u);
        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u));
        const uint32_t ng = C ? (C + 63u) >> 6 : 1u;  // a tile with no chunk still takes one group
        for (uint32_t q = lane; q < ng; q += 64u) B.msk[q] = make_uint2(0u, 0u);
        if (lane < (uint32_t)D) {
            B.acc[lane] = 0u;
            B.fin[lane] = make_uint2(start_sum, fw);
        }
        if (lane == 0u) B.info = make_uint2(ng, C);
        __builtin_amdgcn_wave_barrier();
        if (nch) {
            B.rec[r] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), cstart, meta);
            const uint32_t q = cstart >> 6, b = cstart & 63u;
            if (b < 32u) atomicOr(&B.msk[q].x, 1u << b);
            else atomicOr(&B.msk[q].y, 1u << (b - 32u));
        }
        if (s + 2u < my_tiles) prefetch(s + 2u);  // its LDS slot was read above
        ahead += ng;
    };

    // finish of the wave's tile fs in buffer fs % NB: the big descriptors, edge
    // corrections, fold and store (src/utils.c:46-54)
    auto finish_tile = [&](uint32_t fs) {
        RflatTile<D>& B = T[fs % RF_NB];
        lds_sync();  // this tile's accumulator atomics and edge stashes
        const uint64_t t = rank + (uint64_t)fs * nw;
        const uint2 f = B.fin[lane < (uint32_t)D ? lane : 0u];
        const uint32_t fw = lane < (uint32_t)D ? f.y : 0u;
        uint64_t bigm = __builtin_amdgcn_ballot_w64((fw >> 20) & 1u);
        if (bigm) {
            while (bigm) {  // descriptors longer than FCAP chunks: one wave each
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
                if (lane == 0) B.acc[q] = w;
            }
            lds_sync();
        }
        uint32_t acc = B.acc[lane < (uint32_t)D ? lane : 0u];
        if (fw & (3u << 18)) {
            const bool odd = fw & (1u << 17);
            const int lo = (int)(fw & 15u), lastv = (int)((fw >> 4) & 31u);
            const uint32_t nch = (fw >> 9) & 0xffu;
            uint32_t c = 0;
            if (fw & (1u << 18)) {
                uint4 e = B.edge[2u * lane];
                const int fb1 = (nch == 1u) ? lastv : 16;
                e.x &= ~byte_range_mask(lo, fb1, 0);
                e.y &= ~byte_range_mask(lo, fb1, 1);
                e.z &= ~byte_range_mask(lo, fb1, 2);
                e.w &= ~byte_range_mask(lo, fb1, 3);
                c += odd ? chunk_words<true>(e) : chunk_words<false>(e);
            }
            if (fw & (1u << 19)) {
                uint4 e = B.edge[2u * lane + 1u];
                e.x &= ~byte_range_mask(0, lastv, 0);
                e.y &= ~byte_range_mask(0, lastv, 1);
                e.z &= ~byte_range_mask(0, lastv, 2);
                e.w &= ~byte_range_mask(0, lastv, 3);
                c += odd ? chunk_words<true>(e) : chunk_words<false>(e);
            }
            acc -= c;
        }
        if (fw & (1u << 21)) out[t * D + lane] = finish(f.x, acc);
        ++fin_count;
    };

    // Two banks of U group slots; bank X holds one round.  Per slot: the loaded
    // chunk, the lane's chunk index in its packet (RF_INV: none), the packet's
    // meta word, and a uniform flag word: 1 valid | 2 last group of its tile |
    // buffer << 2.
    u32x4 xa[U], xb[U];
    uint32_t ka[U], kb[U], ma[U], mb[U], fa[U], fb[U];

    auto issue_round = [&](u32x4* x, uint32_t* kk, uint32_t* mt, uint32_t* fl) {
        // plan until the round's U groups are planned (or no tile / buffer is left)
#pragma unroll 1
        while (ahead < (uint32_t)U && s_plan < my_tiles && s_plan < fin_count + RF_NB) {
            plan(s_plan);
            ++s_plan;
        }
        uint32_t sb[U], sg[U], sC[U];
        bool sv[U], sfirst[U], slast[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (cur_g == cur_ng && s_iss < s_plan) {  // the next planned tile
                cur_b = s_iss % RF_NB;
                const uint2 info = T[cur_b].info;
                cur_ng = uniform(info.x);
                cur_C = uniform(info.y);
                cur_g = 0;
                ++s_iss;
            }
            sv[u] = cur_g < cur_ng;
            sb[u] = cur_b;
            sg[u] = cur_g;
            sC[u] = cur_C;
            sfirst[u] = sv[u] && cur_g == 0u;
            slast[u] = sv[u] && cur_g + 1u == cur_ng;
            if (sv[u]) {
                ++cur_g;
                --ahead;
            }
        }
        uint32_t hlo[U], hhi[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint2 h = T[sb[u]].msk[sv[u] ? sg[u] : 0u];
            hlo[u] = sv[u] ? uniform(h.x) : 0u;
            hhi[u] = sv[u] ? uniform(h.y) : 0u;
        }
        uint4 rec[U];
        bool vl[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (sfirst[u]) heads = 0;
            const uint64_t H = ((uint64_t)hhi[u] << 32) | hlo[u];
            const uint64_t Hs = H >> 1;
            const uint32_t cnt = __builtin_amdgcn_mbcnt_hi((uint32_t)(Hs >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)Hs, 0u));
            const uint32_t rk = heads + (uint32_t)(H & 1ull) + cnt - 1u;
            heads += (uint32_t)__popcll(H);
            const uint32_t c = sg[u] * 64u + lane;
            vl[u] = sv[u] && c < sC[u];
            rec[u] = T[sb[u]].rec[vl[u] ? rk : 0u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = sg[u] * 64u + lane;
            kk[u] = vl[u] ? c - rec[u].z : RF_INV;
            const uint64_t ca = vl[u] ? (((uint64_t)rec[u].y << 32) | rec[u].x) + 16ull * (c - rec[u].z) : safe;
            x[u] = group_load_nt(ca);
            mt[u] = vl[u] ? rec[u].w : 0u;
            fl[u] = (uint32_t)sv[u] | ((uint32_t)slast[u] << 1) | (sb[u] << 2);
        }
        nvm += U;
    };

    auto consume_round = [&](u32x4* x, const uint32_t* kk, const uint32_t* mt, const uint32_t* fl) {
        uint32_t nfin = 0;  // tiles whose last group this round reduced
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // 2U - 1 - u later group loads were issued: this round's rest and
            // the next round
            switch (u) {
                case 0: group_wait<2 * U - 1>(x[u]); break;
                case 1: group_wait<2 * U - 2>(x[u]); break;
                case 2: group_wait<2 * U - 3>(x[u]); break;
                case 3: group_wait<2 * U - 4>(x[u]); break;
                case 4: group_wait<2 * U - 5>(x[u]); break;
                case 5: group_wait<2 * U - 6>(x[u]); break;
                case 6: group_wait<2 * U - 7>(x[u]); break;
                default: group_wait<2 * U - 8>(x[u]); break;
            }
            const uint32_t f = uniform(fl[u]);
            if (!(f & 1u)) continue;  // uniform: a placeholder
            RflatTile<D>& B = T[f >> 2];
            const u32x4 raw = x[u];
            uint4 v = make_uint4(raw.x, raw.y, raw.z, raw.w);
            const uint32_t m = mt[u];
            const bool vlu = kk[u] != RF_INV;
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
            val = vlu ? val : 0u;
            const uint32_t P = wave_incl_scan(val);
            const bool first = kk[u] == 0u;
            const bool last = vlu && kk[u] + 1u == (m & 0xFFu);
            const uint32_t add = (first ? val - P : 0u) + ((last || lane == 63u) ? P : 0u);
            const uint32_t slot = (m >> 18) & 63u;
            if (vlu && (first || last || lane == 63u)) atomicAdd(&B.acc[slot], add);
            if (vlu && first && (m & (1u << 10))) B.edge[2u * slot] = make_uint4(raw.x, raw.y, raw.z, raw.w);
            if (vlu && last && (m & (1u << 11))) B.edge[2u * slot + 1u] = make_uint4(raw.x, raw.y, raw.z, raw.w);
            nfin += (f >> 1) & 1u;
        }
#pragma unroll 1
        for (; nfin; --nfin) finish_tile(fin_count);
    };

    prefetch(0);
    if (my_tiles > 1u) prefetch(1);
    issue_round(xa, ka, ma, fa);
    for (;;) {
        issue_round(xb, kb, mb, fb);
        consume_round(xa, ka, ma, fa);
        if (fin_count == my_tiles) break;
        issue_round(xa, ka, ma, fa);
        consume_round(xb, kb, mb, fb);
        if (fin_count == my_tiles) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of this wave left in flight
}


// ------------------------------------ k_wsflat (warp-specialized, lab 12) --
//
// k_flat2's tile with its planning taken off the sweep's critical path.  A
// workgroup is WS_SW sweeper waves and one planner wave, persistent (a few per
// CU), its tiles dealt round robin over the workgroups (XCD-major ranks) so the
// resident workgroups read one window of the batch.  Two tile buffers in LDS:
// while the sweepers sweep tile k (buffer k & 1, k_flat2's phase 2 unchanged),
// the planner finishes tile k - 1 (phase 3 + 4: big packets, edge corrections,
// fold, stores) and plans tile k + 1 (phase 1, one wave-level scan per 64
// descriptors) into the other buffer; one workgroup barrier per tile hands the
// buffers over.  The descriptors of tile k + 1 are loaded at the start of the
// planner's iteration, so their latency hides behind the finish of tile k - 1.
// The sweepers see no phase-1/phase-4 bubbles and no per-tile launch; the
// question this kernel answers is whether k_flat2's gap on
// mixed is those bubbles or its access order.
constexpr int WS_SW = 4;  // sweeper waves per workgroup

template <int TD>
struct WsBuf {
    static constexpr uint32_t FG = (uint32_t)TD * FCAP / 64;
    uint4 rec[TD];       // by rank: {a0 lo, a0 hi, cstart, meta} (k_flat2's meta)
    uint4 edge[2 * TD];  // by descriptor: raw first / last chunk
    uint2 grp[FG];       // by 64-chunk group: head bitmap
    uint2 fin[TD];       // by descriptor: {start_sum, nch | odd 9 | ef 10 | el 11 | lo << 12 | lastv << 16}
    uint32_t acc[TD];    // by descriptor
    uint32_t big[TD];    // descriptors longer than FCAP chunks
    uint16_t hb[FG];     // by 64-chunk group: heads before it
    uint32_t C, nbig;
};

template <int U, int TD, int GORD>
__global__ __launch_bounds__((WS_SW + 1) * 64) void k_wsflat(const uint8_t* __restrict__ base,
                                                             const lvlip_csum_desc* __restrict__ descs,
                                                             uint32_t n, uint16_t* __restrict__ out) {
    static_assert(TD == 64 || TD == 128 || TD == 256, "descriptors per tile");
    constexpr uint32_t NP = TD / 64;  // planner passes per tile
    constexpr uint32_t FG = WsBuf<TD>::FG;
    __shared__ WsBuf<TD> B[2];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    const bool planner = wid == (uint32_t)WS_SW;
    const uint32_t nwg = gridDim.x;
    const uint32_t rank = (nwg & 7u) == 0u ? (blockIdx.x & 7u) * (nwg >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t ntiles = (uint32_t)(((uint64_t)n + TD - 1) / TD);
    if (rank >= ntiles) return;  // workgroup-uniform
    const uint32_t K = (ntiles - 1u - rank) / nwg + 1u;

    uint4 pf[NP];  // planner: the descriptors of the tile it plans next
    auto prefetch = [&](uint32_t k) {
        const uint64_t t0 = (uint64_t)(rank + k * nwg) * TD;
#pragma unroll
        for (uint32_t p = 0; p < NP; ++p) {
            const uint64_t i = t0 + p * 64u + lane;
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(1))) const v4u gv4u;
            v4u v = {0u, 0u, 0u, 0u};
            if (i < n) v = *reinterpret_cast<gv4u*>(reinterpret_cast<uint64_t>(descs + i));
            pf[p] = make_uint4(v.x, v.y, v.z, v.w);
        }
    };
    auto plan = [&](uint32_t k, WsBuf<TD>& b) {
        const uint64_t t0 = (uint64_t)(rank + k * nwg) * TD;
        for (uint32_t g = lane; g < FG; g += 64u) b.grp[g] = make_uint2(0u, 0u);
        lds_sync();
        uint32_t rk = 0, cc = 0, nb = 0;
#pragma unroll
        for (uint32_t p = 0; p < NP; ++p) {
            const uint32_t j = p * 64u + lane;
            const uint64_t i = t0 + j;
            uint32_t nch = 0, meta = 0, fw = 0, start_sum = 0;
            uint64_t a0 = 0;
            bool big = false;
            if (i < n) {
                const uint64_t off = ((uint64_t)pf[p].y << 32) | pf[p].x;
                const uint32_t len = pf[p].z;
                start_sum = pf[p].w;
                if ((int32_t)len > 0) {
                    const uint64_t abs = reinterpret_cast<uint64_t>(base) + off;
                    const bool odd = abs & 1ull;
                    const uint32_t lo = (uint32_t)(abs & 15ull);
                    const uint64_t span = (uint64_t)lo + len;
                    const uint64_t c64 = (span + 15u) >> 4;
                    const uint32_t lastv = (uint32_t)(span - 16ull * (c64 - 1u));
                    big = c64 > FCAP;
                    a0 = abs & ~15ull;
                    nch = big ? 0u : (uint32_t)c64;
                    const bool ef = !big && (lo != 0u || (c64 == 1u && lastv != 16u));
                    const bool el = !big && c64 > 1u && lastv != 16u;
                    const uint32_t fl = ((uint32_t)odd << 9) | ((uint32_t)ef << 10) | ((uint32_t)el << 11);
                    meta = nch | fl | (j << 18);
                    fw = nch | fl | (lo << 12) | (lastv << 16);
                }
            }
            b.acc[j] = 0u;
            b.fin[j] = make_uint2(start_sum, fw);
            const uint32_t sa = (big ? 0x10000u : 0u) | (nch ? 1u : 0u);
            const uint32_t ia = wave_incl_scan(sa), ib = wave_incl_scan(nch);
            const uint32_t e1 = rk + ((ia - sa) & 0xffffu), cs = cc + ib - nch;
            const uint32_t bp = nb + ((ia - sa) >> 16);
            if (big) b.big[bp] = j;
            if (nch) {
                b.rec[e1] = make_uint4((uint32_t)a0, (uint32_t)(a0 >> 32), cs, meta);
                const uint32_t g = cs >> 6, bit = cs & 63u;
                if (bit < 32u) atomicOr(&b.grp[g].x, 1u << bit);
                else atomicOr(&b.grp[g].y, 1u << (bit - 32u));
                for (uint32_t gg = g + 1u; gg < FG && (gg << 6) <= cs + nch; ++gg) b.hb[gg] = (uint16_t)(e1 + 1u);
            }
            const uint32_t ta = uniform(__builtin_amdgcn_readlane(ia, 63)), tb = uniform(__builtin_amdgcn_readlane(ib, 63));
            rk += ta & 0xffffu;
            nb += ta >> 16;
            cc += tb;
        }
        if (lane == 0u) {
            b.hb[0] = 0;
            b.C = cc;
            b.nbig = nb;
        }
    };
    auto finish_tile = [&](uint32_t k, WsBuf<TD>& b) {
        const uint64_t t0 = (uint64_t)(rank + k * nwg) * TD;
        const uint32_t nbig = uniform(b.nbig);
        for (uint32_t q = 0; q < nbig; ++q) {
            const uint32_t tq = uniform(b.big[q]);
            const lvlip_csum_desc d = descs[t0 + tq];
            const uint64_t abs = reinterpret_cast<uint64_t>(base) + d.offset;
            const int lo = (int)(abs & 15ull);
            const uint64_t span = (uint64_t)lo + (uint64_t)(uint32_t)d.len;
            const uint32_t nchq = (uint32_t)((span + 15u) >> 4);
            const uint32_t lastv = (uint32_t)(span - 16ull * (nchq - 1u));
            const uint4* src = reinterpret_cast<const uint4*>(abs & ~15ull);
            uint32_t w = (abs & 1ull) ? wave_packet_sum<4, true>(src, nchq, lo, lastv, lane)
                                      : wave_packet_sum<4, false>(src, nchq, lo, lastv, lane);
            w = wave_sum_dpp(w);
            if (lane == 0) b.acc[tq] = w;
        }
        lds_sync();
#pragma unroll
        for (uint32_t p = 0; p < NP; ++p) {
            const uint32_t j = p * 64u + lane;
            const uint64_t i = t0 + j;
            if (i < n) {
                uint32_t acc = b.acc[j];
                const uint2 f = b.fin[j];
                const uint32_t m = f.y;
                if (m & (3u << 10)) {
                    const bool odd = m & (1u << 9);
                    const int lo = (int)((m >> 12) & 15u), lastv = (int)(m >> 16);
                    uint32_t c = 0;
                    if (m & (1u << 10)) {
                        uint4 e = b.edge[2u * j];
                        const int fb1 = (m & 0xFFu) == 1u ? lastv : 16;
                        e.x &= ~byte_range_mask(lo, fb1, 0);
                        e.y &= ~byte_range_mask(lo, fb1, 1);
                        e.z &= ~byte_range_mask(lo, fb1, 2);
                        e.w &= ~byte_range_mask(lo, fb1, 3);
                        c += odd ? chunk_words<true>(e) : chunk_words<false>(e);
                    }
                    if (m & (1u << 11)) {
                        uint4 e = b.edge[2u * j + 1u];
                        e.x &= ~byte_range_mask(0, lastv, 0);
                        e.y &= ~byte_range_mask(0, lastv, 1);
                        e.z &= ~byte_range_mask(0, lastv, 2);
                        e.w &= ~byte_range_mask(0, lastv, 3);
                        c += odd ? chunk_words<true>(e) : chunk_words<false>(e);
                    }
                    acc -= c;
                }
                out[i] = finish(f.x, acc);
            }
        }
    };
    // k_flat2's phase 2 over buffer b, the WS_SW sweepers
    auto sweep = [&](WsBuf<TD>& b) {
        const uint32_t C = uniform(b.C);
        if (C == 0u) return;
        const uint32_t G = (C + 63u) >> 6;
        const uint32_t rstep = GORD == 1 ? (uint32_t)U : (uint32_t)WS_SW * U;
        const uint32_t gper = (G + WS_SW - 1u) / WS_SW;
        const uint32_t g_lo = GORD == 1 ? wid * gper : wid * (uint32_t)U;
        const uint32_t g_end = GORD == 1 ? (g_lo + gper < G ? g_lo + gper : G) : G;
        for (uint32_t gr = g_lo; gr < g_end; gr += rstep) {
            uint4 x[U], rec[U];
            uint32_t kk[U], hlo[U], hhi[U], hb[U];
            bool vl[U], gv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t g = gr + u;
                gv[u] = g < g_end;
                const uint32_t gc = gv[u] ? g : G - 1u;
                const uint2 gg = b.grp[gc];
                hlo[u] = uniform(gg.x);
                hhi[u] = uniform(gg.y);
                hb[u] = uniform((uint32_t)b.hb[gc]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t H = ((uint64_t)hhi[u] << 32) | hlo[u];
                const uint64_t Hs = H >> 1;
                const uint32_t cnt = __builtin_amdgcn_mbcnt_hi((uint32_t)(Hs >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)Hs, 0u));
                rec[u] = b.rec[(hb[u] + (uint32_t)(H & 1ull) - 1u) + cnt];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = (gr + u) * 64u + lane;
                vl[u] = gv[u] && j < C;
                kk[u] = vl[u] ? j - rec[u].z : 0u;
                x[u] = load_nt_global((((uint64_t)rec[u].y << 32) | rec[u].x) + 16ull * kk[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!gv[u]) break;  // uniform
                uint4 v = x[u];
                const uint32_t m = rec[u].w;
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
                if (vl[u] && (first || last || lane == 63u)) atomicAdd(&b.acc[m >> 18], add);
                if (vl[u] && first && (m & (1u << 10))) b.edge[2u * (m >> 18)] = x[u];
                if (vl[u] && last && (m & (1u << 11))) b.edge[2u * (m >> 18) + 1u] = x[u];
            }
        }
    };

    if (planner) {
        prefetch(0);
        plan(0, B[0]);
    }
    __syncthreads();
    for (uint32_t k = 0; k < K; ++k) {
        WsBuf<TD>& cur = B[k & 1u];
        WsBuf<TD>& oth = B[(k & 1u) ^ 1u];
        if (!planner) {
            sweep(cur);
        } else {
            if (k + 1u < K) prefetch(k + 1u);
            if (k >= 1u) finish_tile(k - 1u, oth);
            if (k + 1u < K) {
                lds_sync();
                plan(k + 1u, oth);
            }
        }
        __syncthreads();
    }
    if (planner) finish_tile(K - 1u, B[(K - 1u) & 1u]);
}


// ------------------------------------------- k_flat2 at a set occupancy (13) --
//
// The product's k_flat2 (U loads per round, block order) compiled for at
// least W waves per SIMD (amdgpu_waves_per_eu): U 8 takes 92 VGPRs, 5 waves
// per SIMD = 5 workgroups per CU; W 6 caps it at 80 (6 workgroups).  The same
// body (flat2_body), only the register budget differs.
template <int U, int W, bool FIN, int PFA = 0, int VAR = 0>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(W, 8))) void k_flat2_occ(
    const uint8_t* __restrict__ base, const DescSrc src, uint32_t n) {
    flat2_body<U, true, 2, DescSrc, 1, false, FIN, PFA, VAR>(base, src, n);
}

// ------------------------------------- k_flat2 over a run-dealt tile map (14) --
//
// The product's k_flat2 U 8 (descriptor prefetch 1 280 tiles ahead), with
// only the map from (block, tile slot) to descriptor changed.  The ~1 280
// resident workgroups each stream their own ~100 KB tile, so together they
// read a ~130 MB window of the batch at once; the window read probes are
// fastest on narrow windows (k_window).  Here a generation of
// NWG consecutive blocks shares a contiguous range of NWG x 256 descriptors,
// dealt in runs of K: run k of block w's tile is the (k NWG + pos(w))-th run
// of the generation, so workgroups that start together read neighbouring
// runs (a window of NWG x K descriptors per run step).  XG: pos groups the
// blocks of one XCD (block b runs on XCD b % 8) so that neighbouring runs,
// which share edge lines, meet in one L2.  The last, partial generation keeps
// the plain map.  A bijection on [0, n): results land where the product's do.
template <int NWG, int K, bool XG>
struct PermSrc {
    static constexpr bool WIN_SUM = false;
    static_assert(NWG % 8 == 0 && FT % K == 0, "generation of whole XCD groups, whole runs per tile");
    const lvlip_csum_desc* descs;
    uint16_t* out;
    uint32_t n;
    __device__ __forceinline__ uint32_t perm(uint32_t i) const {
        constexpr uint32_t GEN = (uint32_t)NWG * FT;  // descriptors per generation
        const uint32_t g = i / GEN;
        if ((uint64_t)(g + 1u) * GEN > n) return i;  // last, partial generation
        const uint32_t b = (i % GEN) / FT, j = i % FT;
        const uint32_t pos = XG ? (b % 8u) * (NWG / 8u) + b / 8u : b;
        return g * GEN + (j / K) * ((uint32_t)NWG * K) + pos * K + j % K;
    }
    __device__ __forceinline__ lvlip_csum_desc get(uint32_t i, uint32_t& ctx) const {
        return DescSrc{descs, out}.get(perm(i), ctx);
    }
    __device__ __forceinline__ void put(uint32_t i, uint16_t c, uint32_t, bool valid, uint64_t) const {
        if (valid) out[perm(i)] = c;
    }
    __device__ __forceinline__ const lvlip_csum_desc* desc_ptr(uint32_t i) const { return descs + perm(i); }
};

// -------------------------- k_window_dyn: the window deal, balanced in the CU --
//
// lab_tail.py's stamps show k_window's waves ending ~25 us apart on tcp1500,
// the same waves late in every launch, and the spread inside each CU (the
// waves sharing a CU end ~10 us apart whatever the workgroup shape).  Here one
// workgroup of WPB waves runs per CU and owns the groups of its WPB ranks of
// the window deal, item i = (j = i / WPB, r = i % WPB) -> group
// j * nw + bx * WPB + r (bx: XCD-major block order).  Each wave's first two
// descriptor windows take its static items (j < 2 * 64/G, r = wave), as
// k_window would; after that a wave claims one item per group from an LDS
// counter, for the window two ahead of the one it issues from.  Claims made at
// the same time are neighbouring items, so the read window stays as narrow as
// the static deal's, and a wave that runs fast claims more.  At the end every
// wave holds at most two windows of claimed items.
//
// The ring itself (pieces, waits, asm loads, metadata, reduction) is
// ring_sweep's; what changes is where a wave's k-th packet comes from:
// s_claim[(k / 64) & 3][(k % 64) / G] holds its item, and the wave's packet
// count grows as claims come back valid.  stamps (optional): t0/t1 per wave.
template <int R, int G, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_window_dyn(const uint8_t* __restrict__ base,
                                                         const lvlip_csum_desc* __restrict__ descs, uint32_t n,
                                                         uint16_t* __restrict__ out, uint64_t* __restrict__ stamps) {
    static_assert(G == 1 || G == 2 || G == 4, "groups tile a 64-packet window");
    constexpr uint32_t GPW = 64u / G;  // groups per descriptor window
    constexpr uint32_t END = 0xffffffffu;
    constexpr uint32_t PIECE = 2048u;
    constexpr uint32_t BAD = 0xffffffffu;
    __shared__ uint4 s_win_all[WPB][2][64];
    __shared__ uint32_t s_claim_all[WPB][4][GPW];
    __shared__ uint32_t s_ctr;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lane16 = lane * 16u;
    const uint32_t wid = uniform(threadIdx.x >> 6);
    uint4(*s_win)[64] = s_win_all[wid];
    uint32_t(*s_claim)[GPW] = s_claim_all[wid];
    const uint64_t nw = (uint64_t)gridDim.x * WPB;
    const uint64_t bx = (gridDim.x & 7u) == 0u ? (uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                                               : (uint64_t)blockIdx.x;
    const uint64_t ng = ((uint64_t)n + G - 1) / G;
    // packet index of item `it`'s packet `p` (0 .. G-1), or BAD
    auto item_pkt = [&](uint32_t it, uint32_t p) -> uint32_t {
        if (it == BAD) return BAD;
        const uint64_t g = (uint64_t)(it / WPB) * nw + bx * WPB + (it % WPB);
        const uint64_t k = g * G + p;
        return (g < ng && k < n) ? (uint32_t)k : BAD;
    };
    if (threadIdx.x == 0) s_ctr = 2u * GPW * WPB;
    // static items of windows 0 and 1: j = v * GPW + q, r = wid (2 GPW slots:
    // 128 for G = 1, so two passes of the wave's lanes)
    for (uint32_t q = lane; q < 2u * GPW; q += 64u) s_claim[q / GPW][q % GPW] = q * WPB + wid;
    __syncthreads();

    // packet of the wave's k (window v = k / 64 must have its claims in LDS)
    auto wave_pkt = [&](uint32_t k) -> uint32_t {
        return item_pkt(s_claim[(k >> 6) & 3u][(k & 63u) / G], k % G);
    };
    // cnt: the wave's packets known so far.  A window's claims are complete
    // before it is fetched; valid packets are a prefix (items only grow).
    uint32_t cnt = 0;
    bool open = true;  // every packet so far valid: later windows may add more
    auto extend = [&](uint32_t v) {  // window v's claims are in LDS
        if (!open) return;
        const uint32_t pk = wave_pkt(v * 64u + lane);
        // valid packets are a prefix of the window: count the leading ones
        const uint64_t ok = __builtin_amdgcn_ballot_w64(pk != BAD);
        const uint32_t c = ~ok == 0ull ? 64u : (uint32_t)__builtin_ctzll(~ok);
        cnt = v * 64u + c;
        open = c == 64u;
    };
    auto fetch = [&](uint32_t v) {  // descriptors of window v into s_win[v & 1]
        uint32_t k = v * 64u + lane;
        k = k < cnt ? k : (cnt ? cnt - 1u : 0u);
        uint32_t pk = cnt ? wave_pkt(k) : 0u;
        pk = pk == BAD ? 0u : pk;  // (never: k < cnt; keeps the DMA inside the array)
        const lvlip_csum_desc* g = descs + pk;
        uint4* win = s_win[v & 1u];
        const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)win);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     :
                     : "v"(g), "s"(lds)
                     : "memory", "m0");
#pragma clang diagnostic pop
    };
    extend(0);
    extend(1);
    if (cnt == 0) {
        if (stamps && lane == 0) {
            stamps[2 * (bx * WPB + wid)] = t_start;
            stamps[2 * (bx * WPB + wid) + 1] = __builtin_amdgcn_s_memrealtime();
        }
        return;
    }
    fetch(0);
    fetch(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    uint32_t m_x, m_y, m_z, m_t, m_s;
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

    uint32_t ip = 0, io = 0;
    u32x4 srd;
    uint32_t tinfo, start;
    auto pull = [&](uint32_t k) {
        srd.x = (uint32_t)__builtin_amdgcn_readlane((int)m_x, (int)k);
        srd.y = (uint32_t)__builtin_amdgcn_readlane((int)m_y, (int)k);
        srd.z = (uint32_t)__builtin_amdgcn_readlane((int)m_z, (int)k);
        srd.w = SRD_WORD3;
        tinfo = (uint32_t)__builtin_amdgcn_readlane((int)m_t, (int)k);
        start = (uint32_t)__builtin_amdgcn_readlane((int)m_s, (int)k);
    };
    pull(0);
    bool claiming = true;
    // one claim per group, for the window two ahead of packet ip's
    // (a slot not claimed is written BAD: the ring of four windows reuses slots)
    auto claim = [&]() {
        uint32_t it = BAD;
        if (lane == 0) {
            if (claiming) it = atomicAdd(&s_ctr, 1u);
            s_claim[((ip >> 6) + 2u) & 3u][(ip & 63u) / G] = it;
        }
        it = (uint32_t)__builtin_amdgcn_readfirstlane((int)it);
        if (item_pkt(it, 0) == BAD) claiming = false;  // every later item is past the pool
    };
    claim();  // group 0 of window 0 -> slot 0 of window 2

    uint32_t gc = 0;
    uint32_t res_w = 0, res_s = 0;
    uint32_t acc = 0;
    u32x4 va[R], vb[R];
    uint32_t s_pkt[R], s_start[R], s_meta[R];

    auto issue = [&](int r) {
        const bool live = ip < cnt;
        u32x4 sr = srd;
        if (!live) sr.z = 0;
        const uint32_t off = lane16 + io;
        va[r] = buffer_load_nt_asm<0>(off, sr);
        vb[r] = buffer_load_nt_asm<0>(off + 1024u, sr);
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
                        lds_sync();          // lane 0's claims for window ip/64 + 1
                        extend((ip >> 6) + 1u);
                        load_window_meta(ip >> 6);
                        fetch((ip >> 6) + 1u);
                    }
                    pull(ip & 63u);
                    if (ip % G == 0u) claim();
                }
            }
        }
    };

    auto consume = [&](int r) {
        piece_wait<2 * (R - 1)>(va[r], vb[r]);
        u32x4 x = va[r], y = vb[r];
        const uint32_t meta = s_meta[r];
        const uint32_t len3 = (meta >> 1) & 3u;
        if ((meta & 1u) && len3) {
            const uint32_t pos = meta >> 3;
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
                uint32_t tt = res_s + res_w;
                tt = (tt & 0xffffu) + (tt >> 16);
                tt = (tt & 0xffffu) + (tt >> 16);
                const uint32_t pk = lane <= k ? wave_pkt(gc + lane) : BAD;
                if (pk != BAD) out[pk] = (uint16_t)~tt;
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (stamps && lane == 0) {
        stamps[2 * (bx * WPB + wid)] = t_start;
        stamps[2 * (bx * WPB + wid) + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// ------------------------------------ k_window with per-wave time stamps --
//
// Diagnostic (lvlip_lab_window_stamps): the product's k_window body, each wave
// stamping the real-time counter (100 MHz) when it starts and when its ring has
// drained, into a buffer of its own (two u64 per wave rank, XCD-major ranks as
// the deal uses).  Shows the launch's ramp (spread of start times) and tail
// (spread of end times).  The stamps go nowhere else.
template <int R, int G, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_window_stamp(const uint8_t* __restrict__ base,
                                                           const lvlip_csum_desc* __restrict__ descs, uint32_t n,
                                                           uint16_t* __restrict__ out, uint64_t* __restrict__ stamps) {
    __shared__ uint4 s_win[WPB][2][64];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t wid = uniform(threadIdx.x >> 6);
    ring_sweep<R, G, 0, WPB>(base, descs, n, out, s_win[wid]);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t rank = (gridDim.x & 7u) == 0u
                              ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * WPB + wid
                              : (uint64_t)blockIdx.x * WPB + wid;
    if ((threadIdx.x & 63u) == 0u) {
        stamps[2 * rank] = t0;
        stamps[2 * rank + 1] = t1;
    }
}

template <int NWG, int K, bool XG>
__global__ __launch_bounds__(FT) void k_flat2_perm(const uint8_t* __restrict__ base, const PermSrc<NWG, K, XG> src,
                                                   uint32_t n) {
    flat2_body<8, true, 2, PermSrc<NWG, K, XG>, 1, false, false, 1280>(base, src, n);
}

}  // namespace lvlip

namespace {

uint32_t grid_for(uint32_t n, uint32_t packets_per_block, int waves_per_cu, int waves_per_block) {
    uint64_t blocks = ((uint64_t)n + packets_per_block - 1) / packets_per_block;
    if (waves_per_cu > 0) {
        const uint64_t cap = (uint64_t)lvlip_host::current_cus() * (uint64_t)waves_per_cu / waves_per_block;
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
    uint64_t waves = (uint64_t)lvlip_host::current_cus() * (uint64_t)waves_per_cu;
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

// k_wflat: waves_per_cu waves on every CU (fewer when the batch has fewer
// tiles); the grid stays a multiple of 8 blocks when it can (XCD-major ranks).
template <int U, int D>
void launch_wflat_ud(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    uint64_t waves = (uint64_t)lvlip_host::current_cus() * (uint64_t)waves_per_cu;
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

template <int U>
void launch_wave_lds(uint32_t grid, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    hipLaunchKernelGGL(lvlip::k_wave_lds<U>, dim3(grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

// k_rflat: waves_per_cu waves on every CU (fewer when the batch has fewer
// tiles); the grid stays a multiple of 8 blocks when it can (XCD-major ranks).
template <int U, int D>
void launch_rflat_ud(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    uint64_t waves = (uint64_t)lvlip_host::current_cus() * (uint64_t)waves_per_cu;
    const uint64_t nt = ((uint64_t)n + D - 1) / D;
    if (waves > nt) waves = nt;
    uint64_t grid = (waves + lvlip::SW_WAVES - 1) / lvlip::SW_WAVES;
    if (grid > 8) grid = grid & ~7ull;
    hipLaunchKernelGGL((lvlip::k_rflat<U, D>), dim3((uint32_t)grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

bool launch_rflat(int u, int tile, int waves_per_cu, hipStream_t s, const void* base,
                  const lvlip_csum_desc* d, uint32_t n, uint16_t* out) {
    switch (u * 1000 + tile) {
#define LVLIP_RF(UU, DD) \
    case UU * 1000 + DD: launch_rflat_ud<UU, DD>(waves_per_cu, s, base, d, n, out); return true;
        LVLIP_RF(2, 16) LVLIP_RF(4, 16) LVLIP_RF(6, 16) LVLIP_RF(8, 16)
        LVLIP_RF(2, 32) LVLIP_RF(4, 32) LVLIP_RF(6, 32) LVLIP_RF(8, 32)
        LVLIP_RF(4, 64) LVLIP_RF(8, 64)
#undef LVLIP_RF
        default: return false;
    }
}

// k_wsflat: wgs_per_cu persistent workgroups on every CU (fewer when the batch
// has fewer tiles), a multiple of 8 when it can (XCD-major ranks).
template <int U, int TD, int GORD>
void launch_wsflat_t(int wgs_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d, uint32_t n,
                     uint16_t* out) {
    uint64_t grid = (uint64_t)lvlip_host::current_cus() * (uint64_t)wgs_per_cu;
    const uint64_t nt = ((uint64_t)n + TD - 1) / TD;
    if (grid > nt) grid = nt;
    if (grid > 8) grid = grid & ~7ull;
    hipLaunchKernelGGL((lvlip::k_wsflat<U, TD, GORD>), dim3((uint32_t)grid), dim3((lvlip::WS_SW + 1) * 64), 0, s,
                       (const uint8_t*)base, d, n, out);
}

bool launch_wsflat(int u, int tile, int gord, int wgs_per_cu, hipStream_t s, const void* base,
                   const lvlip_csum_desc* d, uint32_t n, uint16_t* out) {
    switch ((u * 1000 + tile) * 4 + gord) {
#define LVLIP_WS(UU, TT, GG) \
    case (UU * 1000 + TT) * 4 + GG: launch_wsflat_t<UU, TT, GG>(wgs_per_cu, s, base, d, n, out); return true;
        LVLIP_WS(4, 64, 1) LVLIP_WS(4, 128, 1) LVLIP_WS(4, 256, 1)
        LVLIP_WS(8, 128, 1) LVLIP_WS(8, 256, 1) LVLIP_WS(8, 256, 2) LVLIP_WS(4, 256, 2)
        LVLIP_WS(2, 64, 1) LVLIP_WS(2, 128, 1)
#undef LVLIP_WS
        default: return false;
    }
}

}  // namespace
extern "C" __attribute__((visibility("default"))) int lvlip_lab_window_dyn(const void* base,
                                                                        const lvlip_csum_desc* descs, uint32_t n,
                                                                        uint16_t* out, uint64_t* stamps,
                                                                        uint64_t stamp_bytes, int wpb, int shape,
                                                                        void* stream);
namespace {

int lab_dispatch(const void* base, const lvlip_csum_desc* descs, uint32_t n, uint16_t* out, hipStream_t s,
                 const lvlip_launch_cfg* cfg) {
    const int kernel = cfg ? cfg->kernel : -1;
    int unroll = cfg ? cfg->unroll : 0;
    const int wpc = cfg ? cfg->waves_per_cu : 0;
    switch (kernel) {
        case 1: {  // k_stream: unroll = 2-KiB pieces in flight per wave
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
        case 9: {  // k_wflat: loads per round | descriptors per tile << 8
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
        case 4: {
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
        case 2: {
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
        case 3: {
            // k_flat2's A/B shapes: loads per round | group order + 1 << 8 (1
            // interleaved, 2 quarters, 3 blocks; 0 = LVLIP_FLAT_GROUPS, else
            // blocks) | 1 << 10 for tiles of 512 descriptors (U 4 or 8,
            // quarters or blocks) | 1 << 11 for the pipelined sweep (U 2, 4,
            // 6, 8; blocks); LVLIP_LOAD_POLICY=temporal for plain loads
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
            if (unroll < 0) unroll = 0;
            if ((unroll >> 12) != 0) return LVLIP_EINVAL;
            if ((unroll >> 11) & 1) {
                if ((unroll >> 8) & 7) return LVLIP_EINVAL;
                switch (unroll & 0xff) {
#define LVLIP_FLAT_PIPE(UU)                                                                        \
    case UU:                                                                                       \
        hipLaunchKernelGGL((lvlip::k_flat2<UU, true, 2, lvlip::DescSrc, 1, true>), dim3(grid),     \
                           dim3(lvlip::FT), 0, s, (const uint8_t*)base, lvlip::DescSrc{descs, out}, n); \
        break;
                    LVLIP_FLAT_PIPE(2) LVLIP_FLAT_PIPE(4) LVLIP_FLAT_PIPE(6) LVLIP_FLAT_PIPE(8)
#undef LVLIP_FLAT_PIPE
                    default: return LVLIP_EINVAL;
                }
                break;
            }
            const int uo = (unroll >> 8) & 3;
            const bool d2 = (unroll >> 10) & 1;
            unroll &= 0xFF;
            if (unroll <= 0) unroll = 8;
            const bool nt = load_nt();
            const int gord = uo ? uo - 1 : flat_group_order();
            if (d2) {
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
        case 11: {
            // unroll = 64-chunk group loads per round (low byte: 2, 4, 6, 8;
            // 0 = 4) | descriptors per tile << 8 (16, 32, 64; 0 = 16); 12
            // waves/CU by default
            if (unroll < 0 || (unroll >> 16) != 0) return LVLIP_EINVAL;
            int u = unroll & 0xff, tile = (unroll >> 8) & 0xff;
            if (u == 0) u = 4;
            if (tile == 0) tile = 16;
            if (!launch_rflat(u, tile, wpc > 0 ? wpc : 12, s, base, descs, n, out)) return LVLIP_EINVAL;
            break;
        }
        case 12: {
            // unroll = group loads per round (low byte: 2, 4, 8; 0 = 4) |
            // descriptors per tile / 64 << 8 (1, 2, 4; 0 = 4) | 1 << 12 for
            // block group order (else quarters); 2 workgroups/CU by default
            if (unroll < 0 || (unroll >> 13) != 0) return LVLIP_EINVAL;
            int u = unroll & 0xff, tile = ((unroll >> 8) & 0xf) * 64;
            if (u == 0) u = 4;
            if (tile == 0) tile = 256;
            const int gord = (unroll >> 12) & 1 ? 2 : 1;
            if (!launch_wsflat(u, tile, gord, wpc > 0 ? wpc : 2, s, base, descs, n, out)) return LVLIP_EINVAL;
            break;
        }
        case 13: {
            // k_flat2 at a set occupancy: unroll = loads per round (6, 8) |
            // waves per SIMD << 8 (5, 6, 7) | 1 << 12 for phase 4's words in
            // LDS; or U 8, 5 waves with the descriptors of the tile P x 640
            // ahead prefetched: 8 | 5 << 8 | P << 13 (P 1, 2, 4, 7); the
            // product's shape (P 2) with flat2_body's VAR bits Q (1 s_setprio
            // 2 around the sweep's load issue, 2 around phase 1, 4 the last
            // round dealt to all four waves, 8 no early exit from a round, 32 the
            // sweep's loads without the reduction: wrong results): ... | Q << 16
            if (unroll < 0 || (unroll >> 22) != 0) return LVLIP_EINVAL;
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
            switch (unroll) {
#define LVLIP_FPF(PP)                                                                            \
    case 8 | (5 << 8) | (PP << 13):                                                              \
        hipLaunchKernelGGL((lvlip::k_flat2_occ<8, 5, false, PP * 640>), dim3(grid), dim3(lvlip::FT), 0, s, \
                           (const uint8_t*)base, lvlip::DescSrc{descs, out}, n);                 \
        break;
                LVLIP_FPF(1) LVLIP_FPF(2) LVLIP_FPF(4) LVLIP_FPF(7)
#undef LVLIP_FPF
#define LVLIP_FPR(QQ)                                                                            \
    case 8 | (5 << 8) | (2 << 13) | (QQ << 16):                                                  \
        hipLaunchKernelGGL((lvlip::k_flat2_occ<8, 5, false, 1280, QQ>), dim3(grid), dim3(lvlip::FT), 0, s, \
                           (const uint8_t*)base, lvlip::DescSrc{descs, out}, n);                 \
        break;
                LVLIP_FPR(1) LVLIP_FPR(2) LVLIP_FPR(3) LVLIP_FPR(4) LVLIP_FPR(5) LVLIP_FPR(6) LVLIP_FPR(7) LVLIP_FPR(8) LVLIP_FPR(10) LVLIP_FPR(32)
#undef LVLIP_FPR
                // U 4 (small-packet batches): 8 waves per SIMD without the
                // prefetch (the product's U 4), 7 with it (4 more VGPRs)
                case 4 | (8 << 8):
                    hipLaunchKernelGGL((lvlip::k_flat2_occ<4, 8, false, 0>), dim3(grid), dim3(lvlip::FT), 0, s,
                                       (const uint8_t*)base, lvlip::DescSrc{descs, out}, n);
                    break;
                case 4 | (7 << 8) | (2 << 13):
                    hipLaunchKernelGGL((lvlip::k_flat2_occ<4, 7, false, 1280>), dim3(grid), dim3(lvlip::FT), 0,
                                       s, (const uint8_t*)base, lvlip::DescSrc{descs, out}, n);
                    break;
#define LVLIP_FOCC(UU, WW, FF)                                                                   \
    case UU | (WW << 8) | (FF << 12):                                                            \
        hipLaunchKernelGGL((lvlip::k_flat2_occ<UU, WW, FF>), dim3(grid), dim3(lvlip::FT), 0, s,  \
                           (const uint8_t*)base, lvlip::DescSrc{descs, out}, n);                 \
        break;
                LVLIP_FOCC(8, 5, 0) LVLIP_FOCC(8, 5, 1) LVLIP_FOCC(8, 6, 0) LVLIP_FOCC(8, 6, 1)
                LVLIP_FOCC(6, 7, 0) LVLIP_FOCC(6, 7, 1)
#undef LVLIP_FOCC
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case 14: {
            // k_flat2 U 8 over the run-dealt tile map: unroll = run length K
            // (8, 16, 32, 64) | generation / 640 blocks << 8 (1, 2, 4) | 1 << 12
            // to group each XCD's blocks
            if (unroll < 0 || (unroll >> 13) != 0) return LVLIP_EINVAL;
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
            switch (unroll) {
#define LVLIP_FPM(KK, GG, XX)                                                                          \
    case KK | (GG << 8) | (XX << 12):                                                                  \
        hipLaunchKernelGGL((lvlip::k_flat2_perm<GG * 640, KK, XX>), dim3(grid), dim3(lvlip::FT), 0, s,    \
                           (const uint8_t*)base, lvlip::PermSrc<GG * 640, KK, XX>{descs, out, n}, n);  \
        break;
                LVLIP_FPM(8, 2, 1) LVLIP_FPM(16, 2, 1) LVLIP_FPM(32, 2, 1) LVLIP_FPM(64, 2, 1)
                LVLIP_FPM(16, 2, 0) LVLIP_FPM(16, 1, 1) LVLIP_FPM(16, 4, 1) LVLIP_FPM(32, 1, 1)
#undef LVLIP_FPM
                default: return LVLIP_EINVAL;
            }
            break;
        }
        case 15: {
            // k_window_dyn: unroll = pieces in flight R (2) | packets per group G
            // << 8 (1, 2, 4); waves_per_cu = waves per workgroup (8, 12), one
            // workgroup per CU
            int r = unroll & 0xff, g = (unroll >> 8) & 0xff;
            if (r == 0) r = 2;
            if (g == 0) g = 4;
            const int w = wpc > 0 ? wpc : 12;
            if (lvlip_lab_window_dyn(base, descs, n, out, nullptr, 0, w, r | (g << 8), s) < 0) return LVLIP_EINVAL;
            break;
        }
        case 5: {  // first-generation flat kernel
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FLAT_T - 1) / lvlip::FLAT_T);
            hipLaunchKernelGGL(lvlip::k_flat, dim3(grid), dim3(lvlip::FLAT_T), 0, s, (const uint8_t*)base, descs,
                               n, out);
            break;
        }
        default: return LVLIP_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
}

}  // namespace

extern "C" {

// k_window R 2, G 4 (the MTU shape) at waves_per_cu waves on every CU, with
// per-wave start/end stamps (2 u64 per wave) into `stamps`; returns the number
// of waves (stamps needs 16 B each), or a negative LVLIP_E*.
// k_window_dyn, one workgroup of wpb (8 or 12) waves per CU; shape = R | G << 8
// (R 2; G 1, 2, 4); stamps (2 u64 per wave, XCD-major rank) or null.  Returns
// the number of waves, or a negative LVLIP_E*.
__attribute__((visibility("default"))) int lvlip_lab_window_dyn(const void* base, const lvlip_csum_desc* descs,
                                                                uint32_t n, uint16_t* out, uint64_t* stamps,
                                                                uint64_t stamp_bytes, int wpb, int shape,
                                                                void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !descs || !out || n > LVLIP_MAX_BATCH || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    if (wpb != 8 && wpb != 12) return LVLIP_EINVAL;
    const int r = shape & 0xff, g = (shape >> 8) & 0xff;
    if (r != 2 || (g != 1 && g != 2 && g != 4)) return LVLIP_EINVAL;
    uint64_t grid = (uint64_t)lvlip_host::current_cus();
    const uint64_t ng = ((uint64_t)n + g - 1) / g;
    // at least one group per wave's first window... keep grids with real work
    while (grid > 8 && grid * wpb > ng) grid /= 2;
    if (grid > 8) grid &= ~7ull;
    if (stamps && grid * wpb * 16ull > stamp_bytes) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
#define LVLIP_WDYN(GG, WW)                                                                          \
    if (g == GG && wpb == WW) {                                                                     \
        hipLaunchKernelGGL((lvlip::k_window_dyn<2, GG, WW>), dim3((uint32_t)grid), dim3(64 * WW), 0, s, \
                           (const uint8_t*)base, descs, n, out, stamps);                           \
    }
    LVLIP_WDYN(1, 8) LVLIP_WDYN(2, 8) LVLIP_WDYN(4, 8) LVLIP_WDYN(1, 12) LVLIP_WDYN(2, 12) LVLIP_WDYN(4, 12)
#undef LVLIP_WDYN
    return hipGetLastError() == hipSuccess ? (int)(grid * wpb) : LVLIP_EHIP;
}

// wpb: waves per workgroup (4, 8 or 12): with wpb = waves_per_cu every CU runs
// one workgroup.
__attribute__((visibility("default"))) int lvlip_lab_window_stamps(const void* base, const lvlip_csum_desc* descs,
                                                                   uint32_t n, uint16_t* out, uint64_t* stamps,
                                                                   uint64_t stamp_bytes, int waves_per_cu, int wpb,
                                                                   void* stream) {
    if (!base || !descs || !out || !stamps || n == 0 || waves_per_cu <= 0) return LVLIP_EINVAL;
    if (wpb != 4 && wpb != 8 && wpb != 12) return LVLIP_EINVAL;
    uint64_t waves = (uint64_t)lvlip_host::current_cus() * (uint64_t)waves_per_cu;
    const uint64_t ng = ((uint64_t)n + 3) / 4;
    if (waves > ng) waves = ng;
    uint64_t grid = (waves + wpb - 1) / wpb;
    if (grid > 8) grid = grid & ~7ull;
    if (grid * wpb * 16ull > stamp_bytes) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    switch (wpb) {
        case 4:
            hipLaunchKernelGGL((lvlip::k_window_stamp<2, 4, 4>), dim3((uint32_t)grid), dim3(256), 0, s,
                               (const uint8_t*)base, descs, n, out, stamps);
            break;
        case 8:
            hipLaunchKernelGGL((lvlip::k_window_stamp<2, 4, 8>), dim3((uint32_t)grid), dim3(512), 0, s,
                               (const uint8_t*)base, descs, n, out, stamps);
            break;
        default:
            hipLaunchKernelGGL((lvlip::k_window_stamp<2, 4, 12>), dim3((uint32_t)grid), dim3(768), 0, s,
                               (const uint8_t*)base, descs, n, out, stamps);
    }
    return hipGetLastError() == hipSuccess ? (int)(grid * wpb) : LVLIP_EHIP;
}

// lvlip_csum_batch_dev_ex's contract for the lab kernel ids (1, 2, 3, 4, 5, 9, 11).
__attribute__((visibility("default"))) int lvlip_lab_batch_dev_ex(const void* base,
                                                                  const lvlip_csum_desc* descs, uint32_t n,
                                                                  uint16_t* out, void* stream,
                                                                  const lvlip_launch_cfg* cfg) {
    if (n == 0) return LVLIP_OK;
    if (!base || !descs || !out || n > LVLIP_MAX_BATCH || ((uintptr_t)base & 15u) != 0) return LVLIP_EINVAL;
    for (uint32_t lo = 0; lo < n;) {
        const uint32_t m = n - lo < lvlip_host::kLaunchMax ? n - lo : lvlip_host::kLaunchMax;
        const int rc = lab_dispatch(base, descs + lo, m, out + lo, (hipStream_t)stream, cfg);
        if (rc != LVLIP_OK) return rc;
        lo += m;
    }
    return LVLIP_OK;
}

// The frame calls' A/B variants on k_flat2 with a frame source.
// mode: 0 TX fill, 1 RX header (the flat sweep instead of k_rx_hdr), 2 RX +
// L4; 3 the header-only call on k_rx_hdr with a descriptor prefetch.  variant
// bits (modes 0-2): 1 plain (temporal) TX field stores, 2 eight loads per
// round, 4 block group order (else quarters), 8 block order with the frame
// descriptors prefetched 1 280 tiles ahead (k_flat2's PFA); mode 3: the prefetch distance
// (variant >> 3) x 160 blocks.
__attribute__((visibility("default"))) int lvlip_lab_frames_dev(int mode, int variant, void* base,
                                                                const lvlip_frame_desc* frames, uint32_t n,
                                                                uint8_t* out8, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || n > LVLIP_MAX_BATCH / 2u || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    if (mode != 0 && !out8) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const bool nt = !(variant & 1), u8 = variant & 2, blocks = variant & 4, pf = (variant & 8) && mode != 3;
#define LVLIP_LAB_FR(M)                                                                              \
    (pf ? (u8 ? lvlip::launch_frames_flat<M, 8, 2, 1280>(base, frames, n, out8, s, nt)              \
              : lvlip::launch_frames_flat<M, 4, 2, 1280>(base, frames, n, out8, s, nt))             \
        : u8 ? (blocks ? lvlip::launch_frames_flat<M, 8, 2>(base, frames, n, out8, s, nt)           \
                       : lvlip::launch_frames_flat<M, 8, 1>(base, frames, n, out8, s, nt))          \
             : (blocks ? lvlip::launch_frames_flat<M, 4, 2>(base, frames, n, out8, s, nt)           \
                       : lvlip::launch_frames_flat<M, 4, 1>(base, frames, n, out8, s, nt)))
    switch (mode) {
        case 0: return LVLIP_LAB_FR(lvlip::FR_TX);
        case 1: return LVLIP_LAB_FR(lvlip::FR_RX);
        case 2: return LVLIP_LAB_FR(lvlip::FR_RX_L4);
        case 3: {
            // the header-only call on k_rx_hdr with its descriptor prefetch
            // (variant >> 3) x 160 blocks ahead: 0, 1, 2, 4, 8
            const uint32_t grid = (uint32_t)(((uint64_t)n + 255u) / 256u);
            switch (variant >> 3) {
#define LVLIP_RXH(P)                                                                               \
    case P:                                                                                        \
        hipLaunchKernelGGL(lvlip::k_rx_hdr<P * 160>, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, \
                           frames, n, out8);                                                       \
        break;
                LVLIP_RXH(0) LVLIP_RXH(1) LVLIP_RXH(2) LVLIP_RXH(4) LVLIP_RXH(8)
#undef LVLIP_RXH
                default: return LVLIP_EINVAL;
            }
            return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
        }
        default: return LVLIP_EINVAL;
    }
#undef LVLIP_LAB_FR
}

}  // extern "C"
