// lab_kernels.hip — the A/B kernels of DESIGN.md §4, §8, §9 (liblvlip_lab.so,
// diagnostics; the product library does not contain them).
//
//   k_stream       the ring of k_window with contiguous per-wave ranges
//                  (LVLIP_KERNEL_WAVE = 1), in five load policies
//   k_wflat        k_flat2's sweep one wave per tile, tiles dealt round robin (9)
//   k_flat2_occ    k_flat2 compiled for a set number of waves per SIMD (13)
//   k_flat2        its other shapes (3): group orders, tiles of 512, temporal
//                  loads, U 6 / 12, an LDS pad; and the frame calls' variants
//                  (8 loads per round, block order, plain field stores, the
//                  flat sweep for the header-only RX call, whole-block and
//                  cache-policy field stores for TX fill)
//   k_window_stamp, k_flat2_stamp   the product bodies with per-wave /
//                  per-workgroup real-time stamps (diagnostics)
//
// Pruned in round 4 (VERDICT r03 Next #6), measured and rejected by >= 3 %
// (their records stay in profiles/ and DESIGN.md; restore from git):
// k_wave_simple (id 4), k_wave_lds (2), the first flat kernel k_flat (5):
// last in commit 4e633d9; k_rflat (11), k_wsflat (12), k_flat2_perm (14),
// k_window_dyn (15): last in commit 4e633d9.
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

// POL: the data loads' cache policy (A/B, LVLIP_LOAD_POLICY)
template <int R, int POL = 0>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ base,
                                                const lvlip_csum_desc* __restrict__ descs,
                                                uint32_t n, uint16_t* __restrict__ out) {
    __shared__ uint4 s_win[SW_WAVES][2][64];
    ring_sweep<R, 0, POL>(base, descs, n, out, s_win[uniform(threadIdx.x >> 6)]);
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

// ------------------------------------ k_flat2 with per-workgroup stamps --
//
// Diagnostic (lvlip_lab_flat_stamps, round 4): the product's k_flat2 U 8 body
// (block order, descriptor prefetch 1 280 tiles ahead) with thread 0 of each
// workgroup stamping the real-time counter (100 MHz) at its start and after
// its last store, plus the XCD and HW_ID (CU, SIMD, SE) it ran on:
// stamps[4 b .. 4 b + 3] = {t0, t1, xcc | hw_id << 8, 0}.  For the mixed
// line's process-to-process modes: where a slow process loses
// its time.
__global__ __launch_bounds__(FT) void k_flat2_stamp(const uint8_t* __restrict__ base, const DescSrc src,
                                                    uint32_t n, uint64_t* __restrict__ stamps) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    flat2_body<8, true, 2, DescSrc, 1, false, false, kFlatPrefetchTiles>(base, src, n);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        stamps[4u * blockIdx.x] = t0;
        stamps[4u * blockIdx.x + 1u] = t1;
        stamps[4u * blockIdx.x + 2u] = (uint64_t)(xcc & 0xfu) | ((uint64_t)hwid << 8);
        stamps[4u * blockIdx.x + 3u] = 0;
    }
}

}  // namespace lvlip

namespace {

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

}  // namespace

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
        default: return LVLIP_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
}

}  // namespace

extern "C" {

// k_window R 2, G 4 (the MTU shape) at waves_per_cu waves on every CU, with
// per-wave start/end stamps (2 u64 per wave) into `stamps`; returns the number
// of waves (stamps needs 16 B each), or a negative LVLIP_E*.
// k_flat2_stamp over n <= 2^30 descriptors: 32 B of stamps per workgroup
// (ceil(n / 256) of them) into `stamps`; returns the number of workgroups, or
// a negative LVLIP_E*.
__attribute__((visibility("default"))) int lvlip_lab_flat_stamps(const void* base, const lvlip_csum_desc* descs,
                                                                 uint32_t n, uint16_t* out, uint64_t* stamps,
                                                                 uint64_t stamp_bytes, void* stream) {
    if (!base || !descs || !out || !stamps || n == 0 || n > lvlip_host::kLaunchMax) return LVLIP_EINVAL;
    const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
    if ((uint64_t)grid * 32u > stamp_bytes) return LVLIP_EINVAL;
    hipLaunchKernelGGL(lvlip::k_flat2_stamp, dim3(grid), dim3(lvlip::FT), 0, (hipStream_t)stream,
                       (const uint8_t*)base, lvlip::DescSrc{descs, out}, n, stamps);
    return hipGetLastError() == hipSuccess ? (int)grid : LVLIP_EHIP;
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

// lvlip_csum_batch_dev_ex's contract for the lab kernel ids (1, 3, 9, 13).
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
// descriptors prefetched 1 280 tiles ahead (k_flat2's PFA); mode 0 alone: 16
// / 32 the product's shape with whole 32-B / 64-B block field stores
// (FrameSrc's SEC); mode 3: the prefetch distance (variant >> 3) x 160 blocks;
// modes 4 / 5: the echo reply with LVLIP_ECHO_FULL (the flat sweep) / from the
// field (k_echo_reply), variant = the reply's store form (fr_store_echo_reply:
// 0 three byte stores, 2-6 two u16 stores with that cache policy; the
// patched 16-B window chunk of flags 0 was measured and removed, last in
// commit 72b8c4f); variant 7: no reply store at all (timing only, the
// frames keep the request's bytes); mode 5 variant 8: byte stores with a three-chunk window
// (the product's since round 5), variant 0 etc. the four-chunk window.
__attribute__((visibility("default"))) int lvlip_lab_frames_dev(int mode, int variant, void* base,
                                                                const lvlip_frame_desc* frames, uint32_t n,
                                                                uint8_t* out8, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || n > LVLIP_MAX_BATCH / 2u || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    if (mode != 0 && mode != 4 && mode != 5 && !out8) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (mode == 4 || mode == 5) {
        if (n > (1u << 30)) return LVLIP_EINVAL;  // one launch
#define LVLIP_ECHO(P)                                                                                      \
    case P:                                                                                                \
        if (mode == 4) return lvlip::launch_frames_flat<lvlip::FR_ECHO, 8, 2, 0, 0, P>(base, frames, n, out8, s, false); \
        hipLaunchKernelGGL(lvlip::k_echo_reply<P>, dim3((n + 255u) / 256u), dim3(256), 0, s, (uint8_t*)base,  \
                           frames, n, out8);                                                               \
        return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
        if (mode == 5 && variant == 8) {  // byte stores, a three-chunk parse window (the product)
            hipLaunchKernelGGL((lvlip::k_echo_reply<0, 3>), dim3((n + 255u) / 256u), dim3(256), 0, s,
                               (uint8_t*)base, frames, n, out8);
            return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
        }
        switch (variant) {
            LVLIP_ECHO(0) LVLIP_ECHO(2) LVLIP_ECHO(3) LVLIP_ECHO(4) LVLIP_ECHO(5) LVLIP_ECHO(6) LVLIP_ECHO(7)
            default: return LVLIP_EINVAL;
        }
#undef LVLIP_ECHO
    }
    // TX fill with whole-block field stores (round 4): variant 16 = 32-B
    // sectors, 32 = 64-B blocks, on the product's shape (U 8, blocks;
    // nontemporal 16-B block stores; 2-B fields nontemporal)
    // ... and with the field stores' cache policy set (variant 64 k, k = 1-5:
    // sc0, sc1, sc0 sc1, nt sc1, nt sc0 sc1; FrameSrc's STP = k + 1)
    if (mode == 0 && variant >= 64) {
        switch (variant) {
            case 64: return lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 2>(base, frames, n, out8, s, true);
            case 128: return lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 3>(base, frames, n, out8, s, true);
            case 192: return lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 4>(base, frames, n, out8, s, true);
            case 256: return lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 5>(base, frames, n, out8, s, true);
            case 320: return lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 6>(base, frames, n, out8, s, true);
            default: return LVLIP_EINVAL;
        }
    }
    if (mode == 0 && (variant & 48)) {
        if (variant != 16 && variant != 32) return LVLIP_EINVAL;
        return variant == 16 ? lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 32>(base, frames, n, out8, s, true)
                             : lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 64>(base, frames, n, out8, s, true);
    }
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
