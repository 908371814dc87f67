// lab_probe.hip — read-bandwidth probes (diagnostics, not the product).
//
// Measures what a plain streaming read of HBM reaches on this MI355X under
// different access shapes, so the checksum kernels' roofline fraction can be
// read against both the 8 TB/s spec and the achievable read rate.  Built into
// liblvlip_lab.so; used by scripts/lab_read.py and bench.py's diag block.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint32_t words(uint4 v) {
    return (v.x & 0xffffu) + (v.x >> 16) + (v.y & 0xffffu) + (v.y >> 16) + (v.z & 0xffffu) +
           (v.z >> 16) + (v.w & 0xffffu) + (v.w >> 16);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
    if (NT) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *p;
}

__device__ __forceinline__ uint32_t wsum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// MODE 0: thread-level grid stride, U loads at i + u*stride (interleaved far apart)
// MODE 1: block-contiguous: a block sweeps its own contiguous range; per iteration
//         the block's waves read wpb*U consecutive 1 KiB pieces
// MODE 2: wave-contiguous: a wave sweeps its own range, U consecutive 1 KiB pieces
template <int U, bool NT, int MODE>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ src, uint64_t n16,
                                               uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    if (MODE == 0) {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        for (; i + (U - 1) * stride < n16; i += U * stride) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + i + u * stride);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[u]);
        }
        for (; i < n16; i += stride) acc += words(ld<NT>(src + i));
    } else if (MODE == 4) {
        // packetized like k_stream on tcp1500: 1504-B slots, each read as one full
        // 1 KiB wave-load plus one with lanes 0..29 (the 476-B rest); U packets in
        // flight per wave, wave-contiguous packet ranges
        const uint64_t pk = n16 / 94;
        const uint64_t nw = (uint64_t)gridDim.x * wpb;
        const uint64_t per = (pk + nw - 1) / nw;
        const uint64_t lo = ((uint64_t)blockIdx.x * wpb + wid) * per;
        const uint64_t hi = lo + per < pk ? lo + per : pk;
        const bool part = lane < 30u;
        uint64_t p = lo;
        for (; p + U <= hi; p += U) {
            uint4 v[2 * U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                v[2 * u] = ld<NT>(src + (p + u) * 94 + lane);
                v[2 * u + 1] = ld<NT>(src + (p + u) * 94 + 64 + (part ? lane : 29u));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[2 * u]) + (part ? words(v[2 * u + 1]) : 0u);
        }
        for (; p < hi; ++p) acc += words(ld<NT>(src + p * 94 + lane));
    } else if (MODE == 5) {
        // chip-wide window: chunk c = U consecutive 1 KiB pieces; wave w reads chunks
        // w, w + nw, w + 2 nw, ... so the waves in flight cover one narrow sliding
        // window of the buffer instead of nw far-apart streams
        const uint64_t pieces = n16 / 64;
        const uint64_t nw = (uint64_t)gridDim.x * wpb;
        const uint64_t chunks = pieces / U;
        for (uint64_t c = (uint64_t)blockIdx.x * wpb + wid; c < chunks; c += nw) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + (c * U + u) * 64 + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[u]);
        }
        for (uint64_t p = chunks * U + (uint64_t)blockIdx.x * wpb + wid; p < pieces; p += nw)
            acc += words(ld<NT>(src + p * 64 + lane));
    } else {
        const uint64_t pieces = n16 / 64;  // 1 KiB pieces
        uint64_t lo, hi, step, first;
        if (MODE == 1) {
            const uint64_t per = (pieces + gridDim.x - 1) / gridDim.x;
            lo = (uint64_t)blockIdx.x * per;
            hi = lo + per < pieces ? lo + per : pieces;
            first = lo + wid;
            step = wpb;
        } else {
            const uint64_t nw = (uint64_t)gridDim.x * wpb;
            const uint64_t per = (pieces + nw - 1) / nw;
            lo = ((uint64_t)blockIdx.x * wpb + wid) * per;
            hi = lo + per < pieces ? lo + per : pieces;
            first = lo;
            step = 1;
        }
        uint64_t p = first;
        for (; p + (U - 1) * step < hi; p += U * step) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + (p + u * step) * 64 + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[u]);
        }
        for (; p < hi; p += step) acc += words(ld<NT>(src + p * 64 + lane));
    }
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
}

// Chip-wide window with the chunk size decoupled from the depth: a chunk is
// `cp` consecutive 1 KiB pieces (cp a multiple of U); wave w owns chunks
// w, w + nw, ... and walks each one U pieces (U KiB in flight) at a time.
// The window the waves in flight cover is nw * cp KiB.
// order 2: block-level chunks, see below.
// order 1 numbers the waves XCD-major (block b sits on XCD b % 8 as observed;
// grid a multiple of 8), so consecutive chunks stay on one XCD.
template <int U>
__global__ __launch_bounds__(256) void k_probe_chunk(const uint4* __restrict__ src, uint64_t n16,
                                                     uint32_t cp, uint32_t order,
                                                     uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t pieces = n16 / 64;
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    const uint64_t chunks = pieces / cp;
    if (order == 2) {
        // block chunks (k_flat2's tile sweep in block order): block b owns chunks
        // b, b + grid, ...; its waves take U-piece slices of a chunk round robin,
        // so a block is one stream of 4U KiB per round, cp KiB long
        for (uint64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
            for (uint32_t q = wid * U; q < cp; q += wpb * U) {
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = ld<true>(src + (c * cp + q + u) * 64 + lane);
#pragma unroll
                for (int u = 0; u < U; ++u) acc += words(v[u]);
            }
        }
        for (uint64_t p = chunks * cp + (uint64_t)blockIdx.x * wpb + wid; p < pieces; p += nw)
            acc += words(ld<true>(src + p * 64 + lane));
        acc = wsum(acc);
        if (lane == 0) atomicAdd(sink, acc);
        return;
    }
    const uint64_t rank = order ? ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * wpb + wid
                                : (uint64_t)blockIdx.x * wpb + wid;
    for (uint64_t c = rank; c < chunks; c += nw) {
        for (uint32_t q = 0; q < cp; q += U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<true>(src + (c * cp + q + u) * 64 + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[u]);
        }
    }
    for (uint64_t p = chunks * cp + (uint64_t)blockIdx.x * wpb + wid; p < pieces; p += nw)
        acc += words(ld<true>(src + p * 64 + lane));
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
}

// Packetized chip-wide window: 1504-B slots (tcp1500's layout) in groups of G;
// wave rank r (XCD-major) reads groups r, r + nw, ...; per group all 2G loads
// (one full 1 KiB + one 30-lane load per slot) are issued, then summed.
// SPAN: the group's G slots read as one span in whole 1 KiB loads (the last
// one partial) instead of two loads per slot.
template <int G, bool SPAN>
__global__ __launch_bounds__(256) void k_probe_pkwin(const uint4* __restrict__ src, uint64_t n16,
                                                     uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;
    const uint64_t rank = ((uint64_t)(blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * 4u + wid;
    const uint64_t groups = n16 / 94 / G;
    const bool part = lane < 30u;
    if (SPAN) {
        constexpr uint32_t NCH = 94u * G;            // chunks of the span
        constexpr uint32_t NL = (NCH + 63u) / 64u;   // whole loads
        for (uint64_t g = rank; g < groups; g += nw) {
            uint4 v[NL];
#pragma unroll
            for (uint32_t u = 0; u < NL; ++u) {
                const uint32_t c = u * 64u + lane;
                v[u] = ld<true>(src + g * NCH + (c < NCH ? c : NCH - 1u));
            }
#pragma unroll
            for (uint32_t u = 0; u < NL; ++u) acc += (u * 64u + lane < NCH) ? words(v[u]) : 0u;
        }
        acc = wsum(acc);
        if (lane == 0) atomicAdd(sink, acc);
        return;
    }
    for (uint64_t g = rank; g < groups; g += nw) {
        uint4 v[2 * G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const uint64_t p = g * G + u;
            v[2 * u] = ld<true>(src + p * 94 + lane);
            v[2 * u + 1] = ld<true>(src + p * 94 + 64 + (part ? lane : 29u));
        }
#pragma unroll
        for (int u = 0; u < G; ++u) acc += words(v[2 * u]) + (part ? words(v[2 * u + 1]) : 0u);
    }
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
}

// LDS-DMA (global_load_lds_dwordx4) staging, block-contiguous like MODE 1.
template <int U>
__global__ __launch_bounds__(256) void k_probe_lds(const uint4* __restrict__ src, uint64_t n16,
                                                   uint32_t* __restrict__ sink) {
    __shared__ uint4 slab[4][U][64];
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t pieces = n16 / 64;
    const uint64_t per = (pieces + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < pieces ? lo + per : pieces;
    uint64_t p = lo + wid;
    for (; p + (U - 1) * wpb < hi; p += U * wpb) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_global_load_lds((const void*)(src + (p + u * wpb) * 64 + lane),
                                             (__attribute__((address_space(3))) void*)&slab[wid][u][0],
                                             16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; ++u) acc += words(slab[wid][u][lane]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    for (; p < hi; p += wpb) acc += words(src[p * 64 + lane]);
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
}

// Timeline probe: where the time of a streaming read goes (launch ramp, steady
// state, tail).  Wave-contiguous ranges (DYN = false, MODE 2's shape) or
// granules of `gp` 1-KiB pieces claimed from 8 per-XCD queues (DYN = true:
// queue q holds granules q, q+8, ...; a wave starts on its own XCD's queue and
// moves to the next queue when that one is empty; the next claim is issued
// before the current granule is read).  With tl != null lane 0 of every wave
// writes {t_start, t_end, xcc | hw_id << 8, claims} (s_memrealtime, 100 MHz).
template <int U, bool DYN>
__global__ __launch_bounds__(256) void k_probe_tl(const uint4* __restrict__ src, uint64_t pieces,
                                                  uint32_t gp, uint32_t* __restrict__ ctr,
                                                  unsigned long long* __restrict__ tl,
                                                  uint32_t* __restrict__ sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * wpb + wid;
    uint32_t xcc, hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    xcc &= 7u;
    uint32_t claims = 0;
    auto sweep = [&](uint64_t lo, uint64_t hi) {
        uint64_t p = lo;
        for (; p + U <= hi; p += U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<true>(src + (p + u) * 64 + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += words(v[u]);
        }
        for (; p < hi; ++p) acc += words(ld<true>(src + p * 64 + lane));
    };
    if (!DYN) {
        const uint64_t nw = (uint64_t)gridDim.x * wpb;
        const uint64_t per = (pieces + nw - 1) / nw;
        const uint64_t lo = wave * per;
        const uint64_t hi = lo + per < pieces ? lo + per : pieces;
        if (lo < hi) sweep(lo, hi);
        claims = 1;
    } else {
        const uint64_t ngran = (pieces + gp - 1) / gp;
        uint32_t q = xcc, tries = 0;
        // claim: granule index or ~0 when every queue is empty
        auto claim = [&]() -> uint64_t {
            while (tries < 8u) {
                uint32_t k = 0;
                if (lane == 0) k = atomicAdd(&ctr[q * 32u], 1u);
                k = __builtin_amdgcn_readfirstlane(k);
                const uint64_t g = (uint64_t)k * 8u + q;
                if (g < ngran) return g;
                q = (q + 1u) & 7u;
                ++tries;
            }
            return ~0ull;
        };
        uint64_t g = claim();
        while (g != ~0ull) {
            const uint64_t nxt = claim();
            ++claims;
            const uint64_t lo = g * gp;
            const uint64_t hi = lo + gp < pieces ? lo + gp : pieces;
            sweep(lo, hi);
            g = nxt;
        }
    }
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
    if (tl && lane == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        tl[wave * 4 + 0] = t0;
        tl[wave * 4 + 1] = t1;
        tl[wave * 4 + 2] = xcc | ((unsigned long long)hwid << 8);
        tl[wave * 4 + 3] = claims;
    }
}

template <int U, bool NT, int MODE>
void go(uint32_t grid, hipStream_t s, const void* src, uint64_t n16, uint32_t* sink) {
    hipLaunchKernelGGL((k_probe<U, NT, MODE>), dim3(grid), dim3(256), 0, s, (const uint4*)src, n16,
                       sink);
}

}  // namespace

extern "C" int lvlip_lab_probe(const void* src, uint64_t bytes, uint32_t* sink, int mode,
                               int unroll, int nt, int blocks, void* stream) {
    if (!src || !sink || (bytes & 1023u)) return -1;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t n16 = bytes / 16;
    const uint32_t g = (uint32_t)blocks;
#define CASE(M, U, N) \
    if (mode == M && unroll == U && nt == N) { go<U, (bool)N, M>(g, s, src, n16, sink); return hipGetLastError() == hipSuccess ? 0 : -3; }
#define CASES(M, U) CASE(M, U, 0) CASE(M, U, 1)
    CASES(0, 1) CASES(0, 2) CASES(0, 4) CASES(0, 8)
    CASES(1, 1) CASES(1, 2) CASES(1, 4) CASES(1, 8)
    CASES(2, 1) CASES(2, 2) CASES(2, 4) CASES(2, 8)
    CASES(4, 1) CASES(4, 2) CASES(4, 3) CASES(4, 4)
    CASES(5, 1) CASES(5, 2) CASES(5, 4) CASES(5, 8)
#undef CASES
#undef CASE
    if (mode == 3) {
        if (unroll == 1) hipLaunchKernelGGL(k_probe_lds<1>, dim3(g), dim3(256), 0, s, (const uint4*)src, n16, sink);
        else if (unroll == 2) hipLaunchKernelGGL(k_probe_lds<2>, dim3(g), dim3(256), 0, s, (const uint4*)src, n16, sink);
        else if (unroll == 4) hipLaunchKernelGGL(k_probe_lds<4>, dim3(g), dim3(256), 0, s, (const uint4*)src, n16, sink);
        else if (unroll == 8) hipLaunchKernelGGL(k_probe_lds<8>, dim3(g), dim3(256), 0, s, (const uint4*)src, n16, sink);
        else return -1;
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    return -1;
}

extern "C" int lvlip_lab_probe_chunk(const void* src, uint64_t bytes, uint32_t* sink, int unroll,
                                     uint32_t chunk_pieces, uint32_t order, int blocks, void* stream) {
    if (!src || !sink || (bytes & 1023u) || chunk_pieces == 0 || chunk_pieces % (uint32_t)unroll ||
        (order == 1 && (blocks & 7)) || order > 2 || (order == 2 && chunk_pieces % (4u * (uint32_t)unroll)))
        return -1;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((uint32_t)blocks), b(256);
    const uint64_t n16 = bytes / 16;
#define CH(U) \
    if (unroll == U) { hipLaunchKernelGGL(k_probe_chunk<U>, g, b, 0, s, (const uint4*)src, n16, chunk_pieces, order, sink); return hipGetLastError() == hipSuccess ? 0 : -3; }
    CH(2) CH(3) CH(4) CH(6) CH(8)
#undef CH
    return -1;
}

extern "C" int lvlip_lab_probe_pkwin(const void* src, uint64_t bytes, uint32_t* sink, int group,
                                     int blocks, void* stream) {
    if (!src || !sink || (bytes & 15u) || (blocks & 7)) return -1;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((uint32_t)blocks), b(256);
    const uint64_t n16 = bytes / 16;
#define PW(G) \
    if (group == G) { hipLaunchKernelGGL((k_probe_pkwin<G, false>), g, b, 0, s, (const uint4*)src, n16, sink); return hipGetLastError() == hipSuccess ? 0 : -3; } \
    if (group == 100 + G) { hipLaunchKernelGGL((k_probe_pkwin<G, true>), g, b, 0, s, (const uint4*)src, n16, sink); return hipGetLastError() == hipSuccess ? 0 : -3; }
    PW(1) PW(2) PW(3) PW(4) PW(6) PW(8)
#undef PW
    return -1;
}

// ctr: 8 queue heads at stride 32 u32 (zeroed by the caller before each DYN
// launch); tl: 4 u64 per wave or null.
extern "C" int lvlip_lab_probe_tl(const void* src, uint64_t bytes, uint32_t* sink, int dyn,
                                  int unroll, uint32_t gp, uint32_t* ctr, unsigned long long* tl,
                                  int blocks, void* stream) {
    if (!src || !sink || (bytes & 1023u) || (dyn && (!ctr || gp == 0))) return -1;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t pieces = bytes / 1024;
    const dim3 g((uint32_t)blocks), b(256);
#define TL(U, D) \
    if (unroll == U && (bool)dyn == D) { hipLaunchKernelGGL((k_probe_tl<U, D>), g, b, 0, s, (const uint4*)src, pieces, gp, ctr, tl, sink); return hipGetLastError() == hipSuccess ? 0 : -3; }
    TL(4, false) TL(4, true) TL(8, false) TL(8, true)
#undef TL
    return -1;
}

// ---- scattered field-store probe (round 4, VERDICT r03 Next #1) ----------------
// One lane per frame of a frame-descriptor array (16 B: offset u64, len u32,
// pad): the TX fill's two checksum fields at frame + 24 and frame + 50 (ihl 5,
// TCP), written on their own with nothing else running.  The buffer is
// scratch (modes 0, 3 and 5 store constants).
//   0  two 2-B nontemporal stores (the product's field stores)
//   1  two 2-B loads, then the same bytes stored back nontemporally
//   2  the aligned 32-B sector around each field loaded and stored back whole
//      (nontemporal), once when both fields share it
//   3  the same sectors stored whole without the load (constants)
//   4  the aligned 64-B blocks, loaded and stored back whole
//   5  two 2-B plain (temporal) stores
//   6-10  two 2-B stores with cache policy sc0 / sc1 / sc0 sc1 / nt sc1 / nt sc0 sc1
//   11-16 (round 4, k_probe_sectors) the aligned B-byte block around each field
//      written whole by B/16 adjacent lanes in ONE store instruction (one
//      coalesced request per block, no load; once when both fields share it):
//      11 B 32 nt, 12 B 32 plain, 13 B 64 nt, 14 B 64 plain, 15 B 32 nt sc0 sc1,
//      16 B 128 plain; 17 / 18 B 64 loaded by the same four lanes first, then
//      stored back nt / plain (the blocks' current bytes, as a TX fill must).  HBM3E has no write data mask, so a partial-sector write
//      is a read-modify-write in the memory controller; a whole-sector request
//      is not.
namespace {
typedef unsigned int pv4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) pv4 gpv4;

// salt: 0 at run time, unknown to the compiler (a load stored back unchanged
// would otherwise be removed together with its store)
template <int NQ, bool LOAD>
__device__ __forceinline__ void probe_block(uint64_t a, uint32_t salt) {
    pv4 q[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k)
        q[k] = LOAD ? (*reinterpret_cast<gpv4*>(a + 16u * k) ^ pv4{salt, salt, salt, salt}) : pv4{1u, 2u, 3u, 4u};
#pragma unroll
    for (int k = 0; k < NQ; ++k) __builtin_nontemporal_store(q[k], reinterpret_cast<gpv4*>(a + 16u * k));
}

template <int MODE>
__global__ __launch_bounds__(256) void k_probe_fields(uint8_t* __restrict__ buf, const uint4* __restrict__ fd,
                                                      uint32_t n, uint32_t salt) {
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f >= n) return;
    const uint4 d = fd[f];
    const uint64_t fs = reinterpret_cast<uint64_t>(buf) + (((uint64_t)d.y << 32) | d.x);
    const uint64_t a0 = fs + 24u, a1 = fs + 50u;
    typedef __attribute__((address_space(1))) uint16_t gu16;
    if (MODE == 0 || MODE == 5) {
        if (MODE == 0) {
            __builtin_nontemporal_store((uint16_t)f, reinterpret_cast<gu16*>(a0));
            __builtin_nontemporal_store((uint16_t)f, reinterpret_cast<gu16*>(a1));
        } else {
            *reinterpret_cast<gu16*>(a0) = (uint16_t)f;
            *reinterpret_cast<gu16*>(a1) = (uint16_t)f;
        }
    } else if (MODE == 1) {
        const uint16_t x0 = *reinterpret_cast<gu16*>(a0) ^ (uint16_t)salt;
        const uint16_t x1 = *reinterpret_cast<gu16*>(a1) ^ (uint16_t)salt;
        __builtin_nontemporal_store(x0, reinterpret_cast<gu16*>(a0));
        __builtin_nontemporal_store(x1, reinterpret_cast<gu16*>(a1));
    } else if (MODE >= 6) {
        // 2-B stores with an explicit cache policy: 6 sc0, 7 sc1, 8 sc0 sc1,
        // 9 nt sc1, 10 nt sc0 sc1
        const uint32_t v = f & 0xffffu;
#define PST(BITS) asm volatile("global_store_short %0, %2, off " BITS "\n\tglobal_store_short %1, %2, off " BITS \
                               ::"v"(a0), "v"(a1), "v"(v) : "memory")
        if (MODE == 6) PST("sc0");
        else if (MODE == 7) PST("sc1");
        else if (MODE == 8) PST("sc0 sc1");
        else if (MODE == 9) PST("nt sc1");
        else PST("nt sc0 sc1");
#undef PST
    } else {
        constexpr uint64_t B = MODE == 4 ? 64u : 32u;
        constexpr int NQ = (int)(B / 16u);
        const uint64_t s0 = a0 & ~(B - 1u), s1 = a1 & ~(B - 1u);
        probe_block<NQ, MODE != 3>(s0, salt);
        if (s1 != s0) probe_block<NQ, MODE != 3>(s1, salt);
    }
}

// B/16 lanes per block, two blocks per frame: thread t -> frame t / (2 B/16),
// field (t / (B/16)) & 1, quarter t % (B/16).
template <int B, int POL>
__global__ __launch_bounds__(256) void k_probe_sectors(uint8_t* __restrict__ buf, const uint4* __restrict__ fd,
                                                       uint32_t n, uint32_t salt) {
    constexpr uint32_t QB = B / 16, T = 2 * QB;
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t f = t / T;
    if (f >= n) return;
    const uint32_t r = (uint32_t)(t % T), field = r / QB, q = r % QB;
    const uint4 d = fd[f];
    const uint64_t fs = reinterpret_cast<uint64_t>(buf) + (((uint64_t)d.y << 32) | d.x);
    const uint64_t s0 = (fs + 24u) & ~(uint64_t)(B - 1), s1 = (fs + 50u) & ~(uint64_t)(B - 1);
    if (field == 1 && s1 == s0) return;
    const uint64_t a = (field ? s1 : s0) + 16u * q;
    pv4 v = pv4{salt ^ (uint32_t)f, salt, salt, salt};
    if (POL >= 3) v = *reinterpret_cast<gpv4*>(a) ^ pv4{salt, salt, salt, salt};
    if (POL == 0 || POL == 3) __builtin_nontemporal_store(v, reinterpret_cast<gpv4*>(a));
    else if (POL == 4) *reinterpret_cast<gpv4*>(a) = v;
    else if (POL == 1) *reinterpret_cast<gpv4*>(a) = v;
    else asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(a), "v"(v) : "memory");
}
}  // namespace

extern "C" int lvlip_lab_probe_fields(void* buf, const void* frames, uint32_t n, int mode, void* stream) {
    if (!buf || !frames) return -1;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((n + 255u) / 256u), b(256);
#define PF(M) \
    if (mode == M) { hipLaunchKernelGGL(k_probe_fields<M>, g, b, 0, s, (uint8_t*)buf, (const uint4*)frames, n, 0u); return hipGetLastError() == hipSuccess ? 0 : -3; }
    PF(0) PF(1) PF(2) PF(3) PF(4) PF(5) PF(6) PF(7) PF(8) PF(9) PF(10)
#undef PF
#define PS(M, B, POL)                                                                                          \
    if (mode == M) {                                                                                           \
        const uint64_t th = (uint64_t)n * (2u * (B / 16u));                                                    \
        hipLaunchKernelGGL((k_probe_sectors<B, POL>), dim3((uint32_t)((th + 255u) / 256u)), b, 0, s, (uint8_t*)buf, \
                           (const uint4*)frames, n, 0u);                                                       \
        return hipGetLastError() == hipSuccess ? 0 : -3;                                                       \
    }
    PS(11, 32, 0) PS(12, 32, 1) PS(13, 64, 0) PS(14, 64, 1) PS(15, 32, 2) PS(16, 128, 1) PS(17, 64, 3) PS(18, 64, 4)
#undef PS
    return -1;
}

// ---- address-class probe (round 4): is there XCD <-> memory locality? -------
// The buffer is cut into units of CB bytes; unit u has class u mod 8 and is
// read by the waves of block slot x = ((u mod 8) + shift) mod 8 (block b runs
// on XCD b % 8, as observed).  Each block slot's units form its own stream,
// dealt to its waves in 4 KiB chunks round robin (the window probe's best
// shape), U 1-KiB loads in flight per wave.  If memory were interleaved over
// the stacks at CB granularity by (address / CB) mod 8, and an XCD reached
// some stacks faster than others, one shift would read faster than the rest.
namespace {
template <int U>
__global__ __launch_bounds__(256) void k_probe_xcd(const uint4* __restrict__ src, uint64_t bytes, uint32_t cb_log2,
                                                   uint32_t shift, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t slot = blockIdx.x & 7u;
    const uint64_t nwx = (uint64_t)(gridDim.x >> 3) * 4u;  // waves per block slot
    const uint64_t r = (uint64_t)(blockIdx.x >> 3) * 4u + wid;
    const uint32_t cls = (slot + 8u - (shift & 7u)) & 7u;   // the class this slot reads
    const uint64_t cb = 1ull << cb_log2;
    const uint64_t units = bytes >> cb_log2;
    const uint64_t per_slot = units / 8u;                   // whole rounds of 8 classes
    const uint64_t stream = per_slot << cb_log2;            // bytes of this slot's stream
    const uint64_t chunks = stream / 4096u;
    for (uint64_t c = r; c < chunks; c += nwx) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t q = c * 4096u + (uint64_t)u * 1024u + lane * 16u;  // offset in the slot's stream
            const uint64_t j = q >> cb_log2, off = q & (cb - 1u);
            v[u] = ld<true>(src + (((j * 8u + cls) << cb_log2) + off) / 16u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += words(v[u]);
    }
    acc = wsum(acc);
    if (lane == 0) atomicAdd(sink, acc);
}
}  // namespace

// cb_log2: 8 (256 B) .. 21 (2 MiB); shift 0-7; blocks a multiple of 8.
extern "C" int lvlip_lab_probe_xcd(const void* src, uint64_t bytes, uint32_t* sink, uint32_t cb_log2,
                                   uint32_t shift, int blocks, void* stream) {
    if (!src || !sink || cb_log2 < 8 || cb_log2 > 24 || (blocks & 7) || blocks <= 0) return -1;
    hipLaunchKernelGGL(k_probe_xcd<4>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, bytes, cb_log2, shift, sink);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- cross-XCD atomicity probe -----------------------------------------------
// Every wave's lane 0 takes K tickets from one counter: MODE 0 agent-scope
// atomicAdd (global_atomic_add ... sc0), MODE 1 system scope (... sc0 sc1),
// MODE 2 the agent-scope add from asm with sc1 added.  The host checks that the
// tickets are exactly 0 .. waves*K-1 (one claim per ticket, across XCDs).
namespace {
template <int MODE>
__global__ __launch_bounds__(256) void k_atomics(uint32_t* ctr, uint32_t* tickets, uint32_t k) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane != 0) return;
    for (uint32_t i = 0; i < k; ++i) {
        uint32_t t;
        if (MODE == 0) t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (MODE == 1) t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else {
            const uint32_t one = 1u;
            asm volatile("global_atomic_add %0, %1, %2, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                         : "=v"(t) : "v"(ctr), "v"(one) : "memory");
        }
        tickets[(wave * k + i) * 2] = t;
        tickets[(wave * k + i) * 2 + 1] = xcc & 7u;
    }
}
}  // namespace

extern "C" int lvlip_lab_atomics(uint32_t* ctr, uint32_t* tickets, int mode, int blocks, uint32_t k,
                                 void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((uint32_t)blocks), b(256);
    if (mode == 0) hipLaunchKernelGGL(k_atomics<0>, g, b, 0, s, ctr, tickets, k);
    else if (mode == 1) hipLaunchKernelGGL(k_atomics<1>, g, b, 0, s, ctr, tickets, k);
    else if (mode == 2) hipLaunchKernelGGL(k_atomics<2>, g, b, 0, s, ctr, tickets, k);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- buffer out-of-range semantics probe -------------------------------------
// out[(nr*3 + b)*4 + k] = dword k of buffer_load_dwordx4 at voffset 0 from an SRD
// with base = buf + b (b = 0, 1, 2) and num_records = nr (nr = 0..23).  Tells
// whether the range check zeroes per dword or per instruction, and what an
// unaligned SRD base returns.
namespace {
// One wave; every SRD is built from the uniform loop counter only.  All loads
// stay inside buf[0, 64) (num_records <= 23, base offset <= 4, 16-B loads at
// voffset 0 read at most buf[4 .. 20)).
__global__ void k_oob(const uint8_t* buf, uint32_t* out) {
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x;
    for (uint32_t cs = 0; cs < 72; ++cs) {
        const uint32_t nr = cs / 3, b = (cs % 3);  // base offsets 0, 1, 2
        const uint64_t a = reinterpret_cast<uint64_t>(buf) + b;
        u32x4_t s;
        s.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
        s.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
        s.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)nr);
        s.w = 0x00020000u;
        const uint32_t voff = 0;
        u32x4_t t;
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                     : "=v"(t) : "v"(voff), "s"(s) : "memory");
        if (lane == 0) {
            out[cs * 4 + 0] = t.x;
            out[cs * 4 + 1] = t.y;
            out[cs * 4 + 2] = t.z;
            out[cs * 4 + 3] = t.w;
        }
    }
}
}  // namespace

extern "C" int lvlip_lab_oob(const void* buf, uint32_t* out, void* stream) {
    hipLaunchKernelGGL(k_oob, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)buf, out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
