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
