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
// Byte alignment: the GPU reads whole 16-byte aligned chunks covering
// [offset, offset+len) and zeroes the bytes outside the packet.  When offset is
// odd, each aligned u16 holds (odd-relative byte, even-relative byte), so the
// two bytes of every half-dword are swapped before summing; the reference's
// tail byte (even relative index) then lands in the low byte as it should.
//
// Kernels (roofline: HBM read bandwidth; ~1 VALU op per loaded dword, no MFMA):
//   k_wave  : one wavefront per packet (BASELINE.json north_star).  A wave's 64
//             lanes read consecutive 16-B chunks of its packet (1 KiB per
//             instruction, fully coalesced), U instructions in flight per lane,
//             then a 64-lane u32 reduction and the fold on lane 0.
//   k_wave_lds : the same, but the chunks are staged HBM -> LDS by LDS-DMA
//             (global_load_lds_dwordx4) and read back with ds_read_b128.
//   k_flat  : chunk-balanced tile sweep for ragged batches.  A 256-thread
//             workgroup owns 256 descriptors; their chunk counts are prefix-summed
//             in LDS, every lane takes one chunk per step (coalesced across packet
//             boundaries), a segmented wave reduction keyed by descriptor index
//             merges lanes of one packet, and the segment tails add into per-
//             descriptor u32 accumulators in LDS.  No lane idles on 20-B headers.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "lvlip_csum.h"

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
__global__ __launch_bounds__(256) void k_wave(const uint8_t* __restrict__ base,
                                              const lvlip_csum_desc* __restrict__ descs,
                                              uint32_t n, uint16_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t stride = gridDim.x * wpb;
    for (uint32_t p = uniform(blockIdx.x * wpb + (threadIdx.x >> 6)); p < n; p += stride) {
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
    const uint32_t stride = gridDim.x * 4u;
    for (uint32_t p = uniform(blockIdx.x * 4u + wid); p < n; p += stride) {
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

// ------------------------------------------------- roofline probe (diagnostic) --
// Pure streaming read of `bytes` (multiple of 16) — the achievable HBM read rate
// on this device, measured beside the checksum kernels (bench.py diagnostics).
__global__ __launch_bounds__(256) void k_read_probe(const uint4* __restrict__ src, uint64_t n16,
                                                    uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        acc += chunk_words<false>(a) + chunk_words<false>(b) + chunk_words<false>(c) +
               chunk_words<false>(d);
    }
    for (; i < n16; i += stride) acc += chunk_words<false>(src[i]);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63u) == 0) atomicAdd(sink, acc);
}

}  // namespace lvlip

// ======================================================== host side (C ABI) ==

namespace {

thread_local char g_last_err[256] = "";

int hip_fail(hipError_t e, const char* what) {
    snprintf(g_last_err, sizeof g_last_err, "%s: %s", what, hipGetErrorString(e));
    return LVLIP_EHIP;
}

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
void launch_wave(uint32_t grid, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                 uint32_t n, uint16_t* out) {
    hipLaunchKernelGGL(lvlip::k_wave<U>, dim3(grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
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

int lvlip_csum_batch_dev_ex(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                            uint16_t* out, void* stream, const lvlip_launch_cfg* cfg) {
    if (n == 0) return LVLIP_OK;
    if (!base || !descs || !out || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    if (((uintptr_t)base & 15u) != 0) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int kernel = cfg ? cfg->kernel : LVLIP_KERNEL_AUTO;
    int unroll = cfg ? cfg->unroll : 0;
    const int wpc = cfg ? cfg->waves_per_cu : 0;

    switch (kernel) {
        case LVLIP_KERNEL_AUTO:
        case LVLIP_KERNEL_WAVE: {
            if (unroll <= 0) unroll = 2;
            const uint32_t grid = grid_for(n, 4, wpc, 4);
            switch (unroll) {
                case 1: launch_wave<1>(grid, s, base, descs, n, out); break;
                case 2: launch_wave<2>(grid, s, base, descs, n, out); break;
                case 4: launch_wave<4>(grid, s, base, descs, n, out); break;
                case 8: launch_wave<8>(grid, s, base, descs, n, out); break;
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

int lvlip_csum_batch_dev(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                         uint16_t* out, void* stream) {
    return lvlip_csum_batch_dev_ex(base, descs, n, out, stream, nullptr);
}

// Diagnostic: streaming-read probe over `bytes` of device memory (multiple of 16).
int lvlip_diag_read_probe(const void* src, uint64_t bytes, uint32_t* sink, int waves_per_cu,
                          void* stream) {
    if (!src || !sink || (bytes & 15u) || ((uintptr_t)src & 15u)) return LVLIP_EINVAL;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const int wpc = waves_per_cu > 0 ? waves_per_cu : 32;
    const uint32_t grid = (uint32_t)((uint64_t)cu_count(dev) * wpc / 4);
    hipLaunchKernelGGL(lvlip::k_read_probe, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, bytes / 16, sink);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "probe launch");
    return LVLIP_OK;
}

}  // extern "C"
