// testkit.hip — synthetic-input generators for tests/ and bench.py.
//
// NOT part of the checksum product: liblvlip_testkit.so only fills device
// buffers with the BASELINE.md synthetic workload (splitmix64, seed 0x1E7E1C5)
// fast enough for the 1.5 GB / 9.4 GB configurations.  The byte stream is
// defined identically in oracle/csum_oracle.c (oracle_fill) and
// level-ip_amd/workloads.py (fill_bytes), so CPU and GPU agree on inputs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvlip_csum.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// word j of the stream (bytes 8j..8j+7, little-endian)
__global__ __launch_bounds__(256) void k_fill(uint64_t* __restrict__ dst, uint64_t nwords,
                                              uint64_t seed, uint64_t first_word) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride)
        dst[i] = splitmix64(seed ^ ((first_word + i) * 0xD1B54A32D192ED03ull));
}

// Overwrite whole packets: value[i] = 0 keep, 1 all-0x00, 2 all-0xff.
__global__ __launch_bounds__(256) void k_paint(uint8_t* __restrict__ base,
                                               const lvlip_csum_desc* __restrict__ d,
                                               const uint8_t* __restrict__ value, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wpb = blockDim.x >> 6;
    for (uint32_t p = blockIdx.x * wpb + (threadIdx.x >> 6); p < n; p += gridDim.x * wpb) {
        const uint8_t v = value[p];
        if (v == 0 || d[p].len <= 0) continue;
        const uint8_t b = v == 1 ? 0x00 : 0xff;
        uint8_t* q = base + d[p].offset;
        for (uint32_t k = lane; k < (uint32_t)d[p].len; k += 64) q[k] = b;
    }
}

}  // namespace

extern "C" {

int lvlip_testkit_fill(void* dst, uint64_t bytes, uint64_t seed, uint64_t first_byte,
                       void* stream) {
    if (!dst || (bytes & 7u) || (first_byte & 7u) || ((uintptr_t)dst & 7u)) return LVLIP_EINVAL;
    const uint64_t nwords = bytes / 8;
    if (!nwords) return LVLIP_OK;
    uint64_t grid = (nwords + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_fill, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream,
                       (uint64_t*)dst, nwords, seed, first_byte / 8);
    return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
}

int lvlip_testkit_paint(void* base, const lvlip_csum_desc* d, const uint8_t* value, uint32_t n,
                        void* stream) {
    if (!base || !d || !value) return LVLIP_EINVAL;
    if (!n) return LVLIP_OK;
    uint64_t grid = ((uint64_t)n + 3) / 4;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_paint, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream,
                       (uint8_t*)base, d, value, n);
    return hipGetLastError() == hipSuccess ? LVLIP_OK : LVLIP_EHIP;
}

}  // extern "C"
