// skb_dev.hip — f1/f2 of SURVEY.md §8f for frames already in HBM
// (include/lvlip_skb.h, "device-resident frames").
//
// Default: one fused launch of the flat sweep whose phase 1 parses the frames
// and whose phase 4 applies the results (FrameSrc, flat_src.h).  Kept as an A/B
// path (LVLIP_FRAMES_3PASS=1) and as a cross-check in the tests: the same
// decisions as skb_batch.c (which cites the reference line of each), as
// three stream-ordered steps with no host round trip:
//   plan   one thread per frame parses its Ethernet/IPv4 header bytes and
//          writes its checksum descriptors at fixed slots (2i, 2i+1 when an L4
//          entry may exist, else i; an unused slot is an empty descriptor) plus
//          a plan word,
//   batch  lvlip_csum_batch_dev_ex over the 2n descriptors (AUTO: the flat
//          sweep, as the entries are 20-60 B headers next to payloads),
//   apply  one thread per frame turns its two results into a verdict (RX) or
//          stores them raw into the frame's checksum fields (TX).
// Frames are read with byte loads (any alignment); a frame's bytes are never
// read past its `len`.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

int lvlip_internal_hip_fail(hipError_t e, const char* what);  // csum_kernels.hip
// the fused path (csum_kernels.hip, flat_src.h): mode 0 TX, 1 RX, 2 RX + L4
int lvlip_internal_frames(int mode, const void* base, const lvlip_frame_desc* frames, uint32_t n,
                          uint8_t* out8, void* stream);

namespace {

constexpr uint32_t kEth = 14;
constexpr uint32_t kPending = 0x80;  // verdict deferred until the header checksum is known
constexpr uint32_t kHasHdr = 0x100;  // plan word: slot 2i holds the IPv4 header entry
constexpr uint32_t kHasL4 = 0x200;   // plan word: slot 2i+1 holds a TCP/ICMP entry

__device__ __forceinline__ uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// src/tcp.c:92-95: whole u32 words, carry out of bit 31 lost (as lvlip_pseudo_sum)
__device__ __forceinline__ uint32_t pseudo_lossy(uint32_t s, uint32_t d, uint32_t proto, uint32_t len) {
    return s + d + bswap16(proto) + bswap16(len);
}
// the same words as 16-bit halves (as lvlip_pseudo_sum_rfc)
__device__ __forceinline__ uint32_t pseudo_rfc(uint32_t s, uint32_t d, uint32_t proto, uint32_t len) {
    return (s & 0xffffu) + (s >> 16) + (d & 0xffffu) + (d >> 16) + bswap16(proto) + bswap16(len);
}

__device__ __forceinline__ lvlip_csum_desc mk(uint64_t off, uint32_t len, uint32_t start) {
    lvlip_csum_desc d;
    d.offset = off;
    d.len = (int32_t)len;
    d.start_sum = start;
    return d;
}

__global__ __launch_bounds__(256) void k_rx_plan(const uint8_t* __restrict__ base,
                                                 const lvlip_frame_desc* __restrict__ frames, uint32_t n,
                                                 uint32_t flags, lvlip_csum_desc* __restrict__ descs,
                                                 uint32_t* __restrict__ plan) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const lvlip_frame_desc f = frames[i];
    const uint8_t* h = base + f.offset;
    uint32_t v = 0, w = 0;
    lvlip_csum_desc d0 = mk(0, 0, 0), d1 = mk(0, 0, 0);
    if (f.len < kEth + 20u) {
        v = LVLIP_RX_SHORT;
    } else if (be16(h + 12) != 0x0800u) {  // netdev_receive, src/netdev.c:67-80
        v = LVLIP_RX_NOT_IP;
    } else {
        const uint32_t ver = h[14] >> 4, ihl = h[14] & 0x0fu;
        if (ver != 4u) {  // src/ip_input.c:22
            v = LVLIP_RX_BAD_VERSION;
        } else if (ihl < 5u) {  // src/ip_input.c:27
            v = LVLIP_RX_BAD_IHL;
        } else if (h[22] == 0u) {  // src/ip_input.c:32
            v = LVLIP_RX_TTL0;
        } else if (f.len < kEth + ihl * 4u) {
            v = LVLIP_RX_SHORT;
        } else {
            d0 = mk(f.offset + kEth, ihl * 4u, 0);  // src/ip_input.c:38
            w |= kHasHdr;
            const uint32_t proto = h[23];
            if (proto != 6u && proto != 1u) {  // src/ip_input.c:51-60
                v = kPending | LVLIP_RX_UNKNOWN_PROTO;
            } else if (flags & LVLIP_RX_VERIFY_L4) {
                const uint32_t iplen = be16(h + 16);
                if (iplen < ihl * 4u || f.len < kEth + iplen) {
                    v = kPending | LVLIP_RX_SHORT;
                } else {
                    const uint32_t l4len = iplen - ihl * 4u;
                    const uint32_t seed = proto == 6u ? pseudo_rfc(le32(h + 26), le32(h + 30), 6u, l4len) : 0u;
                    d1 = mk(f.offset + kEth + ihl * 4u, l4len, seed);
                    w |= kHasL4;
                }
            }
        }
    }
    if (flags & LVLIP_RX_VERIFY_L4) {
        descs[2 * i] = d0;
        descs[2 * i + 1] = d1;
    } else {
        descs[i] = d0;  // header entries only: one slot per frame
    }
    plan[i] = w | v;
}

__global__ __launch_bounds__(256) void k_rx_apply(const uint32_t* __restrict__ plan,
                                                  const uint16_t* __restrict__ res, uint32_t n,
                                                  uint32_t slots, uint8_t* __restrict__ verdict) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t w = plan[i];
    uint32_t v = w & 0xffu;
    if (w & kHasHdr) {
        if (res[slots * i] != 0u)
            v = LVLIP_RX_BAD_CSUM;
        else if ((w & kHasL4) && res[slots * i + 1] != 0u && v == 0u)
            v = LVLIP_RX_BAD_L4;
        v = v == 0u ? (uint32_t)LVLIP_RX_OK : (v & ~kPending);
    }
    verdict[i] = (uint8_t)v;
}

__global__ __launch_bounds__(256) void k_tx_plan(const uint8_t* __restrict__ base,
                                                 const lvlip_frame_desc* __restrict__ frames, uint32_t n,
                                                 lvlip_csum_desc* __restrict__ descs,
                                                 uint32_t* __restrict__ plan) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const lvlip_frame_desc f = frames[i];
    const uint8_t* h = base + f.offset;
    lvlip_csum_desc d0 = mk(0, 0, 0), d1 = mk(0, 0, 0);
    uint32_t w = 0;
    if (f.len >= kEth + 20u) {
        const uint32_t ihl = h[14] & 0x0fu, iplen = be16(h + 16), proto = h[23];
        if ((h[14] >> 4) == 4u && ihl >= 5u && iplen >= ihl * 4u && f.len >= kEth + iplen) {
            const uint32_t l4 = kEth + ihl * 4u, l4len = iplen - ihl * 4u;
            // each field's current u16 is taken out of the seed (skb_batch.c):
            // the same sum as the reference's zero-then-checksum, mod 2^32
            if (proto == 6u && l4len >= 20u) {  // src/tcp_output.c:110,126
                d0 = mk(f.offset + l4, l4len,
                        pseudo_lossy(le32(h + 26), le32(h + 30), 6u, l4len) - le16(h + l4 + 16));
                w = kHasL4 | ((l4 + 16u) << 16);
            } else if (proto == 1u && l4len >= 4u) {  // src/icmpv4.c:46-47
                d0 = mk(f.offset + l4, l4len, 0u - le16(h + l4 + 2));
                w = kHasL4 | ((l4 + 2u) << 16);
            }
            d1 = mk(f.offset + kEth, ihl * 4u, 0u - le16(h + 24));  // src/ip_output.c:42,53
            w |= 1u;
        }
    }
    descs[2 * i] = d0;
    descs[2 * i + 1] = d1;
    plan[i] = w;
}

__global__ __launch_bounds__(256) void k_tx_apply(uint8_t* __restrict__ base,
                                                  const lvlip_frame_desc* __restrict__ frames, uint32_t n,
                                                  const uint32_t* __restrict__ plan,
                                                  const uint16_t* __restrict__ res,
                                                  uint8_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t w = plan[i];
    if (status) status[i] = (uint8_t)(w & 1u);
    if (!(w & 1u)) return;
    uint8_t* h = base + frames[i].offset;
    if (w & kHasL4) {  // raw store (no htons), byte by byte: any alignment
        const uint32_t fo = w >> 16, c = res[2 * i];
        h[fo] = (uint8_t)c;
        h[fo + 1] = (uint8_t)(c >> 8);
    }
    const uint32_t c = res[2 * i + 1];
    h[24] = (uint8_t)c;
    h[25] = (uint8_t)(c >> 8);
}

struct Workspace {
    lvlip_csum_desc* descs;
    uint16_t* res;
    uint32_t* plan;
};

inline uint64_t round16(uint64_t x) { return (x + 15u) & ~15ull; }

Workspace carve(void* ws, uint32_t n) {
    uint8_t* p = (uint8_t*)ws;
    Workspace w;
    w.descs = (lvlip_csum_desc*)p;
    w.res = (uint16_t*)(p + 32ull * n);
    w.plan = (uint32_t*)(p + 32ull * n + round16(4ull * n));
    return w;
}

// LVLIP_FRAMES_3PASS=1 (A/B, read once): the plan / batch / apply pipeline
// below instead of the fused sweep (flat_src.h), which is the default.
bool three_pass() {
    static const bool v = [] {
        const char* e = getenv("LVLIP_FRAMES_3PASS");
        return e && e[0] == '1';
    }();
    return v;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? LVLIP_OK : lvlip_internal_hip_fail(e, what);
}

constexpr uint32_t kMaxFrames = LVLIP_MAX_BATCH / 2u;

}  // namespace

extern "C" {

size_t lvlip_frames_workspace_bytes(uint32_t n) {
    return (size_t)(32ull * n + round16(4ull * n) + round16(4ull * n) + 16u);
}

int lvlip_rx_verify_dev(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint32_t flags,
                        uint8_t* verdict, void* workspace, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || !verdict || !workspace || n > kMaxFrames ||
        ((uintptr_t)base & 15u) || ((uintptr_t)workspace & 15u))
        return LVLIP_EINVAL;
    if (!three_pass())
        return lvlip_internal_frames((flags & LVLIP_RX_VERIFY_L4) ? 2 : 1, base, frames, n, verdict,
                                     stream);
    hipStream_t s = (hipStream_t)stream;
    const Workspace w = carve(workspace, n);
    const uint32_t grid = (uint32_t)(((uint64_t)n + 255u) / 256u);
    hipLaunchKernelGGL(k_rx_plan, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, frames, n, flags,
                       w.descs, w.plan);
    int rc = launched("k_rx_plan");
    if (rc != LVLIP_OK) return rc;
    const uint32_t slots = (flags & LVLIP_RX_VERIFY_L4) ? 2u : 1u;
    lvlip_launch_cfg cfg = {LVLIP_KERNEL_AUTO, 0, 0, 0};  // headers (+ payloads): the flat sweep
    rc = lvlip_csum_batch_dev_ex(base, w.descs, slots * n, w.res, stream, &cfg);
    if (rc != LVLIP_OK) return rc;
    hipLaunchKernelGGL(k_rx_apply, dim3(grid), dim3(256), 0, s, w.plan, w.res, n, slots, verdict);
    return launched("k_rx_apply");
}

int lvlip_tx_checksum_dev(void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* status,
                          void* workspace, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || !workspace || n > kMaxFrames || ((uintptr_t)base & 15u) ||
        ((uintptr_t)workspace & 15u))
        return LVLIP_EINVAL;
    if (!three_pass()) return lvlip_internal_frames(0, base, frames, n, status, stream);
    hipStream_t s = (hipStream_t)stream;
    const Workspace w = carve(workspace, n);
    const uint32_t grid = (uint32_t)(((uint64_t)n + 255u) / 256u);
    hipLaunchKernelGGL(k_tx_plan, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, frames, n, w.descs,
                       w.plan);
    int rc = launched("k_tx_plan");
    if (rc != LVLIP_OK) return rc;
    lvlip_launch_cfg cfg = {LVLIP_KERNEL_AUTO, 0, 0, 0};
    rc = lvlip_csum_batch_dev_ex(base, w.descs, 2u * n, w.res, stream, &cfg);
    if (rc != LVLIP_OK) return rc;
    hipLaunchKernelGGL(k_tx_apply, dim3(grid), dim3(256), 0, s, (uint8_t*)base, frames, n, w.plan, w.res,
                       status);
    return launched("k_tx_apply");
}

}  // extern "C"
