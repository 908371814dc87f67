// csum_kernels.hip — gfx950 (CDNA4) kernels for level-ip's Internet checksum:
// Group 2 of include/lvlip_csum.h (device-resident batches) and the
// device-resident frame calls of include/lvlip_skb.h (f1, f2, f4).
//
// The arithmetic (bit-exact with src/utils.c:22-55) and the shared building
// blocks (the ring of k_window, the chunk sweep k_flat2) are in csum_dev.h.
//
// Kernels of the product (roofline: HBM read bandwidth; ~1 VALU op per loaded
// dword, no MFMA).  AUTO picks by the caller's length hint:
//   k_window  : from 896 B.  One wavefront per packet, persistent, a ring of
//               2-KiB pieces in flight per wave; packets dealt to the waves in
//               small groups round robin over the grid, so the waves in flight
//               read one narrow window of the batch.
//   k_flat2   : below 896 B and for unknown sizes (ragged batches: 20-B headers
//               next to payloads).  A chunk-balanced tile sweep over 16-B chunks
//               that crosses packet boundaries; segment sums by a DPP prefix
//               scan.  Also the frame calls' kernel (flat_src.h).
//   k_lane    : up to 32 B (IPv4 headers alone): a few lanes per packet.
//   k_rx_hdr  : the header-only RX frame call, one lane per frame (csum_dev.h).
//   k_echo_reply : f4, the RFC 1624 echo reply of verified requests, one lane
//               per frame (LVLIP_ECHO_FULL, icmpv4_reply's full sum, runs on
//               k_flat2 with a frame source).
// The A/B variants still under study (k_stream, k_wflat, k_flat2's other
// shapes and occupancies, the frame calls' store forms) live in
// liblvlip_lab.so (lab_kernels.hip); the ones rejected by >= 3 % were pruned
// in round 4.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "csum_dev.h"

namespace lvlip {

// ------------------------------------------------------------ k_window --
//
// ring_sweep (csum_dev.h) with the packets dealt in groups of G round robin
// over the grid.
template <int R, int G>
__global__ __launch_bounds__(256) void k_window(const uint8_t* __restrict__ base,
                                                const lvlip_csum_desc* __restrict__ descs,
                                                uint32_t n, uint16_t* __restrict__ out) {
    static_assert(G > 0, "k_window deals groups of G >= 1 packets");
    __shared__ uint4 s_win[SW_WAVES][2][64];
    ring_sweep<R, G, 0>(base, descs, n, out, s_win[uniform(threadIdx.x >> 6)]);
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

// k_echo_reply (f4, RFC 1624) is in csum_dev.h, so that the lab library
// can instantiate its store variants.
}  // namespace lvlip

// ======================================================== host side (C ABI) ==

namespace {

using lvlip_host::cu_count;
using lvlip_host::current_cus;
using lvlip_host::kLaunchMax;

thread_local char g_last_err[256] = "";

int hip_fail(hipError_t e, const char* what) {
    snprintf(g_last_err, sizeof g_last_err, "%s: %s", what, hipGetErrorString(e));
    return LVLIP_EHIP;
}

// k_window: waves_per_cu waves on every CU (fewer when the batch has fewer
// groups), R pieces in flight per wave, groups of G packets.  The grid stays a
// multiple of 8 blocks when it can, so the ranks are XCD-major.
template <int R, int G>
void launch_window_g(int waves_per_cu, hipStream_t s, const void* base, const lvlip_csum_desc* d,
                     uint32_t n, uint16_t* out) {
    uint64_t waves = (uint64_t)current_cus() * (uint64_t)waves_per_cu;
    const uint64_t ng = ((uint64_t)n + G - 1) / G;
    if (waves > ng) waves = ng;
    uint64_t grid = (waves + lvlip::SW_WAVES - 1) / lvlip::SW_WAVES;
    if (grid > 8) grid = grid & ~7ull;
    hipLaunchKernelGGL((lvlip::k_window<R, G>), dim3((uint32_t)grid), dim3(256), 0, s,
                       (const uint8_t*)base, d, n, out);
}

// Packets per group: the caller's (cfg->unroll >> 8), else by the length hint
// (DESIGN.md §4).
int window_group(int requested, int len_hint) {
    if (requested == 1 || requested == 2 || requested == 3 || requested == 4 || requested == 8)
        return requested;
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

// AUTO's k_lane range: hints below this many bytes (scripts/shape_sweep.py,
// DESIGN.md §4).
constexpr int kLaneHintMax = 33;

// LVLIP_KERNEL_AUTO's choice for n descriptors of average length `hint`
// (0 = unknown), measured on MI355X: the interleaved stream
// (k_window) on uniform MTU/jumbo segments, the flat sweep on mixed
// header/payload batches (it stays within ~10 % elsewhere, so it is the choice
// when sizes are unknown), lane groups for IPv4 headers alone.  wpc and unroll
// come in as the caller's (0 = choose) and leave as the launch's.
int auto_select(int hint, uint32_t n, int* unroll, int* wpc) {
    if (hint >= 896) {
        // the interleaved stream, shapes from scripts/shape_sweep.py
        // (DESIGN.md §4): 2 pieces in flight per wave; more waves per CU for
        // smaller packets (per-packet work); groups of 4 packets below
        // 1792 B, 2 up to 4 KiB, 3 for jumbo packets (power-of-two group
        // bytes such as 2 x 4096 measured 3 % slow)
        if (*wpc <= 0) *wpc = hint < 1280 ? 16 : (hint < 1792 ? 12 : 8);
        if (*unroll <= 0) {
            // ... but at least 16 groups per wave, or the last round of
            // groups leaves most waves idle (45 776 packets of 64 KiB: G 3
            // 6 698, G 1 6 974 GB/s)
            const uint64_t nw = (uint64_t)current_cus() * (uint64_t)*wpc;
            int g = hint < 1792 ? 4 : (hint < 4096 ? 2 : 3);
            while (g > 1 && (uint64_t)n < 16ull * (uint64_t)g * nw) --g;
            *unroll = 2 | (g << 8);
        }
        return LVLIP_KERNEL_WINDOW;
    }
    // up to 32 B (IPv4 headers alone, 20-32 B in 32-B slots): two lanes per
    // packet read every slot pair as one contiguous wave load, no tile plan
    // (20 / 32 B: 2 819 / 4 356 vs 2 474 / 4 121 GB/s for the flat sweep;
    // 36 B: 3 108 vs 3 469)
    if (hint > 0 && hint < kLaneHintMax) {
        *unroll = 4 | (2 << 8) | (2 << 16);
        return LVLIP_KERNEL_LANE;
    }
    // below ~900 B the flat sweep leads (uniform 512 / 768 B: 6 442 / 6 482
    // vs 3 973 / 5 916 GB/s for the stream), 4 loads per round below 176 B
    // (64 / 128 / 160 B: 4 926 / 6 134 / 6 148 vs 3 984 / 5 723 / 5 806 with
    // 8), 2 below 40 B, 8 otherwise (192 / 224 / 256 B: 6 340 / 6 387 / 6 348
    // vs 6 225 / 6 226 / 6 273 with 4, since U 8's descriptor prefetch;
    // mixed: 2-3 % ahead of 4)
    if (*unroll <= 0) *unroll = (hint > 0 && hint < 40) ? 2 : (hint > 0 && hint < 176) ? 4 : 8;
    return LVLIP_KERNEL_FLAT;
}

// One launch of the selected kernel over n <= kLaunchMax descriptors.
int dispatch_one(const void* base, const lvlip_csum_desc* descs, uint32_t n, uint16_t* out,
                 hipStream_t s, const lvlip_launch_cfg* cfg) {
    int kernel = cfg ? cfg->kernel : LVLIP_KERNEL_AUTO;
    int unroll = cfg ? cfg->unroll : 0;
    int wpc = cfg ? cfg->waves_per_cu : 0;
    const int hint = cfg ? cfg->len_hint : 0;
    if (kernel == LVLIP_KERNEL_AUTO) kernel = auto_select(hint, n, &unroll, &wpc);

    switch (kernel) {
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
            switch (r) {
                case 2: launch_window<2>(w, s, base, descs, n, out, group, hint); break;
                case 3: launch_window<3>(w, s, base, descs, n, out, group, hint); break;
                case 4: launch_window<4>(w, s, base, descs, n, out, group, hint); break;
                default: return LVLIP_EINVAL;
            }
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
        case LVLIP_KERNEL_FLAT: {
            // unroll = 64-chunk loads per round: 2, 4 or 8 (0 = 8: 92 VGPRs, 5
            // workgroups per CU with 8 KiB in flight per wave, 2-3 % ahead of 4
            // on mixed); groups in block order; at U 8 each
            // tile's threads prefetch the descriptors kFlatPrefetchTiles tiles
            // ahead into their XCD's L2 (csum_dev.h; at U 2 / 4 the four
            // registers it holds would cost a wave per SIMD, unmeasured).  The other orders, tile sizes,
            // occupancies and load policies measured against it are lab
            // variants (liblvlip_lab.so).
            if (unroll < 0) return LVLIP_EINVAL;
            if (unroll == 0) unroll = 8;
            const uint32_t grid = (uint32_t)(((uint64_t)n + lvlip::FT - 1) / lvlip::FT);
            switch (unroll) {
#define LVLIP_FLAT(UU)                                                                         \
    case UU:                                                                                   \
        hipLaunchKernelGGL((lvlip::k_flat2<UU, true, 2, lvlip::DescSrc, 1, false,                \
                                           UU == 8 ? lvlip::kFlatPrefetchTiles : 0>),             \
                           dim3(grid), dim3(lvlip::FT), 0, s, (const uint8_t*)base,                \
                           lvlip::DescSrc{descs, out}, n);                                        \
        break;
                LVLIP_FLAT(2) LVLIP_FLAT(4) LVLIP_FLAT(8)
#undef LVLIP_FLAT
                default: return LVLIP_EINVAL;
            }
            break;
        }
        default:
            // the retired and lab-only ids (1, 2, 4-7, 9: liblvlip_lab.so) and
            // anything else
            return LVLIP_EINVAL;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    return LVLIP_OK;
}

// The frame calls (include/lvlip_skb.h): the header-only RX call on k_rx_hdr,
// TX fill and RX + L4 on k_flat2 with a frame source in block order (RX + L4
// 4 loads per round; TX 8, its field stores `nt sc0 sc1`) (the
// measured alternatives are lab variants).
int launch_rx_hdr(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* out8,
                  hipStream_t s) {
    for (uint32_t f0 = 0; f0 < n;) {
        const uint32_t m = n - f0 < kLaunchMax ? n - f0 : kLaunchMax;
        hipLaunchKernelGGL(lvlip::k_rx_hdr<0>, dim3((m + 255u) / 256u), dim3(256), 0, s,
                           (const uint8_t*)base, frames + f0, m, out8 + f0);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_rx_hdr");
        f0 += m;
    }
    return LVLIP_OK;
}

constexpr uint32_t kMaxFrames = LVLIP_MAX_BATCH / 2u;  // two entries per frame

// k_window batches of many groups per wave run as launches of about this many
// groups per wave (lvlip_csum_batch_dev_ex)
constexpr uint64_t kWindowGroupsPerWave = 80;

}  // namespace

// Descriptors per launch for a batch of n with the resolved cfg c.
static uint32_t launch_piece(const lvlip_launch_cfg& c, uint32_t n) {
    // Long k_window launches lose rate: the persistent waves drift apart over
    // a launch, and the window of the batch they read widens.  A batch of more
    // than 1.5 x kWindowGroupsPerWave groups per wave goes out as launches of
    // about kWindowGroupsPerWave groups per wave, back to back on the stream,
    // which restart the waves in step (round 3's split_tune_once.sh:
    // 8M MTU segments 6 725 GB/s in one launch, 6 866 in 8; 64M 6 450 in one,
    // 6 850 in 64; 1M jumbo 7 113 in one, 7 146 in 2).  The configs' 1M MTU
    // batch (85 groups per wave) stays one launch.  Results are the same bits:
    // each launch checksums its own descriptor range.
    uint32_t piece = kLaunchMax;
    if (c.kernel == LVLIP_KERNEL_WINDOW) {
        const int g = window_group((c.unroll >> 8) & 0xff, c.len_hint);
        const uint64_t waves = (uint64_t)current_cus() * (uint64_t)(c.waves_per_cu > 0 ? c.waves_per_cu : 8);
        const uint64_t per_launch = waves * (uint64_t)g * kWindowGroupsPerWave;
        if ((uint64_t)n > per_launch + per_launch / 2u) {
            const uint64_t parts = ((uint64_t)n + per_launch / 2u) / per_launch;
            const uint64_t per = ((uint64_t)n + parts - 1) / parts;
            if (per < piece) piece = (uint32_t)per;
        }
    }
    return piece;
}

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

// Hidden: the host context (csum_ctx.cpp, frames_host.cpp) records its HIP
// failures here too, and Group 4 hands a worker thread's message to the
// calling thread.
void lvlip_set_last_hip_error(const char* msg) { snprintf(g_last_err, sizeof g_last_err, "%s", msg ? msg : ""); }

// Hidden: loads this file's code object on the current device (every product
// kernel is in it), so a context's first call does not pay the load inside
// its first launch (~2 ms, measured as the first 64-frame call's time outside
// its host steps).  Launches nothing.
int lvlip_kernels_load(void) {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&lvlip::k_window<3, 4>)) == hipSuccess ? 0 : -1;
}

int lvlip_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

uint32_t lvlip_batch_launches(uint32_t n, const lvlip_launch_cfg* cfg) {
    if (n == 0 || n > LVLIP_MAX_BATCH) return 0;
    lvlip_launch_cfg c = cfg ? *cfg : lvlip_launch_cfg{LVLIP_KERNEL_AUTO, 0, 0, 0};
    if (c.kernel == LVLIP_KERNEL_AUTO) c.kernel = auto_select(c.len_hint, n, &c.unroll, &c.waves_per_cu);
    const uint32_t piece = launch_piece(c, n);
    return (uint32_t)(((uint64_t)n + piece - 1) / piece);
}

int lvlip_auto_kernel(int32_t len_hint, uint32_t n, lvlip_launch_cfg* resolved) {
    int unroll = 0, wpc = 0;
    const int k = auto_select(len_hint, n, &unroll, &wpc);
    if (resolved) {
        resolved->kernel = k;
        resolved->unroll = unroll;
        resolved->waves_per_cu = wpc;
        resolved->len_hint = len_hint;
    }
    return k;
}

int lvlip_csum_batch_dev_ex(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                            uint16_t* out, void* stream, const lvlip_launch_cfg* cfg) {
    if (n == 0) return LVLIP_OK;
    if (!base || !descs || !out || n > LVLIP_MAX_BATCH) return LVLIP_EINVAL;
    if (((uintptr_t)base & 15u) != 0) return LVLIP_EINVAL;
    // AUTO resolved once for the whole batch (its shape depends on n)
    lvlip_launch_cfg c = cfg ? *cfg : lvlip_launch_cfg{LVLIP_KERNEL_AUTO, 0, 0, 0};
    if (c.kernel == LVLIP_KERNEL_AUTO) c.kernel = auto_select(c.len_hint, n, &c.unroll, &c.waves_per_cu);
    const uint32_t piece = launch_piece(c, n);
    for (uint32_t lo = 0; lo < n;) {
        const uint32_t m = n - lo < piece ? n - lo : piece;
        const int rc = dispatch_one(base, descs + lo, m, out + lo, (hipStream_t)stream, &c);
        if (rc != LVLIP_OK) return rc;
        lo += m;
    }
    return LVLIP_OK;
}

int lvlip_csum_batch_dev(const void* base, const lvlip_csum_desc* descs, uint32_t n,
                         uint16_t* out, void* stream) {
    return lvlip_csum_batch_dev_ex(base, descs, n, out, stream, nullptr);
}

// ---- f1/f2/f4 on device-resident frames (include/lvlip_skb.h) ----

size_t lvlip_frames_workspace_bytes(uint32_t) { return 0; }

int lvlip_rx_verify_dev(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint32_t flags,
                        uint8_t* verdict, void* /*workspace*/, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || !verdict || n > kMaxFrames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    // RX + L4: U 4 in block order (round 3, same process: 253 vs 257 us for
    // quarters on 2M frames, U 8 258-259; profiles/r03_ab_frames_shape.json)
    // launch_rx_hdr records its own HIP error (hip_fail clears it with
    // hipGetLastError); launch_frames_flat leaves it pending (hipPeekAtLastError)
    if (!(flags & LVLIP_RX_VERIFY_L4)) return launch_rx_hdr(base, frames, n, verdict, s);
    const int rc = lvlip::launch_frames_flat<lvlip::FR_RX_L4, 4, 2>(base, frames, n, verdict, s, true);
    if (rc == LVLIP_EHIP) return hip_fail(hipGetLastError(), "frame call");
    return rc;
}

int lvlip_tx_checksum_dev(void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* status,
                          void* /*workspace*/, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || n > kMaxFrames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    // U 8 in block order (round 3, same process: 369 vs 374 us for U 4
    // quarters on 2M frames; profiles/r03_ab_frames_shape.json); the field
    // stores `nt sc0 sc1` (round 4, same process, 7 rounds on 2M frames:
    // 364.1 vs 369.6 us for nt, 392.7 plain, 385 sc1, 420 / 410 whole 32-B /
    // 64-B blocks; profiles/r04_tx_store.json)
    const int rc = lvlip::launch_frames_flat<lvlip::FR_TX, 8, 2, 0, 0, 6>(base, frames, n, status,
                                                                         (hipStream_t)stream, true);
    if (rc == LVLIP_EHIP) return hip_fail(hipGetLastError(), "frame call");
    return rc;
}

// The host frame calls' device step (frames_host.cpp; hidden, not part of the
// ABI): mode 0 TX records (FrameSrc<FR_TX_REC>, the TX fill's shape, u64 per
// frame into `out`), 1 RX header and 2 RX + L4 (the verdicts, as
// lvlip_rx_verify_dev).  `base` and `frames` may be device addresses of
// mapped host memory, and so may `out`.
int lvlip_frames_host_launch(int mode, const void* base, const lvlip_frame_desc* frames, uint32_t n,
                             void* out, void* stream) {
    if (mode == 1) return lvlip_rx_verify_dev(base, frames, n, 0u, (uint8_t*)out, nullptr, stream);
    if (mode == 2) return lvlip_rx_verify_dev(base, frames, n, LVLIP_RX_VERIFY_L4, (uint8_t*)out, nullptr, stream);
    if (mode != 0) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || !out || n > kMaxFrames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    const int rc = lvlip::launch_frames_flat<lvlip::FR_TX_REC, 8, 2>(base, frames, n, (uint8_t*)out,
                                                                     (hipStream_t)stream, false);
    if (rc == LVLIP_EHIP) return hip_fail(hipGetLastError(), "frame call");
    return rc;
}

int lvlip_icmp_echo_reply_dev_ex(void* base, const lvlip_frame_desc* frames, uint32_t n, uint32_t flags,
                                 uint8_t* status, void* stream) {
    if (flags & ~LVLIP_ECHO_FULL) return LVLIP_EINVAL;
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (flags & LVLIP_ECHO_FULL) {
        // the whole messages: the flat sweep with a frame source (round 5;
        // one lane per frame summing its message alone ran 3-4x slower,
        // DESIGN.md §9)
        if (n > kMaxFrames * 2u) return LVLIP_EINVAL;
        const int rc = lvlip::launch_frames_flat<lvlip::FR_ECHO, 8, 2, 0, 0, lvlip::kEchoStore>(base, frames, n, status, s, false);
        if (rc == LVLIP_EHIP) return hip_fail(hipGetLastError(), "k_flat2 echo");
        return rc;
    }
    for (uint32_t f0 = 0; f0 < n;) {
        const uint32_t m = n - f0 < kLaunchMax ? n - f0 : kLaunchMax;
        hipLaunchKernelGGL((lvlip::k_echo_reply<lvlip::kEchoStore, 3>), dim3((m + 255u) / 256u), dim3(256), 0, s,
                           (uint8_t*)base, frames + f0, m, status ? status + f0 : nullptr);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_echo_reply");
        f0 += m;
    }
    return LVLIP_OK;
}

int lvlip_icmp_echo_reply_dev(void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* status,
                              void* stream) {
    return lvlip_icmp_echo_reply_dev_ex(base, frames, n, 0u, status, stream);
}

}  // extern "C"
