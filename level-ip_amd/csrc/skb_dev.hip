// skb_dev.hip — f1/f2 of SURVEY.md §8f for frames already in HBM
// (include/lvlip_skb.h, "device-resident frames").
//
// Each call is one launch of the flat sweep (csum_kernels.hip, k_flat2) with a
// frame source (flat_src.h): phase 1 parses every frame's Ethernet/IPv4 header
// into its checksum entries with the decisions of skb_batch.c (which cites the
// reference line of each), phase 4 turns the results into ip_rcv's verdict (RX)
// or stores them raw into the frame's checksum fields (TX).  No plan,
// descriptor or result array goes through HBM; DESIGN.md §9 has the
// measurements against the earlier plan / batch / apply pipeline.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

// csum_kernels.hip: mode 0 TX fill, 1 RX header verify, 2 RX with L4
int lvlip_internal_frames(int mode, const void* base, const lvlip_frame_desc* frames, uint32_t n,
                          uint8_t* out8, void* stream);

namespace {

constexpr uint32_t kMaxFrames = LVLIP_MAX_BATCH / 2u;  // two entries per frame

}  // namespace

extern "C" {

size_t lvlip_frames_workspace_bytes(uint32_t) { return 0; }

int lvlip_rx_verify_dev(const void* base, const lvlip_frame_desc* frames, uint32_t n, uint32_t flags,
                        uint8_t* verdict, void* /*workspace*/, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || !verdict || n > kMaxFrames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    return lvlip_internal_frames((flags & LVLIP_RX_VERIFY_L4) ? 2 : 1, base, frames, n, verdict, stream);
}

int lvlip_tx_checksum_dev(void* base, const lvlip_frame_desc* frames, uint32_t n, uint8_t* status,
                          void* /*workspace*/, void* stream) {
    if (n == 0) return LVLIP_OK;
    if (!base || !frames || n > kMaxFrames || ((uintptr_t)base & 15u)) return LVLIP_EINVAL;
    return lvlip_internal_frames(0, base, frames, n, status, stream);
}

}  // extern "C"
