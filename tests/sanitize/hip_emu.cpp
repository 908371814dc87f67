// tests/sanitize/hip_emu.cpp — TEST INFRASTRUCTURE ONLY: a CPU stand-in for
// the few HIP runtime calls of the host context (csum_ctx.cpp) and the host
// frame calls (frames_host.cpp), and for their device steps, so that those two
// files run under ASan + UBSan and TSan on a machine without a GPU
// (tests/test_sanitize_host.py; GPU sanitizers are not available on the
// MI355X pool, and tests/sanitize/ctx_san.cpp runs the same code with ASan on
// the real GPU).
//
// "Device" memory is host memory, copies are memcpy at once, streams and
// events do nothing (every enqueued step has already happened).  The device
// steps are restated with the library's own host-side decisions
// (skb_batch.c: lvlip_tx_plan / lvlip_rx_plan / lvlip_rx_apply, the same
// decisions as the kernels' FrameSrc, pinned to the oracle by the GPU tests)
// over the oracle's checksum: what is under test here is the host code around
// them (pieces, slots, offsets, descriptors, records, the apply and its undo,
// the pool threads), not the arithmetic.
#include <hip/hip_runtime_api.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lvlip_csum.h"
#include "lvlip_skb.h"

extern "C" uint16_t oracle_checksum(const void* addr, int count, int start_sum);

extern "C" {

const char* hipGetErrorString(hipError_t) { return "emulated"; }
hipError_t hipGetDeviceCount(int* n) {
    *n = 1;
    return hipSuccess;
}
hipError_t hipGetDevice(int* d) {
    *d = 0;
    return hipSuccess;
}
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned int) {
    *p = aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) {
    free(p);
    return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t bytes) { return hipHostMalloc(p, bytes, 0); }
hipError_t hipFree(void* p) {
    free(p);
    return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) {
    *d = h;
    return hipSuccess;
}
hipError_t hipHostRegister(void*, size_t, unsigned int) { return hipSuccess; }
hipError_t hipHostUnregister(void*) { return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    static char token;
    *s = (hipStream_t)&token;
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned int) {
    static char token;
    *e = (hipEvent_t)&token;
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind, hipStream_t) {
    memcpy(dst, src, bytes);
    return hipSuccess;
}

static thread_local char g_err[256];
const char* lvlip_last_hip_error(void) { return g_err; }
void lvlip_set_last_hip_error(const char* msg) { snprintf(g_err, sizeof g_err, "%s", msg ? msg : ""); }

// Group 2 (csum_kernels.hip) on the CPU: the oracle per descriptor
int lvlip_csum_batch_dev_ex(const void* base, const lvlip_csum_desc* d, uint32_t n, uint16_t* out, void*,
                            const lvlip_launch_cfg*) {
    if (n && (!base || !d || !out || ((uintptr_t)base & 15u))) return LVLIP_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        out[i] = oracle_checksum((const uint8_t*)base + d[i].offset, d[i].len, (int)d[i].start_sum);
    return LVLIP_OK;
}

// csum_kernels.hip's code-object load: nothing to load on the CPU
int lvlip_kernels_load(void) { return 0; }

// The frame calls' device step (csum_kernels.hip lvlip_frames_host_launch):
// mode 0 TX records, 1 RX header, 2 RX + L4.  Every byte a frame's decisions
// may read lies inside its descriptor's len, so an overread shows up in ASan.
int lvlip_frames_host_launch(int mode, const void* base, const lvlip_frame_desc* fd, uint32_t n, void* out,
                             void*) {
    if (n && (!base || !fd || !out || ((uintptr_t)base & 15u))) return LVLIP_EINVAL;
    for (uint32_t i = 0; i < n; ++i) {
        lvlip_frame f;
        f.head = (uint8_t*)base + fd[i].offset;
        f.len = fd[i].len;
        if (f.len == 0) f.head = nullptr;
        lvlip_csum_iov iov[2];
        uint16_t cs[2];
        if (mode == 0) {
            uint8_t* field[2];
            const uint32_t m = f.head ? lvlip_tx_plan(&f, 1, iov, field) : 0xFFFFFFFFu;
            uint64_t r = 0;
            if (m != 0xFFFFFFFFu) {
                r = 1ull << 40;
                for (uint32_t k = 0; k < m; ++k) {
                    const uint16_t c = oracle_checksum(iov[k].ptr, iov[k].len, (int)iov[k].start_sum);
                    if (field[k] == f.head + 24)
                        r |= c;
                    else
                        r |= ((uint64_t)c << 16) | ((uint64_t)(field[k] - f.head) << 32);
                }
            }
            ((uint64_t*)out)[i] = r;
        } else {
            uint8_t v = 0;
            uint32_t tag[2];
            const uint32_t m = lvlip_rx_plan(&f, 1, mode == 2 ? LVLIP_RX_VERIFY_L4 : 0u, &v, iov, tag);
            for (uint32_t k = 0; k < m; ++k) cs[k] = oracle_checksum(iov[k].ptr, iov[k].len, (int)iov[k].start_sum);
            lvlip_rx_apply(1, &v, m, tag, cs);
            ((uint8_t*)out)[i] = v;
        }
    }
    return LVLIP_OK;
}

}  // extern "C"
