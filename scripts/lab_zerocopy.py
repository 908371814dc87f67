"""Lab (diagnostic, not the product): which batch kernel reads packets in
HOST memory fastest over PCIe (the LVLIP_REG_ZEROCOPY path: the kernel reads
a registered region in place).  The batch is copied into pinned host memory
(torch pin_memory; its device address from hipHostGetDevicePointer), the
descriptors and results stay in HBM, and each kernel variant is launched on
it with HIP events around the launch alone; rounds interleave the variants.
Every variant's results are checked equal to the oracle's.

    python scripts/lab_zerocopy.py OUT.json [WORKLOAD] [ROUNDS] [hostmalloc|registered]

registered: the batch in plain pages pinned in place with hipHostRegister
(mapped), as lvlip_csum_register pins a stack's slab.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd"), os.path.join(ROOT, "oracle")]


def main(path, workload="tcp1500", rounds=3, memory="hostmalloc"):
    import torch

    import lvlip
    import pyoracle  # the checker (test infrastructure)
    import workloads

    K = lvlip
    variants = {
        "auto": (K.KERNEL_AUTO, 0, 0),
        # WINDOW: R pieces in flight (low byte) | packets per group << 8; waves/CU
        "window_r2g1_w12": (K.KERNEL_WINDOW, 2 | (1 << 8), 12),
        "window_r3_w8": (K.KERNEL_WINDOW, 3, 8),
        "window_r4_w16": (K.KERNEL_WINDOW, 4, 16),
        "window_r4_w24": (K.KERNEL_WINDOW, 4, 24),
        "wave_u2": (K.KERNEL_WAVE, 2, 0),
        "flat_u8": (K.KERNEL_FLAT, 8, 0),
        "flat_u4": (K.KERNEL_FLAT, 4, 0),
    }
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    b = workloads.make(workload)
    hostb = np.ascontiguousarray(b.host_bytes())
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    if memory == "hostmalloc":  # torch's pinned allocator (hipHostMalloc)
        pinned = torch.empty(hostb.size + 4096, dtype=torch.uint8).pin_memory()
        pinned[: hostb.size] = torch.from_numpy(hostb)
        hptr = pinned.data_ptr()
    else:  # plain pages pinned in place, as lvlip_csum_register does (hipHostRegisterMapped = 2)
        buf = np.empty(hostb.size + 8192, np.uint8)
        off = (-buf.ctypes.data) % 4096
        reg = buf[off:off + hostb.size + 4096]
        reg[: hostb.size] = hostb
        hptr = reg.ctypes.data
        assert hip.hipHostRegister(ctypes.c_void_p(hptr), reg.size, 2) == 0
    dptr = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(hptr), 0) == 0
    assert dptr.value % 16 == 0
    res_mem = memory
    descs = torch.from_numpy(np.ascontiguousarray(b.descs, dtype=lvlip.DESC_DTYPE).view(np.uint8).copy()).to(dev)
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    want = pyoracle.batch(hostb, b.descs, threads=min(16, os.cpu_count() or 1))
    hint = b.algo_bytes // b.n
    res = {"workload": workload, "memory": res_mem, "bytes": b.algo_bytes, "GBps": {}, "parity": {}}

    def launch(v):
        k, u, w = v
        lvlip.batch_dev(dptr.value, descs.data_ptr(), b.n, out.data_ptr(), stream.cuda_stream, k, u, w, hint)

    for name, v in variants.items():
        out.zero_()
        launch(v)
        torch.cuda.synchronize()
        ok = bool(np.array_equal(out.cpu().numpy().view(np.uint16), want))
        res["parity"][name] = ok
        assert ok, name
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for name, v in variants.items():
            ts = []
            for _ in range(3):
                e0.record(stream)
                launch(v)
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            gbps = round(b.algo_bytes / sorted(ts)[1] / 1e6, 2)
            res["GBps"].setdefault(name, []).append(gbps)
            print(name, res["GBps"][name], flush=True)
    if memory != "hostmalloc":
        hip.hipHostUnregister(ctypes.c_void_p(hptr))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "tcp1500",
         int(sys.argv[3]) if len(sys.argv) > 3 else 3, sys.argv[4] if len(sys.argv) > 4 else "hostmalloc")
