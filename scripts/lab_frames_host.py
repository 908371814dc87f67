"""Lab: the host frame calls' pipeline (frames_host.cpp) under different
piece ramps, gather thread counts and sources, interleaved rounds in one
process, with LVLIP_FRAME_TRACE's per-step host times.

    python scripts/lab_frames_host.py OUT.json [ROUNDS]

The frames: bench.py's mixed frames (valid IPv4/TCP/ICMP, filled by the
device TX call), a 512K-frame prefix copied to host memory as one slab, and
the same frames scattered over 1616-B slots in random order.  Each config is
a context created under its environment (LVLIP_FIRST_PIECE, LVLIP_PIECE_MAX,
LVLIP_GATHER_THREADS, LVLIP_COPY_ORDER); each call is timed (wall, 1 warm-up
+ 3).  LAB_CONFIGS picks configs (comma list, default: all), LAB_SRC the
sources (comma list of slab, scattered, dma: the slab registered
LVLIP_REG_DMA; "all": slab and scattered; default scattered)."""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd")]

CONFIGS = {
    "default": {},
    "t8": {"LVLIP_GATHER_THREADS": "8"},
    "noramp": {"LVLIP_FIRST_PIECE": str(32 << 20)},
    "order0": {"LVLIP_COPY_ORDER": "0"},
}


def main(out_path, rounds=3):
    import torch

    import bench
    import lvlip

    dev = torch.device("cuda", 0)
    base, fd, pay = bench.mixed_frames_hbm(lvlip, torch, dev)
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    lvlip.tx_checksum_dev(base, fdt)
    torch.cuda.synchronize()
    n = min(fd.size, 1 << 19)
    fd = fd[:n]
    end = int(fd["offset"][n - 1]) + int(fd["len"][n - 1])
    host = base[: (end + 15) // 16 * 16].cpu().numpy().copy()
    del base
    stride = 1616
    slot = np.random.default_rng(7).permutation(n)
    scat = np.zeros(n * stride, np.uint8)
    for i in range(n):
        o, ln = int(fd["offset"][i]), int(fd["len"][i])
        scat[int(slot[i]) * stride:int(slot[i]) * stride + ln] = host[o:o + ln]

    def arr_of(buf, offsets):
        fr = np.zeros(n, dtype=[("head", "<u8"), ("len", "<u4"), ("pad", "<u4")])
        fr["head"] = buf.ctypes.data + offsets
        fr["len"] = fd["len"]
        return fr, ctypes.cast(fr.ctypes.data, ctypes.POINTER(lvlip.Frame))

    slab = arr_of(host, fd["offset"].astype(np.uint64))
    sc = arr_of(scat, slot.astype(np.uint64) * stride)
    lib = lvlip.lib()
    verdict = np.zeros(n, np.uint8)
    hb = 20 * n + int(pay["len"][:n].sum())
    res = {}
    os.environ["LVLIP_FRAME_TRACE"] = "1"
    names = os.environ.get("LAB_CONFIGS", ",".join(CONFIGS)).split(",")
    srcs = os.environ.get("LAB_SRC", "scattered")
    srcs = ["slab", "scattered"] if srcs == "all" else srcs.split(",")
    arrs = {"slab": slab[1], "scattered": sc[1], "dma": slab[1]}
    for rnd in range(rounds):
        for name in names:
            env = CONFIGS[name]
            for k, v in env.items():
                os.environ[k] = v
            try:
                ctx = lvlip.Context(0)
            finally:
                for k in env:
                    del os.environ[k]
            for src in srcs:
                arr = arrs[src]
                if src == "dma":
                    ctx.register(host, lvlip.REG_DMA)
                for call, fn in (("tx", lambda: lib.lvlip_tx_checksum(ctx._h, arr, n)),
                                 ("rx_l4", lambda: lib.lvlip_rx_verify(ctx._h, arr, n, 1, verdict.ctypes.data))):
                    assert fn() == 0
                    t0 = time.perf_counter()
                    for _ in range(3):
                        assert fn() == 0
                    ms = (time.perf_counter() - t0) / 3 * 1e3
                    key = f"{name}/{src}/{call}"
                    res.setdefault(key, []).append(round(hb / ms / 1e6, 2))
                    print(key, res[key], file=sys.stderr, flush=True)
                if src == "dma":
                    ctx.unregister(host)
            ctx.close()
    with open(out_path, "w") as f:
        json.dump({"GBps_checksummed": res, "frames": n}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
