"""Lab (diagnostic, not the product): which threads of the process spend the
host CPU time of the host frame calls (bench.py --frames reports the process
total as cpu_ns_per_frame).  512K of the mixed config's frames in host memory,
each call R times from the slab / a DMA region / a zero-copy region, with the
per-thread CPU time (utime + stime of /proc/self/task/*/stat) before and after.

    python scripts/lab_cpu_threads.py OUT.json [R]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd")]

TICK = os.sysconf("SC_CLK_TCK")


def threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            with open(f"/proc/self/task/{tid}/comm") as f:
                comm = f.read().strip()
        except OSError:
            continue
        rest = st[st.rindex(")") + 2:].split()
        out[int(tid)] = (comm, (int(rest[11]) + int(rest[12])) / TICK)
    return out


def main():
    path = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    import torch

    import bench
    import lvlip

    dev = torch.device("cuda", 0)
    base, fd, pay = bench.mixed_frames_hbm(lvlip, torch, dev)
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    lvlip.tx_checksum_dev(base, fdt)
    torch.cuda.synchronize()
    nh = 1 << 19
    end = int(fd["offset"][nh - 1]) + int(fd["len"][nh - 1])
    host = base[: (end + 15) // 16 * 16].cpu().numpy().copy()
    fd = fd[:nh]
    del base, fdt
    import ctypes

    fr = np.zeros(nh, dtype=[("head", "<u8"), ("len", "<u4"), ("pad", "<u4")])
    fr["head"] = host.ctypes.data + fd["offset"].astype(np.uint64)
    fr["len"] = fd["len"]
    arr = ctypes.cast(fr.ctypes.data, ctypes.POINTER(lvlip.Frame))
    lib = lvlip.lib()
    verdict = np.zeros(nh, np.uint8)
    res = {"frames": nh, "reps": reps, "env": {k: v for k, v in os.environ.items() if k.startswith("LVLIP_")}}
    with lvlip.Context(0) as ctx:
        for src, flag in (("slab", None), ("dma", lvlip.REG_DMA), ("zerocopy", lvlip.REG_ZEROCOPY)):
            if flag is not None:
                ctx.register(host, flag)
            for name, call in (("tx_fill", lambda: lib.lvlip_tx_checksum(ctx._h, arr, nh)),
                               ("rx_header_l4", lambda: lib.lvlip_rx_verify(ctx._h, arr, nh, lvlip.RX_VERIFY_L4,
                                                                            verdict.ctypes.data))):
                assert call() == 0
                a, c0, t0 = threads(), time.process_time(), time.perf_counter()
                for _ in range(reps):
                    assert call() == 0
                wall = time.perf_counter() - t0
                cpu = time.process_time() - c0
                b = threads()
                per = {}
                for tid, (comm, t) in b.items():
                    d = t - a.get(tid, (comm, 0.0))[1]
                    if d > 0:
                        key = "main" if tid == os.getpid() else comm
                        per[key] = per.get(key, 0.0) + d
                top = sorted(per.items(), key=lambda kv: -kv[1])[:8]
                r = {"ms": round(wall / reps * 1e3, 3), "cpu_ns_per_frame": round(cpu / reps / nh * 1e9, 2),
                     "threads_ns_per_frame": {k: round(v / reps / nh * 1e9, 2) for k, v in top}}
                res[f"{src}_{name}"] = r
                print(src, name, r, flush=True)
            if flag is not None:
                ctx.unregister(host)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
