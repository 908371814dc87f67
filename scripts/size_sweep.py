#!/usr/bin/env python3
"""Kernel time vs batch size (diagnostic): fits t = a + bytes / B for the AUTO
checksum kernel and the lab read probe on the same buffers, so the fixed
per-launch cost (ramp + tail) is separated from the streaming rate.
Writes JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def timed(fn, stream, reps=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    wl = os.environ.get("LAB_WORKLOAD", "tcp1500")
    sizes = [int(x) for x in os.environ.get("LAB_SIZES", "131072,262144,524288,1048576,2097152,4194304").split(",")]
    kernels = os.environ.get("LAB_KERNELS", "auto").split(",")
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    rows = []
    for n in sizes:
        b = workloads.make(wl, n=n)
        base, descs, out = workloads.to_device(b, dev)
        hint = b.algo_bytes // max(b.n, 1)
        row = {"n": n, "algo_bytes": b.algo_bytes}
        for k in kernels:
            def f():
                lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                                lvlip.KERNEL_NAMES[k], 0, 0, hint)
            row[k + "_ms"] = min(timed(f, s) for _ in range(3))
        nb = base.numel() & ~1023
        row["probe_bytes"] = nb
        row["probe_ms"] = min(timed(lambda: lab.lvlip_lab_probe(base.data_ptr(), nb, sink.data_ptr(), 1, 8, 1,
                                                                 cus * 2, s.cuda_stream), s)
                              for _ in range(3))
        # the window-order read probe (4 KiB chunks dealt round robin)
        row["wprobe_ms"] = min(timed(lambda: lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(),
                                                                       4, 4, 1, cus * 2, s.cuda_stream), s)
                               for _ in range(3))
        print(json.dumps(row), flush=True)
        rows.append(row)
        del base, descs, out
        torch.cuda.empty_cache()
    fits = {}
    for key, bytes_key in [(k + "_ms", "algo_bytes") for k in kernels] + [("probe_ms", "probe_bytes"),
                                                                              ("wprobe_ms", "probe_bytes")]:
        x = np.array([r[bytes_key] for r in rows], dtype=np.float64)
        y = np.array([r[key] for r in rows], dtype=np.float64)
        slope, icpt = np.polyfit(x, y, 1)
        fits[key] = {"fixed_us": round(icpt * 1e3, 2), "stream_GBps": round(1 / slope / 1e6, 1)}
    print(json.dumps({"fits": fits}), flush=True)
    if out_path:
        with open(out_path, "w") as fh:
            json.dump({"workload": wl, "rows": rows, "fits": fits}, fh, indent=1)


if __name__ == "__main__":
    main()
