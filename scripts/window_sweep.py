#!/usr/bin/env python3
"""Lab: k_window launch shapes against k_stream (AUTO) on one resident batch.

Group size G is chosen through the length hint (window_group in
csum_kernels.hip: 5000 -> 1, 1500 -> 2, 1000 -> 4, 300 -> 8; LVLIP_WINDOW_GROUP
overrides it for the whole process).  Interleaved rounds in one process, after
a clock settle; prints the median GB/s of algorithmic bytes per variant.

  LAB_WORKLOAD=tcp1500 python scripts/window_sweep.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402

HINT_G = {5000: 1, 1500: 2, 1000: 4, 300: 8}


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
    dev = torch.device("cuda", 0)
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    hint = b.algo_bytes // b.n
    shapes = [(g, r, w) for g in (5000, 1500, 1000) for r in (2, 3, 4) for w in (8,)]
    shapes += [(1500, 3, 12), (1500, 2, 12), (5000, 2, 12), (1500, 3, 6), (1500, 4, 6)]
    variants = [("auto", 0, 0, hint)] + [("window", r, w, g) for g, r, w in shapes]

    def mk(k, u, w, h):
        return lambda: lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),
                                       s.cuda_stream, lvlip.KERNEL_NAMES[k], u, w, h)
    ref = None
    res = {}
    timed(mk("auto", 0, 0, hint), s, reps=500)  # clock settle
    for rnd in range(3):
        for k, u, w, h in variants:
            f = mk(k, u, w, h)
            ms = timed(f, s)
            key = "stream auto" if k == "auto" else f"window G{HINT_G[h]} R{u} w{w}"
            res.setdefault(key, []).append(b.algo_bytes / ms / 1e6)
            if rnd == 0:  # every variant computes the same checksums
                torch.cuda.synchronize()
                got = out.cpu().numpy().copy()
                if ref is None:
                    ref = got
                assert np.array_equal(got, ref), key
        print(f"round {rnd} done", flush=True)
    summary = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in sorted(summary.items(), key=lambda kv: -kv[1]):
        print(f"{k:28s} {v:8.1f} GB/s", flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"workload": wl, "median_GBps": summary, "rounds": res}, f, indent=1)


if __name__ == "__main__":
    main()
