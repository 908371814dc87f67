#!/usr/bin/env python3
"""Lab: how k_stream's launch time evolves from a cold start (GPU box).

The driver's round-end bench runs `bench.py --steps 20 --warmup 5`: 25 launches
of ~0.24 ms, a 5 ms timed region right after the batch is generated.  This
script times every one of the first launches on its own (an event pair per
launch, no host syncs between them) in a fresh process, then repeats the
bench's 5+20 pattern after an idle gap, to see whether the first milliseconds
of GPU work run at the steady-state rate.

  python scripts/warm_curve.py [--workload tcp1500] [--launches 400]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def per_launch(step, stream, k):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    ev[0].record(stream)
    for i in range(k):
        step()
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    return np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(k)])


def bench_pattern(step, stream, warm, steps):
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="tcp1500")
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--kernel", default="auto")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    b = workloads.make(a.workload)
    base, descs, out = workloads.to_device(b, dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    hint = b.algo_bytes // b.n
    kern = lvlip.KERNEL_NAMES[a.kernel]

    def step():
        lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), stream.cuda_stream,
                        kern, 0, 0, hint)

    gb = b.algo_bytes / 1e6
    t = per_launch(step, stream, a.launches)
    print(f"cold per-launch ms, first 12: {np.round(t[:12], 4).tolist()}", flush=True)
    for lo in (0, 5, 25, 50, 100, 200, 300):
        hi = min(lo + 25, t.size)
        if lo < hi:
            m = float(np.mean(t[lo:hi]))
            print(f"  launches {lo:4d}-{hi - 1:4d}: mean {m:.4f} ms = {gb / m:.0f} GB/s", flush=True)
    for gap in (0.0, 1.0, 3.0):
        time.sleep(gap)
        ms = bench_pattern(step, stream, 5, 20)
        ms2 = bench_pattern(step, stream, 50, 200)
        print(f"after {gap:.0f} s idle: 5+20 -> {gb / ms:.0f} GB/s; then 50+200 -> {gb / ms2:.0f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
