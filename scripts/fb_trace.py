#!/usr/bin/env python3
"""Slot weights of WAVE launches over time (diagnostic, LVLIP_FB_TRACE): per
launch, each slot's weight (x 1/8 of the batch) and its longest block (us)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

trace = torch.zeros(65536 * 2, dtype=torch.int64, device="cuda")
os.environ["LVLIP_FB_TRACE"] = str(trace.data_ptr())
import lvlip  # noqa: E402
import workloads  # noqa: E402

wl = os.environ.get("AB_WORKLOAD", "tcp1500")
b = workloads.make(wl)
base, descs, out = workloads.to_device(b)
hint = b.algo_bytes // b.n
s = torch.cuda.current_stream()
for launch in range(int(os.environ.get("FB_LAUNCHES", "16"))):
    trace.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    lvlip.batch_torch(base, descs, out, kernel=lvlip.KERNEL_WAVE, len_hint=hint)
    e1.record(s)
    torch.cuda.synchronize()
    a = trace.cpu().numpy().reshape(-1, 2)
    a = a[a[:, 1] != 0]
    slot = a[:, 1] & 0xFFFFFFFF
    dur = (a[:, 0] & 0xFFFFFFFF) / 100.0
    w = (a[:, 0] >> 32) / (2 ** 24 / 8)
    row = []
    for q in range(8):
        m = slot == q
        row.append(f"{w[m][0]:.3f}/{dur[m].max():6.1f}" if m.any() else "-")
    print(f"launch {launch:2d} {e0.elapsed_time(e1) * 1000:7.1f} us | " + " ".join(row), flush=True)
