#!/usr/bin/env python3
"""Timeline of k_stream_dyn (diagnostic): per-streamer stamps (LVLIP_TAIL_TRACE)
— start, end — plus segments popped, grouped by XCD, by wave index in the
workgroup and by SIMD.  One process, tcp1500 (or AB_WORKLOAD)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

wl = os.environ.get("AB_WORKLOAD", "tcp1500")
trace = torch.zeros(65536 * 8, dtype=torch.int64, device="cuda")
os.environ["LVLIP_TAIL_TRACE"] = str(trace.data_ptr())
import lvlip  # noqa: E402
import workloads  # noqa: E402

b = workloads.make(wl)
base, descs, out = workloads.to_device(b)
hint = b.algo_bytes // b.n
for _ in range(5):
    trace.zero_()
    lvlip.batch_torch(base, descs, out, kernel=lvlip.KERNEL_WAVE_DYN, len_hint=hint)
torch.cuda.synchronize()
a = trace.cpu().numpy().reshape(-1, 8)
a = a[a[:, 0] != 0]
t0 = a[:, 0].min()
en = (a[:, 2] - t0) / 100.0
pops = a[:, 3]
x = a[:, 4]
wid = a[:, 6]
hw = a[:, 7]
simd = (hw >> 4) & 3
slot = hw & 15
print(f"{wl}: streamers {len(a)} end p10/p50/p90/max "
      f"{np.percentile(en, 10):.1f}/{np.percentile(en, 50):.1f}/{np.percentile(en, 90):.1f}/{en.max():.1f} us, "
      f"pops {pops.sum()}")
for name, key, k in [("xcc", x, 8), ("wid", wid, 4), ("simd", simd, 4)]:
    for q in range(k):
        m = key == q
        if m.any():
            print(f" {name}{q}: n {m.sum()} end p10/p50/p90/max {np.percentile(en[m], 10):.1f}/"
                  f"{np.percentile(en[m], 50):.1f}/{np.percentile(en[m], 90):.1f}/{en[m].max():.1f} pops {pops[m].sum()}")
# per (wid, simd) table of median end
print(" median end by wid x simd:")
for w in range(4):
    row = []
    for sd in range(4):
        m = (wid == w) & (simd == sd)
        row.append(f"{np.median(en[m]):6.1f}({m.sum():4d})" if m.any() else "   -   ")
    print("  wid", w, " ".join(row))
