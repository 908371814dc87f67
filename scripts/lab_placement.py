#!/usr/bin/env python3
"""Placement lab (diagnostic): is blockIdx % 8 -> XCC_ID the same from one
launch to the next?  Runs the timeline probe back to back and prints, per
launch, the XCC of blocks 0..7 and whether every block b has xcc(b) ==
xcc(b % 8)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402

lab = lvlip.lab()
cus = torch.cuda.get_device_properties(0).multi_processor_count
nb = int(os.environ.get("PL_MB", "1572")) * 1000000 // 1024 * 1024
buf = torch.empty(nb, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")
ctr = torch.zeros(256, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for bpc in (2, 4, 5):
    grid = cus * bpc
    tl = torch.zeros(grid * 4 * 4, dtype=torch.int64, device="cuda")
    rows = []
    for launch in range(12):
        assert lab.lvlip_lab_probe_tl(buf.data_ptr(), nb, sink.data_ptr(), 0, 8, 0, ctr.data_ptr(),
                                      tl.data_ptr(), grid, s.cuda_stream) == 0
        torch.cuda.synchronize()
        a = tl.cpu().numpy().reshape(grid, 4, 4)
        x = (a[:, 0, 2] & 7).astype(int)  # xcc of wave 0 of each block
        first8 = x[:8].tolist()
        consistent = bool(np.all(x == np.array(first8 * ((grid + 7) // 8))[:grid]))
        # per slot end time (max over its waves)
        en = (a[:, :, 1] - a[:, :, 0].min()) / 100.0
        slot_end = [round(float(en[b::8].max()), 1) for b in range(8)]
        rows.append((first8, consistent, slot_end))
        print(f"bpc {bpc} launch {launch:2d}: xcc(b%8) {first8} all-consistent {consistent} "
              f"slot end {slot_end}", flush=True)
