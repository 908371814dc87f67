#!/usr/bin/env python3
"""Cross-XCD atomicity lab (diagnostic): do returning atomics on hipMalloc'd
(coarse-grained) memory hand out unique tickets across the eight XCDs?  Prints,
per mode, the number of duplicate tickets, per-XCD counts and the time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402


def main():
    lab = lvlip.lab()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    blocks, k = cus * 4, 8
    waves = blocks * 4
    s = torch.cuda.current_stream()
    for mode, name in [(0, "agent sc0"), (1, "system sc0 sc1"), (2, "asm sc0 sc1")]:
        for rep in range(2):
            ctr = torch.zeros(64, dtype=torch.int32, device="cuda")
            tk = torch.full((waves * k * 2,), -1, dtype=torch.int32, device="cuda")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert lab.lvlip_lab_atomics(ctr.data_ptr(), tk.data_ptr(), mode, blocks, k, s.cuda_stream) == 0
            e1.record(s)
            torch.cuda.synchronize()
            a = tk.cpu().numpy().view(np.uint32).reshape(-1, 2)
            t = a[:, 0]
            u = np.unique(t)
            dup = t.size - u.size
            final = int(ctr[0].item())
            print(f"mode {mode} ({name}) rep {rep}: tickets {t.size} unique {u.size} dup {dup} "
                  f"max {int(t.max())} final ctr {final} time {e0.elapsed_time(e1) * 1000:.1f} us "
                  f"per-xcc {np.bincount(a[:, 1], minlength=8).tolist()}", flush=True)


if __name__ == "__main__":
    main()
