#!/usr/bin/env python3
"""Which buffer's placement moves the mixed batch's k_flat2 time (GPU box).

The mixed bench line is bimodal across processes (6.24 vs 6.42 TB/s, same
box, same data; the streaming read probes over the same buffer do not move).
In one process: 2 copies of the packet buffer, 3 of the descriptors, 3 of the
result buffer (each copy a separate allocation, with spacer allocations of
odd sizes between them), AUTO timed on every combination, 3 interleaved
rounds of 20 launches; prints the median GB/s per combination, and checks
every combination computes the same checksums.
  python scripts/lab_buffer_placement.py [out.json]
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


def main():
    dev = torch.device("cuda", 0)
    b = workloads.make("mixed")
    s = torch.cuda.current_stream(dev)
    hint = b.algo_bytes // b.n
    spacers, bases, descs, outs = [], [], [], []
    for k in range(2):
        bb, dd, oo = workloads.to_device(b, dev)
        bases.append(bb)
        descs.append(dd)
        outs.append(oo)
        spacers.append(torch.empty((k + 1) * 37 << 20, dtype=torch.uint8, device=dev))
    descs.append(descs[0].clone())
    spacers.append(torch.empty(91 << 20, dtype=torch.uint8, device=dev))
    outs.append(torch.empty_like(outs[0]))
    torch.cuda.synchronize()
    combos = [(i, j, k) for i in range(len(bases)) for j in range(len(descs)) for k in range(len(outs))]

    def run(c):
        i, j, k = c
        lvlip.batch_dev(bases[i].data_ptr(), descs[j].data_ptr(), b.n, outs[k].data_ptr(), s.cuda_stream,
                        0, 0, 0, hint)

    ref = None
    for c in combos:
        run(c)
        torch.cuda.synchronize()
        got = outs[c[2]].cpu().numpy().copy()
        if ref is None:
            ref = got
        assert np.array_equal(got, ref), c
    # settle the clocks
    for _ in range(600):
        run(combos[0])
    torch.cuda.synchronize()
    res = {c: [] for c in combos}
    for _ in range(3):
        for c in combos:
            for _ in range(3):
                run(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                run(c)
            e1.record(s)
            torch.cuda.synchronize()
            res[c].append(b.algo_bytes / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e9)
    rows = []
    for c in combos:
        med = float(np.median(res[c]))
        addr = (hex(bases[c[0]].data_ptr()), hex(descs[c[1]].data_ptr()), hex(outs[c[2]].data_ptr()))
        rows.append({"base": c[0], "descs": c[1], "out": c[2], "GBps": round(med, 1),
                     "rounds": [round(x, 1) for x in res[c]], "addr": addr})
        print(f"base {c[0]} descs {c[1]} out {c[2]}  {med:8.1f} GB/s  {addr}", flush=True)
    if len(sys.argv) > 1:
        json.dump({"workload": "mixed", "rows": rows}, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
