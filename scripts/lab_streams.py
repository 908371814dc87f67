#!/usr/bin/env python3
"""Does the stream (hardware queue) move the mixed batch's k_flat2 time? (GPU box)

The mixed line is bimodal across processes while buffer
placement inside a process does not move it (lab_buffer_placement.py).  Here,
in one process: the default stream, four new streams and two high-priority
streams (HIP maps streams onto its hardware queues round robin), AUTO timed on
each, 3 interleaved rounds of 20 launches after a clock settle; checks every
stream computes the same checksums.
  python scripts/lab_streams.py [out.json]
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
    wl = os.environ.get("ST_WORKLOAD", "mixed")
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b, dev)
    hint = b.algo_bytes // b.n
    streams = [("default", torch.cuda.current_stream(dev))]
    streams += [(f"new{i}", torch.cuda.Stream(dev)) for i in range(4)]
    streams += [(f"high{i}", torch.cuda.Stream(dev, priority=-1)) for i in range(2)]
    torch.cuda.synchronize()

    def run(s):
        lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream, 0, 0, 0, hint)

    ref = None
    for name, s in streams:
        out.zero_()
        torch.cuda.synchronize()
        run(s)
        torch.cuda.synchronize()
        got = out.cpu().numpy().copy()
        if ref is None:
            ref = got
        assert np.array_equal(got, ref), name
    for _ in range(600):
        run(streams[0][1])
    torch.cuda.synchronize()
    res = {n: [] for n, _ in streams}
    for _ in range(3):
        for name, s in streams:
            for _ in range(3):
                run(s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                run(s)
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(b.algo_bytes / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e9)
    rows = []
    for name, _ in streams:
        med = float(np.median(res[name]))
        rows.append({"stream": name, "GBps": round(med, 1), "rounds": [round(x, 1) for x in res[name]]})
        print(f"{wl} {name:8s} {med:8.1f} GB/s  {[round(x) for x in res[name]]}", flush=True)
    if len(sys.argv) > 1:
        json.dump({"workload": wl, "rows": rows}, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
