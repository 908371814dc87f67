#!/usr/bin/env python3
"""Lab (round 4): is there locality between an XCD and parts of HBM?

  python scripts/lab_numa.py out.json

The tcp1500 buffer (1.5 GB) is read by lvlip_lab_probe_xcd: units of CB bytes
with class (address / CB) mod 8, each class read only by the waves of one
block slot (block b runs on XCD b % 8), slot = (class + shift) mod 8; 8 waves
per CU, 4 KiB chunks of each slot's stream dealt round robin to its waves.
For every CB (256 B .. 2 MiB) all eight shifts are timed in interleaved
rounds, beside the plain window probe (bench diag window_c4).  If the memory
behind some address classes were nearer to some XCDs, one shift per CB would
read measurably faster than the others; if the eight agree, an XCD-aware deal
of packets by address buys nothing."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def timed(fn, s, reps=10, warm=2):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    out_path = sys.argv[1]
    dev = torch.device("cuda", 0)
    b = workloads.make("tcp1500")
    base, _, _ = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    lab.lvlip_lab_probe_xcd.restype = ctypes.c_int
    lab.lvlip_lab_probe_xcd.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nb = base.numel() & ~((1 << 21) * 8 - 1)  # whole rounds of 8 x 2 MiB units
    blocks = cus * 2
    res = {}
    for rnd in range(3):
        ms = timed(lambda: lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(), 4, 4, 1, blocks,
                                                     s.cuda_stream), s)
        res.setdefault("window_c4", []).append(round(nb / ms / 1e6, 1))
        for lg in (8, 10, 12, 13, 14, 16, 18, 21):
            for sh in range(8):
                rc = lab.lvlip_lab_probe_xcd(base.data_ptr(), nb, sink.data_ptr(), lg, sh, blocks, s.cuda_stream)
                assert rc == 0, rc
                ms = timed(lambda: lab.lvlip_lab_probe_xcd(base.data_ptr(), nb, sink.data_ptr(), lg, sh, blocks,
                                                           s.cuda_stream), s)
                res.setdefault(f"cb{1 << lg}_s{sh}", []).append(round(nb / ms / 1e6, 1))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print("window_c4", med["window_c4"], flush=True)
    summary = {}
    for lg in (8, 10, 12, 13, 14, 16, 18, 21):
        row = [med[f"cb{1 << lg}_s{sh}"] for sh in range(8)]
        summary[1 << lg] = {"by_shift_GBps": row, "spread_pct": round((max(row) - min(row)) / min(row) * 100, 2)}
        print(f"CB {1 << lg:8d}: " + " ".join(f"{x:7.1f}" for x in row) + f"  spread {summary[1 << lg]['spread_pct']} %",
              flush=True)
    with open(out_path, "w") as f:
        json.dump({"bytes": nb, "blocks": blocks, "median_GBps": med, "rounds": res, "by_cb": summary}, f, indent=1)


if __name__ == "__main__":
    main()
