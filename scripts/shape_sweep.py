#!/usr/bin/env python3
"""Launch shape vs packet length (diagnostic, GPU box): for uniform batches of
L-byte packets (16-B aligned slots, ~1.5 GB), times AUTO, k_stream shapes
(pieces in flight R x waves per CU w) and k_window shapes (R x w x group),
interleaved rounds in one process.  The tables behind AUTO's choice in
dispatch_one (csum_kernels.hip).

env: SH_LENS (default 512,768,1024,1500,2048,3000,4096,9000),
     SH_SHAPES (default 2x8,2x16,3x8,3x12,4x8,4x16), SH_ROUNDS (2),
     SH_WINDOW (k_window shapes RxWxG: pieces in flight, waves/CU, packets per group),
     SH_TOTAL (bytes of packet slots per length, default 1.5e9),
     SH_FLAT (k_flat2 unrolls, e.g. 8,4; default none),
     SH_WFLAT (k_wflat shapes UxWxD: loads per round, waves/CU, descriptors per tile),
     SH_LANE (k_lane shapes SxPxK[xM]: lanes per packet, packets per group, chunks per lane,
              load mode)
writes JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402


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
    lens = [int(x) for x in os.environ.get("SH_LENS", "512,768,1024,1500,2048,3000,4096,9000").split(",")]
    shapes = [tuple(int(v) for v in s.split("x"))
              for s in os.environ.get("SH_SHAPES", "2x8,2x16,3x8,3x12,4x8,4x16").split(",") if s]
    rounds = int(os.environ.get("SH_ROUNDS", "2"))
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    total = int(float(os.environ.get("SH_TOTAL", "1.5e9")))  # bytes of packet slots per length
    g = torch.Generator(device=dev)
    g.manual_seed(0x1E7E1C5)
    base = torch.randint(0, 256, (total + 16 * 9008,), dtype=torch.uint8, device=dev, generator=g)
    res = {}
    for L in lens:
        stride = (L + 15) // 16 * 16
        n = total // stride
        d = np.zeros(n, dtype=lvlip.DESC_DTYPE)
        d["offset"] = np.arange(n, dtype=np.uint64) * stride
        d["len"] = L
        d["start_sum"] = np.arange(n, dtype=np.uint32) * 2654435761
        descs = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        algo = n * L + 2 * n
        row = res.setdefault(str(L), {})
        variants = [("auto", 0, 0)] + [("wave", r, w) for r, w in shapes]
        # k_window shapes: SH_WINDOW = RxWxG,... (pieces in flight, waves/CU, group)
        for sh in filter(None, os.environ.get("SH_WINDOW", "").split(",")):
            r, w, gsz = (int(v) for v in sh.split("x"))
            variants.append(("window", r | (gsz << 8), w))
        for u in filter(None, os.environ.get("SH_FLAT", "").split(",")):
            variants.append(("flat", int(u), 0))
        for sh in filter(None, os.environ.get("SH_WFLAT", "").split(",")):
            u, w, dd = (int(v) for v in sh.split("x"))
            variants.append(("wflat", u | (dd << 8), w))
        for sh in filter(None, os.environ.get("SH_LANE", "").split(",")):
            v = [int(t) for t in sh.split("x")]
            sl, pl, ch, md = v + [0] * (4 - len(v))
            variants.append(("lane", pl | (ch << 8) | (sl << 16) | (md << 24), 0))
        for _ in range(rounds):
            for k, r, w in variants:
                def f():
                    lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), n, out.data_ptr(), s.cuda_stream,
                                    lvlip.KERNEL_NAMES[k], r, w, L)
                ms = timed(f, s)
                key = f"{k}-{r & 0xff}x{w}" + (f"g{(r >> 8) & 0xff}" if r >> 8 else "")  # g = group / tile
                key += f"s{(r >> 16) & 0xff}" if r >> 16 else ""  # k_lane: lanes per packet
                key += f"m{r >> 24}" if r >> 24 else ""  # k_lane: load mode
                row.setdefault(key, []).append(round(algo / ms / 1e6, 1))
        best = max(row, key=lambda k: max(row[k]))
        print(f"L={L:5d} n={n:8d} " + "  ".join(f"{k}:{max(v):7.1f}" for k, v in row.items()) + f"  best {best}",
              flush=True)
        del descs, out
    if out_path:
        json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
