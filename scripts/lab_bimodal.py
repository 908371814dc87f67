#!/usr/bin/env python3
"""Lab: AUTO's hint-only choice on bimodal batches (GPU box).

AUTO picks the kernel from the average length alone (dispatch_one).  A batch of
small and MTU packets mixed can have an average above the flat sweep's range
while a third of its packets are tiny, which is where the stream kernel is
weakest.  For a few small-packet fractions this times AUTO (with the batch's
average as the hint), the flat sweep and the stream shapes, checking that all
give the same checksums.

  python scripts/lab_bimodal.py [out.json]
"""
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
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(7)
    total = int(1.5e9)
    g = torch.Generator(device=dev)
    g.manual_seed(0x1E7E1C5)
    base = torch.randint(0, 256, (total + 4096,), dtype=torch.uint8, device=dev, generator=g)
    res = {}
    for small_frac in (0.1, 0.3, 0.5):
        # lengths: small ones U[40, 100], large ones U[1400, 1460]
        n_est = int(total / (small_frac * 70 + (1 - small_frac) * 1430 + 16))
        small = rng.random(n_est) < small_frac
        ln = np.where(small, rng.integers(40, 101, n_est), rng.integers(1400, 1461, n_est)).astype(np.int64)
        slots = (ln + 15) // 16 * 16
        off = np.concatenate([[0], np.cumsum(slots)[:-1]])
        keep = off + slots <= total
        d = np.zeros(int(keep.sum()), dtype=lvlip.DESC_DTYPE)
        d["offset"], d["len"] = off[keep], ln[keep]
        d["start_sum"] = rng.integers(0, 2**32, d.size, dtype=np.uint64).astype(np.uint32)
        n = d.size
        descs = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        algo = int(d["len"].sum()) + 2 * n
        hint = int(d["len"].mean())
        variants = [("auto", 0, 0), ("flat", 8, 0), ("flat", 4, 0), ("window", 2 | (4 << 8), 16),
                    ("window", 2 | (4 << 8), 12)]
        outs, row = {}, {}
        for _ in range(2):
            for k, u, w in variants:
                out = outs.setdefault((k, u, w), torch.empty(n, dtype=torch.int16, device=dev))

                def f():
                    lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), n, out.data_ptr(), s.cuda_stream,
                                    lvlip.KERNEL_NAMES[k], u, w, hint)
                ms = timed(f, s)
                row.setdefault(f"{k}-{u:#x}-w{w}", []).append(round(algo / ms / 1e6, 1))
        ref = outs[variants[1]]
        assert all(torch.equal(o, ref) for o in outs.values()), "variants disagree"
        res[str(small_frac)] = {"n": n, "hint": hint, "GBps": {k: max(v) for k, v in row.items()}}
        print(small_frac, n, hint, res[str(small_frac)]["GBps"], flush=True)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
