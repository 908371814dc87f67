#!/usr/bin/env python3
"""A/B of k_rx_hdr's descriptor prefetch (GPU box): the header-only RX call on
the mixed config's 2M frames (bench.py --frames' frames), the product against
the lab's k_rx_hdr with the frame descriptors P x 160 blocks ahead prefetched
(lvlip_lab_frames_dev mode 3), interleaved rounds in one process; checks all
verdicts agree.
  python scripts/rx_pf_ab.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    b = workloads.make("mixed")
    base, _, _ = workloads.to_device(b, dev)
    hdr, pay = b.descs[0::2], b.descs[1::2]
    n = hdr.size
    fstart = torch.from_numpy((hdr["offset"] - 14).astype(np.int64)).to(dev)
    iplen = torch.from_numpy((20 + pay["len"]).astype(np.int64)).to(dev)
    proto = torch.from_numpy(np.where(pay["start_sum"] != 0, 6, 1).astype(np.int64)).to(dev)

    def put(k, vals):
        base[fstart + k] = vals.to(torch.uint8) if torch.is_tensor(vals) else vals

    put(12, 0x08), put(13, 0x00), put(14, 0x45), put(15, 0)
    put(16, iplen >> 8), put(17, iplen & 0xFF), put(22, 64), put(23, proto)
    fd = np.zeros(n, dtype=lvlip.FRAME_DESC_DTYPE)
    fd["offset"] = hdr["offset"] - 14
    fd["len"] = 34 + pay["len"]
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    s = torch.cuda.current_stream(dev)
    variants = [("product", lambda: lvlip.rx_verify_dev(base, fdt, 0, stream=s))]
    for p in (0, 1, 2, 4, 8):
        variants.append((f"pf{p * 160}", (lambda p: lambda: lvlip.frames_variant_dev(3, p << 3, base, fdt, stream=s))(p)))
    ref = None
    for name, fn in variants:
        v = fn()
        torch.cuda.synchronize()
        v = v.cpu().numpy()
        if ref is None:
            ref = v
        assert np.array_equal(v, ref), name
    for _ in range(300):
        variants[0][1]()
    torch.cuda.synchronize()
    res = {name: [] for name, _ in variants}
    for _ in range(int(os.environ.get("AB_ROUNDS", "9"))):
        for name, fn in variants:
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    rows = []
    for name, _ in variants:
        med = float(np.median(res[name]))
        rows.append({"variant": name, "us": round(med, 2), "Mframes_per_s": round(n / med, 1),
                     "rounds_us": [round(x, 2) for x in res[name]]})
        print(f"rx_header {name:8s} {med:8.2f} us  {n / med:8.1f} Mframes/s  {[round(x, 1) for x in res[name]]}",
              flush=True)
    if len(sys.argv) > 1:
        json.dump({"frames": n, "rows": rows}, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
