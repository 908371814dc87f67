"""Round 6 A/B: what bounds LVLIP_ECHO_FULL's flat sweep.  On the mixed
config's 2M frames in HBM (every ICMP frame an echo request, as bench.py's
echo diag makes them), interleaved rounds of:
  full      the product's ECHO_FULL sweep (lab mode 4 variant 0, the same
            kernel as lvlip_icmp_echo_reply_dev_ex)
  nostore   the same sweep with no reply store (variant 7: timing only)
  rxl4      RX verify with L4 over the same frames (the same parse, twice
            the summed bytes)
HIP events around each launch, the requests restored before each.  Prints
one JSON object (median ms per variant).

    python scripts/echo_bound_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import lvlip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    base, fd, pay = bench.mixed_frames_hbm(lvlip, torch, dev)
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    stream = torch.cuda.current_stream(dev)
    icmp = pay["start_sum"] == 0
    t_off = torch.from_numpy((fd["offset"][icmp] + 34).astype(np.int64)).to(dev)
    variants = {
        "full": lambda: lvlip.frames_variant_dev(4, 0, base, fdt, stream=stream),
        "nostore": lambda: lvlip.frames_variant_dev(4, 7, base, fdt, stream=stream),
        "rxl4": lambda: lvlip.rx_verify_dev(base, fdt, lvlip.RX_VERIFY_L4, stream=stream),
    }
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = {k: [] for k in variants}
    for _ in range(7):
        for k, fn in variants.items():
            base[t_off] = 8
            base[t_off + 1] = 0
            fn()  # warm (and the argument tensors' first use) outside the pair
            base[t_off] = 8
            base[t_off + 1] = 0
            torch.cuda.synchronize()
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ms[k].append(e0.elapsed_time(e1))
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 4) for k, v in ms.items()} |
                     {"icmp_bytes": int(pay["len"][icmp].sum()), "frames": int(fd.size)}))


if __name__ == "__main__":
    main()
