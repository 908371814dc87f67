#!/usr/bin/env python3
"""A/B of the device frame calls' sweep shape (GPU box).

  python scripts/lab_frames_ab.py out.json [rounds]

The mixed config's 2M frames made valid IPv4/TCP/ICMP frames in HBM (as
bench.py --frames builds them).  TX fill and RX verify with L4 run as the
product calls (k_flat2 U 4, quarter order) and as the lab's frame variants
(liblvlip_lab.so lvlip_lab_frames_dev: U 4 / U 8, quarters / blocks), in
interleaved rounds in one process, HIP events, 10 launches each.  Every
variant's verdicts (RX) and status plus frame bytes (TX, which is idempotent:
the fill subtracts each field's current value) must equal the product's.
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


def timed(fn, stream, reps=10, warm=2):
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
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
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
    l4 = int(pay["len"].sum())
    nbytes = 20 * n + l4

    calls = {
        "tx_product": lambda: lvlip.tx_checksum_dev(base, fdt, stream=s),
        "rx_l4_product": lambda: lvlip.rx_verify_dev(base, fdt, lvlip.RX_VERIFY_L4, stream=s),
    }
    for v, name in ((0, "u4_quarters"), (2, "u8_quarters"), (4, "u4_blocks"), (6, "u8_blocks"),
                    (12, "u4_blocks_pf"), (14, "u8_blocks_pf")):
        calls[f"tx_{name}"] = (lambda vv: lambda: lvlip.frames_variant_dev(0, vv, base, fdt, stream=s))(v)
        calls[f"rx_l4_{name}"] = (lambda vv: lambda: lvlip.frames_variant_dev(2, vv, base, fdt, stream=s))(v)

    # equality: TX first (fills the fields), then everything against the product
    ref_tx = calls["tx_product"]().cpu().numpy().copy()
    torch.cuda.synchronize()
    ref_bytes = base.cpu().numpy().copy()
    ref_rx = calls["rx_l4_product"]().cpu().numpy().copy()
    ok_frac = float((ref_rx == lvlip.RX_OK).mean())  # random L4 headers: many fail L4 (timing is the same)
    print(f"RX+L4 verdicts OK: {ok_frac:.3f}; TX filled: {float((ref_tx == 1).mean()):.3f}", flush=True)
    for k, fn in calls.items():
        got = fn().cpu().numpy()
        torch.cuda.synchronize()
        want = ref_tx if k.startswith("tx") else ref_rx
        assert np.array_equal(got, want), k
        if k.startswith("tx"):
            assert np.array_equal(base.cpu().numpy(), ref_bytes), k
    res = {}
    for _ in range(rounds):
        for k, fn in calls.items():
            ms = timed(fn, s)
            res.setdefault(k, []).append(round(ms * 1e3, 2))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in sorted(med.items()):
        print(f"{k:18s} {v:8.2f} us  {nbytes / v / 1e3:7.1f} GB/s  rounds {res[k]}", flush=True)
    with open(out_path, "w") as f:
        json.dump({"frames": n, "checksummed_bytes": nbytes, "rx_ok_frac": ok_frac, "median_us": med, "rounds_us": res}, f, indent=1)


if __name__ == "__main__":
    main()
