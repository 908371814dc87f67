#!/usr/bin/env python3
"""Lab (round 4, VERDICT r03 Next #1): what the device TX fill's field stores cost.

  python scripts/lab_tx_store.py out.json [rounds]
  python scripts/lab_tx_store.py --only NAME [reps]     (for rocprofv3 passes)

The mixed config's 2M frames made valid IPv4/TCP/ICMP frames in HBM (as
bench.py --frames builds them).  Timed in interleaved rounds in one process,
HIP events, 10 launches each:
  tx_product     lvlip_tx_checksum_dev (k_flat2 U 8, 2-B field stores; `nt sc0
                 sc1` since round 4)
  tx_nt          the same with nontemporal 2-B stores (round 3's product; variant 6)
  tx_plain       the same with plain (temporal) 2-B field stores (variant 7)
  tx_sec32       the same kernel writing the aligned 32-B sector around each
                 field whole (lab frames variant 16; 2-B stores where the sector
                 leaves the frame)
  tx_sec64       the same with 64-B blocks (variant 32)
  tx_sc0 .. tx_ntsc0sc1  2-B field stores with the cache-policy bits sc0, sc1,
                 sc0 sc1, nt sc1, nt sc0 sc1 (variants 64-320)
  (tx_cb64 / tx_cb64_reload_only / tx_cb64_noreload, whole 64-B blocks by
                 four lanes in one store and its halves, variants 512 / 576 /
                 640: measured in profiles/r04_tx_store_cb64.json, removed,
                 last in commit fe59a5a)
  rx_l4          lvlip_rx_verify_dev with L4: the same sweep without stores
  st_*           lvlip_lab_probe_fields on a scratch copy of the buffer: the two
                 fields of every frame (+24, +50) stored alone, no sweep:
                 st_2b (2-B nt), st_2b_rmw (2-B load + nt store), st_sec32
                 (32-B sector load + whole nt store), st_sec32_noload,
                 st_blk64 (64-B block load + store), st_2b_plain, and 2-B
                 stores with each cache policy (st_2b_sc0 .. st_2b_ntsc0sc1)
Every TX variant's status and frame bytes must equal the product's (the fill
is idempotent: it subtracts each field's current value).
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402

PROBES = {"st_2b": 0, "st_2b_rmw": 1, "st_sec32": 2, "st_sec32_noload": 3, "st_blk64": 4, "st_2b_plain": 5,
          "st_2b_sc0": 6, "st_2b_sc1": 7, "st_2b_sc0sc1": 8, "st_2b_ntsc1": 9, "st_2b_ntsc0sc1": 10}
# TX fill variants of lvlip_lab_frames_dev mode 0 (the product's shape, U 8 blocks)
TX_VARIANTS = {"tx_nt": 6, "tx_plain": 7, "tx_sec32": 16, "tx_sec64": 32, "tx_sc0": 64, "tx_sc1": 128, "tx_sc0sc1": 192,
               "tx_ntsc1": 256, "tx_ntsc0sc1": 320}
# timing probes that write wrong frame bytes: run on a scratch copy, not checked
# (round 4's tx_cb64_noreload, variant 640, until commit fe59a5a)
TX_SCRATCH = {}


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


def setup(dev):
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
    nbytes = 20 * n + int(pay["len"].sum())
    return base, fdt, n, nbytes


def main():
    dev = torch.device("cuda", 0)
    base, fdt, n, nbytes = setup(dev)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    lab.lvlip_lab_probe_fields.restype = ctypes.c_int
    lab.lvlip_lab_probe_fields.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]
    scratch = base.clone()
    calls = {
        "tx_product": lambda: lvlip.tx_checksum_dev(base, fdt, stream=s),
        "rx_l4": lambda: lvlip.rx_verify_dev(base, fdt, lvlip.RX_VERIFY_L4, stream=s),
    }
    for k, v in TX_VARIANTS.items():
        calls[k] = (lambda vv: lambda: lvlip.frames_variant_dev(0, vv, base, fdt, stream=s))(v)
    # each launch on a fresh copy of the frames (the variant destroys them),
    # beside the product on a fresh copy: compare the two, not the others
    scratch_tx = base.clone() if TX_SCRATCH else None
    if TX_SCRATCH:
        calls["tx_product_copied"] = lambda: (scratch_tx.copy_(base),
                                              lvlip.tx_checksum_dev(scratch_tx, fdt, stream=s))
    for k, v in TX_SCRATCH.items():
        calls[k] = (lambda vv: lambda: (scratch_tx.copy_(base),
                                        lvlip.frames_variant_dev(0, vv, scratch_tx, fdt, stream=s)))(v)
    for k, m in PROBES.items():
        calls[k] = (lambda mm: lambda: lab.lvlip_lab_probe_fields(scratch.data_ptr(), fdt.data_ptr(), n, mm,
                                                                  s.cuda_stream))(m)
    if sys.argv[1] == "--only":
        reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
        fn = calls[sys.argv[2]]
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        print(f"ran {sys.argv[2]} x{reps}", flush=True)
        return
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    ref_st = calls["tx_product"]().cpu().numpy().copy()
    torch.cuda.synchronize()
    ref_bytes = base.cpu().numpy().copy()
    filled = float((ref_st == 1).mean())
    print(f"TX filled: {filled:.3f}", flush=True)
    for k in list(TX_VARIANTS) + ["tx_product"]:
        got = calls[k]().cpu().numpy()
        torch.cuda.synchronize()
        assert np.array_equal(got, ref_st), k
        assert np.array_equal(base.cpu().numpy(), ref_bytes), k
    # how many fields the 32-B / 64-B variants write as whole blocks
    fd = fdt.cpu().numpy().view(lvlip.FRAME_DESC_DTYPE)
    fs = fd["offset"].astype(np.int64) + base.data_ptr()
    fe = fs + fd["len"]
    blk = {}
    for B in (32, 64):
        ins = lambda a: ((a & ~(B - 1)) >= fs) & ((a & ~(B - 1)) + B <= fe)  # noqa: E731
        l4f = fs + 34 + np.where(ref_bytes[fd["offset"] + 23] == 6, 16, 2)
        blk[B] = {"hdr_inside": float(ins(fs + 24).mean()), "l4_inside": float(ins(l4f).mean()),
                  "shared": float((((fs + 24) & ~(B - 1)) == (l4f & ~(B - 1))).mean())}
    print("block coverage", blk, flush=True)
    res = {}
    for _ in range(rounds):
        for k, fn in calls.items():
            ms = timed(fn, s)
            res.setdefault(k, []).append(round(ms * 1e3, 2))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in med.items():
        extra = f"{nbytes / v / 1e3:7.1f} GB/s" if not k.startswith("st_") else ""
        print(f"{k:16s} {v:8.2f} us  {extra} rounds {res[k]}", flush=True)
    with open(out_path, "w") as f:
        json.dump({"frames": n, "checksummed_bytes": nbytes, "tx_filled_frac": filled, "block_coverage": blk,
                   "median_us": med, "rounds_us": res}, f, indent=1)


if __name__ == "__main__":
    main()
