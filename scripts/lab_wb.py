#!/usr/bin/env python3
"""Lab (round 4): what scattered field writes cost once their write-back is paid.

  python scripts/lab_wb.py out.json [rounds]

The stores-alone timings of scripts/lab_tx_store.py leave the write-back of
plain stores to whatever runs next (the ~256 MB of dirty blocks fit the
memory-side cache, and repeated launches re-dirty the same lines).  Here every
store form runs in a pair with the RX + L4 sweep over the mixed config's 2M
frames (the TX fill's own read stream, no stores), so the sweep's reads push
the dirty blocks out to HBM inside the timed region:

  pair(form) = 10 x [rx_l4 ; lvlip_lab_probe_fields(form) on a scratch copy]
  cost(form) = pair(form) / 10 - rx_l4 alone

beside tx_product (the fused fill, 2-B `nt sc0 sc1` stores), whose cost over
rx_l4 is the figure to beat (~110 us).  Forms (lab_probe.hip k_probe_fields /
k_probe_sectors): 2-B stores nt / plain / nt sc0 sc1; the 32-B sector written
by one lane in two 16-B stores; the aligned 32-, 64- or 128-B block written by
adjacent lanes in ONE store instruction (whole-sector requests: no
read-modify-write in the memory controller, HBM3E having no write data mask),
and the 64-B block loaded by those lanes first and stored back.
Interleaved rounds in one process, HIP events.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

import lab_tx_store  # noqa: E402
import lvlip  # noqa: E402

FORMS = {"2b_nt": 0, "2b_plain": 5, "2b_ntsc0sc1": 10, "sec32_1lane_nt": 3, "sec32_nt": 11, "sec32_plain": 12,
         "blk64_nt": 13, "blk64_plain": 14, "sec32_ntsc0sc1": 15, "blk128_plain": 16, "blk64_load_nt": 17,
         "blk64_load_plain": 18}
REPS = 10


def main():
    dev = torch.device("cuda", 0)
    base, fdt, n, nbytes = lab_tx_store.setup(dev)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    lab.lvlip_lab_probe_fields.restype = ctypes.c_int
    lab.lvlip_lab_probe_fields.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]
    # scratch with 256 B of tail room: a 128-B block around the last frame's
    # second field may end up to 79 B past that frame
    scratch = torch.zeros(base.numel() + 256, dtype=torch.uint8, device=dev)
    scratch[:base.numel()].copy_(base)

    def store(m):
        rc = lab.lvlip_lab_probe_fields(scratch.data_ptr(), fdt.data_ptr(), n, m, s.cuda_stream)
        assert rc == 0, (m, rc)

    def rx():
        lvlip.rx_verify_dev(base, fdt, lvlip.RX_VERIFY_L4, stream=s)

    calls = {"rx_l4": rx, "tx_product": lambda: lvlip.tx_checksum_dev(base, fdt, stream=s)}
    for k, m in FORMS.items():
        calls["st_" + k] = (lambda mm: lambda: store(mm))(m)
        calls["pair_" + k] = (lambda mm: lambda: (rx(), store(mm)))(m)
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    res = {}
    for _ in range(rounds):
        for k, fn in calls.items():
            res.setdefault(k, []).append(round(lab_tx_store.timed(fn, s, reps=REPS) * 1e3, 2))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    cost = {k: round(med["pair_" + k] - med["rx_l4"], 2) for k in FORMS}
    cost["tx_product (fused)"] = round(med["tx_product"] - med["rx_l4"], 2)
    for k, v in med.items():
        print(f"{k:22s} {v:8.2f} us  rounds {res[k]}", flush=True)
    print("cost over rx_l4 (us):", json.dumps(cost), flush=True)
    with open(sys.argv[1], "w") as f:
        json.dump({"frames": n, "checksummed_bytes": nbytes, "reps_per_timing": REPS, "median_us": med,
                   "cost_over_rx_l4_us": cost, "rounds_us": res}, f, indent=1)


if __name__ == "__main__":
    main()
