#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run of `bench.py --frames` (KRE="k_flat2|k_rx_hdr")
into profiles/<tag>_frames_pmc.json: per device frame call (TX fill, RX header on
k_rx_hdr and on k_flat2, RX header + L4) the kernel's median duration, HBM bytes
from the PMC passes, and the algorithmic bytes.

The trace names every flat frame launch `k_flat2` (truncated), so calls are told
apart by order: bench.py's frames_dev times tx_fill (nontemporal field stores),
tx_fill_plain, rx_header (k_rx_hdr), rx_header_flat (k_flat2), rx_header_l4, each 3 warm-ups + 10 reps, then one
rx_header for the all-OK check.  That order is checked against the kernel names
and grid sizes (RX header-only uses one slot per frame, the others two).

hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, as scripts/prof_summary.py.
Algorithmic bytes: the checksummed bytes (20 B per header + the L4 bytes) plus
the bytes the call writes (TX: two 2-B fields and a status byte per frame; RX: a
verdict byte per frame).

usage: frames_summary.py <profile dir> <tag>
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import workloads  # noqa: E402

MODES = (["tx_fill"] * 13 + ["tx_fill_plain"] * 13 + ["rx_header"] * 13 + ["rx_header_flat"] * 13
         + ["rx_header_l4"] * 13 + ["rx_header"])
KERNEL = {"tx_fill": "k_flat2", "tx_fill_plain": "k_flat2", "rx_header": "k_rx_hdr",
          "rx_header_flat": "k_flat2", "rx_header_l4": "k_flat2"}


def dispatches(path, value_col=None):
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(("k_flat2", "lvlip::k_flat2",
                                                                                   "k_rx_hdr", "lvlip::k_rx_hdr"))]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    b = workloads.make("mixed")
    n = b.descs.size // 2
    l4 = int(b.descs[1::2]["len"].sum())
    algo = {"tx_fill": 20 * n + l4 + 5 * n, "tx_fill_plain": 20 * n + l4 + 5 * n,
            "rx_header": 20 * n + n, "rx_header_flat": 20 * n + n,
            "rx_header_l4": 20 * n + l4 + n}
    # the device calls come first; later k_flat2 launches (the host-API timings
    # of bench.py --frames) are not part of this summary
    trace = dispatches(os.path.join(prof, "trace", "trace_kernel_trace.csv"))[: len(MODES)]
    assert len(trace) == len(MODES), (len(trace), len(MODES))
    per = {m: {"dur_ns": [], "grid": set()} for m in algo}
    for r, m in zip(trace, MODES):
        assert KERNEL[m] in r["Kernel_Name"], (m, r["Kernel_Name"])
        per[m]["dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        per[m]["grid"].add(int(r["Grid_Size_X"]))
    assert per["rx_header"]["grid"] == {256 * ((n + 255) // 256)}, per["rx_header"]["grid"]
    assert per["rx_header_flat"]["grid"] == {256 * ((n + 255) // 256)}, per["rx_header_flat"]["grid"]
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        rows = dispatches(os.path.join(prof, sub, f"{sub}_counter_collection.csv"))[: len(MODES)]
        assert len(rows) == len(MODES), (sub, len(rows))
        for r, m in zip(rows, MODES):
            per[m].setdefault(counter, []).append(float(r["Counter_Value"]))
    out = {"tag": tag, "workload": "bench.py --frames: the mixed config's 2M frames as IPv4/TCP/ICMP",
           "frames": n, "calls": {}}
    for m, v in per.items():
        dur = statistics.median(v["dur_ns"])
        hbm = (2 * statistics.median(v["FETCH_SIZE"]) + statistics.median(v["WRITE_SIZE"])) * 1024
        out["calls"][m] = {
            "launches": len(v["dur_ns"]), "median_duration_ns": dur,
            "algorithmic_bytes": algo[m], "algorithmic_GBps": round(algo[m] / dur, 1),
            "hbm_bytes_per_launch": round(hbm), "traffic_over_algo": round(hbm / algo[m], 3),
            "fetch_kb": statistics.median(v["FETCH_SIZE"]), "write_kb": statistics.median(v["WRITE_SIZE"]),
        }
    dst = os.path.join(ROOT, "profiles", f"{tag}_frames_pmc.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
