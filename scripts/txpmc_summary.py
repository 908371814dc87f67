#!/usr/bin/env python3
"""Summarise `scripts/gpu_steps.sh txpmc` (rocprofv3 FETCH_SIZE / WRITE_SIZE
passes of scripts/lab_tx_store.py --only <variant>, one process per variant and
counter, plus one kernel-trace pass of the product's TX fill) into
profiles/<tag>_frames_pmc.json: per call the median kernel duration (from the
counter runs' own dispatch timestamps where present, else the trace), HBM bytes
per launch and the algorithmic bytes.

hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE reports half the
bytes of wide streaming reads on gfx950 (the profile.sh / prof_summary.py rule);
the parse's sparse 64-B window loads are counted twice by that rule (DESIGN.md
§10 item 6), so traffic_over_algo is an upper bound for the frame calls.
Algorithmic bytes: 20 B per IPv4 header + the L4 bytes (the checksummed
bytes), plus what the call writes (TX: two 2-B fields and a status byte per
frame; RX: a verdict byte per frame).

usage: txpmc_summary.py <gpurun_out/txpmc> <tag>
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import workloads  # noqa: E402

KERNELS = ("k_flat2", "lvlip::k_flat2", "k_probe", "(anonymous namespace)::k_probe")


def rows(path):
    out = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].split("<")[0].split("(")[0].strip()
           .endswith(("k_flat2", "k_probe_fields"))]
    out.sort(key=lambda r: int(r["Dispatch_Id"]))
    return out


def main():
    d, tag = sys.argv[1], sys.argv[2]
    b = workloads.make("mixed")
    n = b.descs.size // 2
    summed = 20 * n + int(b.descs[1::2]["len"].sum())
    algo = {"tx": summed + 5 * n, "rx": summed + n}
    calls = {}
    for sub in sorted(os.listdir(d)):
        if sub == "trace":
            continue
        v, counter = sub.rsplit("_", 2)[0], "_".join(sub.rsplit("_", 2)[1:])
        files = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        rs = rows(files[0])
        vals = [float(r["Counter_Value"]) for r in rs]
        calls.setdefault(v, {})[counter] = statistics.median(vals) if vals else None
    out = {"tag": tag, "workload": "scripts/lab_tx_store.py: the mixed config's 2M frames as IPv4/TCP/ICMP "
                                   "frames in HBM, 20 launches per variant", "frames": n, "calls": {}}
    tr = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
    dur = None
    if tr:
        ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows(tr[0])]
        dur = statistics.median(ds) if ds else None
        out["tx_product_trace_median_ns"] = dur
        out["tx_product_trace_launches"] = len(ds)
    for v, c in sorted(calls.items()):
        if c.get("FETCH_SIZE") is None or c.get("WRITE_SIZE") is None:
            continue
        a = algo["rx" if v.startswith("rx") else "tx"]
        hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        out["calls"][v] = {"fetch_kb": c["FETCH_SIZE"], "write_kb": c["WRITE_SIZE"],
                           "hbm_bytes_per_launch": round(hbm), "algorithmic_bytes": a,
                           "traffic_over_algo": round(hbm / a, 3)}
    dst = os.path.join(ROOT, "profiles", f"{tag}_frames_pmc.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
