#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into profiles/<tag>_pmc_<workload>.json.

hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read
(MI355X_MICROARCH.md, HBM); WRITE_SIZE is taken as reported (2-B result stores,
uncalibrated, ~0.1 % of the traffic).  Also copies the PMC run's kernel-trace stats csv (as <tag>_<workload>_pmc_run_kernel_stats.csv,
not over the full command's trace summary)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

prof, tag, workload, kernel_label, algo = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5])
kre = sys.argv[6] if len(sys.argv) > 6 else "k_stream"


def counters(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kre in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


c = {}
for sub in ("sq", "sq2", "fetch", "write"):
    p = os.path.join(prof, sub, f"{sub}_counter_collection.csv")
    if os.path.exists(p):
        c.update(counters(p))
stats = {}
for r in csv.DictReader(open(os.path.join(prof, "trace", "trace_kernel_stats.csv"))):
    stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                        "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
k = next(v for n, v in stats.items() if kre in n)
hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
rec = {"tag": tag, "kernels": [{
    "workload": workload, "kernel": kernel_label, "kernel_regex": kre,
    "avg_duration_ns": k["avg_ns"], "calls": k["calls"],
    "algo_bytes_per_launch": algo,
    "achieved_GBps_from_trace": algo / k["avg_ns"],
    "hbm_bytes_per_launch": hbm, "traffic_over_algo": hbm / algo if algo else None,
    "counters": c,
    "note": "FETCH_SIZE doubled (gfx950 reports half of 16-B/lane streaming reads); "
            "profiled runs clock lower than un-profiled ones (MI355X_MICROARCH.md DVFS item 2)"}]}
os.makedirs("profiles", exist_ok=True)
out = f"profiles/{tag}_pmc_{workload}.json"
json.dump(rec, open(out, "w"), indent=1)
# the short PMC run's own trace summary; profiles/<tag>_<workload>_kernel_stats.csv
# is the full bench command's trace (scripts/evidence.sh step 2), kept apart
shutil.copy(os.path.join(prof, "trace", "trace_kernel_stats.csv"),
            f"profiles/{tag}_{workload}_pmc_run_kernel_stats.csv")
print(out, json.dumps(rec["kernels"][0], indent=None)[:400])
