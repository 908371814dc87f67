#!/usr/bin/env python3
"""Lab: the per-call CPU drop-in (include/lvlip_csum.h Group 1) on one core, by
word-sum path, next to the reference's own checksum() (oracle/_ref, -O0).

Every path runs in a child process of its own, because the library picks the
path once (LVLIP_CPU_SUM, read at the first call).  The harness is bench.py's
cpu_baseline one (pyoracle.batch, one thread, per packet through a ctypes
function pointer), so the numbers compare with dropin_one_core_GBps there.
Each child checks its output against the oracle before timing.

  python scripts/dropin_paths.py [--workloads tcp1500,mixed,tcp64] [--seconds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def child(workload: str, seconds: float, path: str) -> dict:
    import numpy as np

    import lvlip
    import pyoracle
    import workloads

    sb = workloads.make(workload, n=65536)
    host = sb.host_bytes()
    want = pyoracle.batch(host, sb.descs, threads=8, opt=2)
    if path == "reference":
        if pyoracle.reflib() is None:
            return {"workload": workload, "path": path, "skipped": "oracle/_ref not built"}
        run = lambda: pyoracle.batch(host, sb.descs, threads=1, opt=0, use_reference=True)  # noqa: E731
    else:
        run = lambda: pyoracle.batch(host, sb.descs, threads=1, csum_fn=lvlip.lib().checksum)  # noqa: E731
    if not np.array_equal(run(), want):
        raise SystemExit(f"{path} on {workload}: checksums differ from the oracle")
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        run()
        reps += 1
    dt = time.perf_counter() - t0
    return {"workload": workload, "path": path, "GBps": round(sb.algo_bytes * reps / dt / 1e9, 3),
            "ns_per_packet": round(dt / reps / sb.n * 1e9, 1), "packets": sb.n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="tcp1500,mixed,tcp64")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--child", nargs=2, metavar=("WORKLOAD", "PATH"))
    a = ap.parse_args()
    if a.child:
        print(json.dumps(child(a.child[0], a.seconds, a.child[1])), flush=True)
        return
    for w in a.workloads.split(","):
        for path in ("reference", "scalar", "avx2", "avx512"):
            env = dict(os.environ, LVLIP_CPU_SUM=path)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--seconds", str(a.seconds),
                                "--child", w, path], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise SystemExit(r.stderr[-2000:])
            print(r.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
