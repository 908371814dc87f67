#!/usr/bin/env python3
"""A/B of the stream kernel's schedule (diagnostic): by default WAVE_DYN
(static segments + dynamic tail) against WAVE_STATIC; AB_KERNELS picks others
(e.g. wave,wave_static: slot weights from the last launch vs none), interleaved rounds
on one resident batch, each launch timed alone with HIP events on its stream.
The tail knobs are environment variables read once per process
(LVLIP_TAIL_PCT, LVLIP_TAIL_CHUNK), so sweep them with one process each.
Prints one JSON line: median GB/s (algorithmic bytes) per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def main():
    wl = os.environ.get("AB_WORKLOAD", "tcp1500")
    reps = int(os.environ.get("AB_REPS", "20"))
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b)
    hint = b.algo_bytes // b.n
    s = torch.cuda.current_stream()
    names = os.environ.get("AB_KERNELS", "wave_dyn,wave_static").split(",")
    variants = {k: lvlip.KERNEL_NAMES[k] for k in names}
    res = {k: [] for k in variants}
    for _ in range(3):
        for name, k in variants.items():
            lvlip.batch_torch(base, descs, out, kernel=k, len_hint=hint)
    torch.cuda.synchronize()
    for rnd in range(5):
        for name, k in variants.items():
            ev = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                lvlip.batch_torch(base, descs, out, kernel=k, len_hint=hint)
                e1.record(s)
                ev.append((e0, e1))
            torch.cuda.synchronize()
            ms = sorted(a.elapsed_time(c) for a, c in ev)
            res[name].append(b.algo_bytes / ms[len(ms) // 2] / 1e6)
    med = {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}
    print(json.dumps({"workload": wl, "tail_pct": os.environ.get("LVLIP_TAIL_PCT", "15"),
                      "tail_chunk": os.environ.get("LVLIP_TAIL_CHUNK", "16384"),
                      "median_GBps": med, "rounds": res}), flush=True)


if __name__ == "__main__":
    main()
