#!/usr/bin/env python3
"""Read-bandwidth lab: times the lab probes (pure streaming reads) and the
checksum kernels on one resident buffer, interleaved rounds in one process.
Prints one line per variant (GB/s, median of rounds) and writes JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
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
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    wl = os.environ.get("LAB_WORKLOAD", "tcp1500")
    dev = torch.device("cuda", 0)
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    nb = base.numel() & ~1023
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    variants = []
    if os.environ.get("LAB_SET") == "csum":
        variants = [("probe", 1, 8, 1, 2), ("probe", 2, 4, 1, 2)]
    for mode in (() if os.environ.get("LAB_SET") == "csum" else (1, 2)):
        for u in (4, 8):
            for nt in (0, 1):
                for bpc in (2, 4, 8):
                    variants.append(("probe", mode, u, nt, bpc))
    for u in (() if os.environ.get("LAB_SET") == "csum" else (4, 8)):
        for bpc in (2, 4):
            variants.append(("probe", 3, u, 0, bpc))
    ck = [("csum", k, u, w) for k, u, w in [
        ("wave", 2, 4), ("wave", 2, 8), ("wave", 2, 12), ("wave", 2, 16), ("wave", 2, 24),
        ("wave", 3, 8), ("wave", 3, 12), ("wave", 3, 16), ("wave", 4, 8), ("wave", 4, 16),
        ("flat", 0, 0)]]
    res = {}
    for rnd in range(3):
        for v in variants:
            _, mode, u, nt, bpc = v
            f = lambda: lab.lvlip_lab_probe(base.data_ptr(), nb, sink.data_ptr(), mode, u, nt,  # noqa
                                            cus * bpc, s.cuda_stream)
            assert f() == 0
            ms = timed(f, s)
            res.setdefault(f"probe m{mode} u{u} nt{nt} bpc{bpc}", []).append(nb / ms / 1e6)
        for v in ck:
            _, k, u, w = v
            f = lambda: lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),  # noqa
                                        s.cuda_stream, lvlip.KERNEL_NAMES[k], u, w)
            ms = timed(f, s)
            res.setdefault(f"csum {k} u{u} w{w}", []).append(b.algo_bytes / ms / 1e6)
    summary = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in sorted(summary.items(), key=lambda kv: -kv[1]):
        print(f"{k:32s} {v:8.1f} GB/s")
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"workload": wl, "bytes": nb, "median_GBps": summary, "rounds": res}, f, indent=1)


if __name__ == "__main__":
    main()
