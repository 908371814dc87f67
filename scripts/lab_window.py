#!/usr/bin/env python3
"""Lab: does the order in which the waves walk the buffer move the HBM read ceiling?

Probe modes (level-ip_amd/csrc/lab_probe.hip), all nontemporal 16-B/lane loads:
  m0  thread-level grid stride (U loads a grid-stride apart)
  m1  block-contiguous ranges
  m2  wave-contiguous ranges (k_stream's layout: nw far-apart streams)
  m5  chip-wide window (wave w reads U-KiB chunks w, w+nw, ...)
  c   chunk probe: order 0/1 wave chunks (window when small), order 2 block chunks
Interleaved rounds in one process; prints the median GB/s per variant.

  LAB_WORKLOAD=tcp1500 python scripts/lab_window.py [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def timed(fn, stream, reps=20, warm=3):
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
    lab_set = os.environ.get("LAB_SET", "")
    if lab_set == "chunk":
        # (mode "c", depth U, chunk pieces, wave order, blocks per CU)
        for cp in (4, 8, 12, 16, 24, 32, 48, 64, 128, 512):
            variants.append(("c", 4, cp, 0, 2))
        for cp in (4, 8, 16, 32):
            variants.append(("c", 2, cp, 0, 2))
            variants.append(("c", 2, cp, 0, 4))
        for cp in (8, 16, 32):
            variants.append(("c", 8, cp, 0, 2))
        variants += [(5, 4, 0, 0, 2), (2, 8, 0, 0, 2), (1, 8, 0, 0, 2)]
    elif lab_set == "chunk2":
        for u, cp in ((3, 3), (4, 4), (3, 6), (6, 6), (4, 8), (2, 2)):
            for order in (0, 1):
                variants.append(("c", u, cp, order, 2))
        for u, cp in ((3, 3), (4, 4), (6, 6)):
            variants.append(("c", u, cp, 0, 3))
        variants += [(2, 8, 0, 0, 2)]
    elif lab_set == "ragged":
        # the mixed buffer: window vs contiguous orders at 8 and 32 waves/CU
        variants += [("c", 4, 4, 1, 2), ("c", 4, 4, 1, 8), ("c", 4, 16, 1, 8), ("c", 8, 8, 1, 4),
                     (2, 8, 0, 0, 2), (2, 4, 0, 0, 8), (1, 8, 0, 0, 2), (1, 4, 0, 0, 8)]
    elif lab_set == "blockchunk":
        # k_flat2-like block streams on the mixed buffer: block chunks of cp KiB
        # (the tile's bytes), 4 waves taking U-KiB slices round robin, bpc blocks
        # per CU; against the chip-wide window and contiguous wave ranges
        for cp in (32, 64, 128, 256):
            for bpc in (2, 5, 8):
                variants.append(("c", 8, cp, 2, bpc))
        for cp in (16, 32, 64, 128):
            variants.append(("c", 4, cp, 2, 5))
        variants += [("c", 4, 4, 1, 2), ("c", 8, 8, 1, 2), (2, 8, 0, 0, 2), (2, 8, 0, 0, 5), (1, 8, 0, 0, 5)]
    elif lab_set == "pkwin":
        # group g: two loads per slot; 100 + g: the group's span in whole loads
        for g in (1, 2, 3, 4, 6, 8, 101, 102, 103, 104, 106, 108):
            variants.append(("p", g, 0, 0, 2))
        for g in (2, 3):
            variants.append(("p", g, 0, 0, 3))
        variants += [("c", 4, 4, 1, 2), (4, 3, 0, 0, 2), (2, 8, 0, 0, 2)]
    else:
        for mode in (0, 2, 5):
            for u in (1, 2, 4, 8):
                for bpc in (2, 4, 8):
                    if mode == 2 and u < 4:
                        continue
                    variants.append((mode, u, 0, 0, bpc))
        variants.append((1, 8, 0, 0, 2))
    # settle the clocks before the first variant (scripts/warm_curve.py)
    hint = b.algo_bytes // b.n

    def csum():
        lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                        lvlip.KERNEL_AUTO, 0, 0, hint)
    timed(csum, s, reps=300)
    res = {}
    for rnd in range(3):
        for mode, u, cp, order, bpc in variants:
            if mode == "p":
                f = lambda: lab.lvlip_lab_probe_pkwin(base.data_ptr(), nb & ~15, sink.data_ptr(), u,  # noqa
                                                      cus * bpc, s.cuda_stream)
                key = f"probe pkwin G{u} bpc{bpc}"
            elif mode == "c":
                f = lambda: lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(), u,  # noqa
                                                      cp, order, cus * bpc, s.cuda_stream)
                key = f"probe chunk u{u} cp{cp} o{order} bpc{bpc}"
            else:
                f = lambda: lab.lvlip_lab_probe(base.data_ptr(), nb, sink.data_ptr(), mode, u, 1,  # noqa
                                                cus * bpc, s.cuda_stream)
                key = f"probe m{mode} u{u} bpc{bpc}"
            assert f() == 0, (mode, u, cp, bpc)
            ms = timed(f, s)
            res.setdefault(key, []).append(nb / ms / 1e6)
        ms = timed(csum, s)
        res.setdefault("csum auto", []).append(b.algo_bytes / ms / 1e6)
        print(f"round {rnd} done", flush=True)
    summary = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in sorted(summary.items(), key=lambda kv: -kv[1]):
        print(f"{k:32s} {v:8.1f} GB/s", flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"workload": wl, "bytes": nb, "median_GBps": summary, "rounds": res}, f, indent=1)


if __name__ == "__main__":
    main()
