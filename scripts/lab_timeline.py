#!/usr/bin/env python3
"""Timeline lab (diagnostic): where a streaming read's time goes — launch ramp,
steady state, tail — for static wave-contiguous ranges vs dynamically claimed
granules (per-XCD queues).  Each launch is timed alone with HIP events (queue
heads zeroed outside the event pair); one extra launch per variant records
per-wave s_memrealtime stamps (100 MHz).  Prints one line per variant and writes
JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    sizes = [int(float(x) * 1e6) // 1024 * 1024 for x in
             os.environ.get("TL_MB", "1572.864,9437.184").split(",")]
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    ctr = torch.zeros(8 * 32, dtype=torch.int32, device=dev)
    variants = [(0, 8, 0, 2), (0, 4, 0, 4)]
    if os.environ.get("TL_BPC"):  # oversubscribed static grids: blocks per CU
        variants = [(0, 8, 0, int(b)) for b in os.environ["TL_BPC"].split(",")]
    if os.environ.get("TL_DYN"):
        for gp in (16, 64):
            variants.append((1, 8, gp, 2))
    res = {}
    for nb in sizes:
        buf = torch.empty(nb, dtype=torch.uint8, device=dev)
        buf.fill_(0x5a)
        for rnd in range(3):
            for dyn, u, gp, bpc in variants:
                grid = cus * bpc
                ms = []
                for rep in range(8):
                    ctr.zero_()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    rc = lab.lvlip_lab_probe_tl(buf.data_ptr(), nb, sink.data_ptr(), dyn, u, gp,
                                                ctr.data_ptr(), None, grid, s.cuda_stream)
                    assert rc == 0, rc
                    e1.record(s)
                    ms.append((e0, e1))
                torch.cuda.synchronize()
                t = sorted(a.elapsed_time(b) for a, b in ms[2:])
                key = f"{nb / 1e9:.2f}GB dyn{dyn} u{u} gp{gp} bpc{bpc}"
                res.setdefault(key, {"GBps": []})["GBps"].append(nb / t[len(t) // 2] / 1e6)
        for dyn, u, gp, bpc in variants:
            grid = cus * bpc
            nwave = grid * 4
            tl = torch.zeros(nwave * 4, dtype=torch.int64, device=dev)
            ctr.zero_()
            rc = lab.lvlip_lab_probe_tl(buf.data_ptr(), nb, sink.data_ptr(), dyn, u, gp,
                                        ctr.data_ptr(), tl.data_ptr(), grid, s.cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            a = tl.cpu().numpy().reshape(nwave, 4)
            t0 = a[:, 0].astype(np.int64)
            t1 = a[:, 1].astype(np.int64)
            base = t0.min()
            st = (t0 - base) / 100.0  # us
            en = (t1 - base) / 100.0
            xcc = a[:, 2] & 7
            per_xcc_end = {int(x): float(np.max(en[xcc == x])) for x in range(8) if np.any(xcc == x)}
            per_xcc_pct = {int(x): [round(float(np.percentile(en[xcc == x], q)), 1) for q in (0, 10, 50, 90, 100)]
                           for x in range(8) if np.any(xcc == x)}
            key = f"{nb / 1e9:.2f}GB dyn{dyn} u{u} gp{gp} bpc{bpc}"
            r = res[key]
            r["GBps_med"] = sorted(r["GBps"])[1]
            r["start_us"] = [float(np.percentile(st, p)) for p in (50, 99, 100)]
            r["end_us"] = [float(np.percentile(en, p)) for p in (0, 10, 50, 90, 99, 100)]
            r["span_us"] = float(en.max())
            r["ideal_steady_us"] = float(np.median(en))
            r["per_xcc_end_us"] = per_xcc_end
            r["claims_max"] = int(a[:, 3].max())
            r["per_xcc_end_pct_us"] = per_xcc_pct
            r["n_waves_per_xcc"] = {int(x): int(np.sum(xcc == x)) for x in range(8)}
            r["xcc_busy_end_us"] = {int(x): float(np.max(en[xcc == x])) for x in range(8) if np.any(xcc == x)}
            print(f"{key:34s} {r['GBps_med']:7.1f} GB/s  start p50/p99/max "
                  f"{r['start_us'][0]:.2f}/{r['start_us'][1]:.2f}/{r['start_us'][2]:.2f} us  "
                  f"end p0/p10/p50/p90/p99/max " + "/".join(f"{x:.1f}" for x in r["end_us"]) +
                  f" us  xcc_end " + ",".join(f"{v:.0f}" for v in per_xcc_end.values()), flush=True)
            for x, v in per_xcc_pct.items():
                print(f"    xcc{x} waves {r['n_waves_per_xcc'][x]} end p0/p10/p50/p90/max {v}", flush=True)
        del buf
        torch.cuda.empty_cache()
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
