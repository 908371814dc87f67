#!/usr/bin/env python3
"""Lab: ramp and tail of the k_window launch on the tcp1500 batch.

  python scripts/lab_tail.py out.json [waves_per_cu [waves_per_workgroup]]

After a clock settle with AUTO launches, runs k_window (R 2, G 4, the MTU
shape) with per-wave real-time stamps (liblvlip_lab.so
lvlip_lab_window_stamps; 100 MHz counter) for 30 back-to-back launches, each
with its own stamp buffer, and reports per launch: the spread of the waves'
start times (ramp), the spread of their end times (tail), and the wave-time
lost to the tail, i.e. the mean over waves of (last end - this wave's end) over
the launch's span.  Results are checked against AUTO's.
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


def main():
    out_path = sys.argv[1]
    wpc = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    wl = os.environ.get("TAIL_WORKLOAD", "tcp1500")
    dev = torch.device("cuda", 0)
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    lab.lvlip_lab_window_stamps.restype = ctypes.c_int
    lab.lvlip_lab_window_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p]
    wpb = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    hint = b.algo_bytes // b.n
    lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                    lvlip.KERNEL_AUTO, 0, 0, hint)
    torch.cuda.synchronize()
    want = out.cpu().numpy().copy()
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(8):
            lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                            lvlip.KERNEL_AUTO, 0, 0, hint)
        torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record(s)
    for _ in range(30):
        lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                        lvlip.KERNEL_AUTO, 0, 0, hint)
    eb.record(s)
    torch.cuda.synchronize()
    auto_ms = ea.elapsed_time(eb) / 30
    launches = 30
    nbytes = 1 << 20  # per launch: 16 B per wave, room for 64K waves
    stamps = torch.zeros((launches, nbytes // 8), dtype=torch.int64, device=dev)
    nw = 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    dyn = False  # k_window_dyn (TAIL_DYN=1) was pruned in round 4 (last in commit 4e633d9)
    for k in range(launches):
        nw = lab.lvlip_lab_window_stamps(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),
                                         stamps[k].data_ptr(), nbytes, wpc, wpb, s.cuda_stream)
        assert nw > 0, nw
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / launches
    assert np.array_equal(out.cpu().numpy(), want), "stamped k_window differs from AUTO"
    st = stamps[:, : 2 * nw].cpu().numpy().reshape(launches, nw, 2).astype(np.int64)
    res = []
    for k in range(launches):
        t_start, t_end = st[k, :, 0], st[k, :, 1]
        z = t_start.min()
        span = t_end.max() - z
        s_rel = (t_start - z) * 10.0 / 1000.0  # us
        e_rel = (t_end - z) * 10.0 / 1000.0
        res.append({
            "span_us": round(span * 10.0 / 1000.0, 2),
            "start_p50_us": round(float(np.percentile(s_rel, 50)), 2),
            "start_p99_us": round(float(np.percentile(s_rel, 99)), 2),
            "start_max_us": round(float(s_rel.max()), 2),
            "end_min_us": round(float(e_rel.min()), 2),
            "end_p10_us": round(float(np.percentile(e_rel, 10)), 2),
            "end_p50_us": round(float(np.percentile(e_rel, 50)), 2),
            "end_p90_us": round(float(np.percentile(e_rel, 90)), 2),
            "tail_loss_frac": round(float((e_rel.max() - e_rel).mean() / e_rel.max()), 4),
            "ramp_loss_frac": round(float(s_rel.mean() / e_rel.max()), 4),
        })
    summ = {k2: round(float(np.median([r[k2] for r in res[2:]])), 4) for k2 in res[0]}
    # per XCD and per wave slot of the block: median end time (launches 3-30).
    # Ranks are XCD-major: rank = (xcd * grid/8 + block/8) * 4 + wave (block
    # b runs on XCD b % 8, as observed)
    rel = (st[2:, :, 1] - st[2:, :, 0].min(axis=1, keepdims=True)) * 10.0 / 1000.0
    xcd = np.arange(nw) // max(1, nw // 8)
    slot = np.arange(nw) % 4
    by_xcd = {int(x): round(float(np.median(rel[:, xcd == x])), 2) for x in range(8)}
    by_slot = {int(w): round(float(np.median(rel[:, slot == w])), 2) for w in range(4)}
    # within launches: are the same waves late every time? correlation of
    # per-wave end times between consecutive launches
    cors = [float(np.corrcoef(rel[k], rel[k + 1])[0, 1]) for k in range(rel.shape[0] - 1)]
    summ.update({"end_median_by_xcd_us": by_xcd, "end_median_by_wave_slot_us": by_slot,
                 "end_corr_consecutive_launches": round(float(np.median(cors)), 3)})
    raw = st[2:5].tolist()
    summ["GBps_from_span"] = round(b.algo_bytes / (summ["span_us"] * 1e3), 1)
    summ["GBps_auto_events"] = round(b.algo_bytes / auto_ms / 1e6, 1)
    rec = {"workload": wl, "waves_per_cu": wpc, "waves_per_workgroup": wpb, "dyn": dyn, "waves": nw, "ms_per_launch_events": round(ms, 5),
           "GBps": round(b.algo_bytes / ms / 1e6, 1), "median_over_launches_3_30": summ, "launches": res,
           "raw_stamps_launches_3_5": raw}
    print(json.dumps({k2: rec[k2] for k2 in ("workload", "waves", "ms_per_launch_events", "GBps")}), summ,
          flush=True)
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=0)


if __name__ == "__main__":
    main()
