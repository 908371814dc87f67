#!/usr/bin/env python3
"""Lab (round 4, VERDICT r03 Next #2): the mixed line's process-to-process modes.

  python scripts/lab_modes.py out.json

One process: the mixed batch in HBM, a 250-ms settle, then
  * the bench's measurement (50 + 200 AUTO launches, HIP events) -> the mode;
  * the window read probe over the same buffer (bench diag's window_c4);
  * 20 launches of k_flat2_stamp (the product's U 8 body with per-workgroup
    start/end stamps, XCD and HW_ID; lvlip_lab_flat_stamps), results checked
    against AUTO's;
  * the virtual addresses of the buffers modulo 2 MiB and 1 GiB, the process's
    own HIP device ordinal and PCI id, and a gpu_metrics reading under load.
Run it in several processes, then compare a slow one with a fast one
(scripts/lab_modes_cmp.py).
"""
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def metrics(box):
    try:
        r = subprocess.run(["rocm-smi", "--showmetrics", "--json"], capture_output=True, text=True, timeout=20)
        raw = json.loads(r.stdout) if r.stdout.strip().startswith("{") else {}
        card = next(iter(raw.values())) if raw else {}
        box["m"] = {k: card.get(k) for k in ("current_gfxclk (MHz)", "current_socket_power (W)",
                                             "average_gfxclk_frequency (MHz)", "current_uclk (MHz)",
                                             "throttle_status", "indep_throttle_status")}
    except Exception as e:  # noqa: BLE001 (diagnostic)
        box["m"] = repr(e)


def timed(fn, s, reps, warm):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def va(t):
    p = t.data_ptr()
    return {"mod_2MiB": p % (2 << 20), "mod_1GiB": p % (1 << 30), "hex": hex(p)}


def main():
    out_path = sys.argv[1]
    dev = torch.device("cuda", 0)
    b = workloads.make("mixed")
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    hint = b.algo_bytes // b.n
    lab = lvlip.lab()
    lab.lvlip_lab_flat_stamps.restype = ctypes.c_int
    lab.lvlip_lab_flat_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]

    def step():
        lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                        lvlip.KERNEL_AUTO, 0, 0, hint)

    step()
    torch.cuda.synchronize()
    want = out.cpu().numpy().copy()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    ms = timed(step, s, 200, 50)
    gbps = b.algo_bytes / ms / 1e6
    box = {}
    th = threading.Thread(target=lambda: (time.sleep(0.3), metrics(box)))
    th.start()
    ms2 = timed(step, s, 4000, 0)
    th.join()
    # the window read probe (bench diag window_c4)
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    nb = base.numel() & ~1023
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    pms = timed(lambda: lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(), 4, 4, 1, cus * 2,
                                                  s.cuda_stream), s, 20, 3)
    # stamped launches
    L = 20
    grid = (b.n + 255) // 256
    st = torch.zeros((L, grid * 4), dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for k in range(L):
        rc = lab.lvlip_lab_flat_stamps(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), st[k].data_ptr(),
                                       grid * 32, s.cuda_stream)
        assert rc == grid, rc
    e1.record(s)
    torch.cuda.synchronize()
    sms = e0.elapsed_time(e1) / L
    assert np.array_equal(out.cpu().numpy(), want), "stamped k_flat2 differs from AUTO"
    a = st.cpu().numpy().reshape(L, grid, 4)
    t_s, t_e, hw = a[:, :, 0], a[:, :, 1], a[:, :, 2]
    z = t_s.min(axis=1, keepdims=True)
    rs, re_ = (t_s - z) / 100.0, (t_e - z) / 100.0  # us (100 MHz)
    xcc = (hw & 0xF).astype(np.int64)
    hid = hw >> 8
    cu = (hid >> 8) & 0xF
    sh = (hid >> 12) & 0x1
    se = (hid >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    per = []
    for k in range(L):
        d = re_[k] - rs[k]
        rec = {"span_us": round(float(re_[k].max()), 2),
               "wg_dur_us_p10_p50_p90": [round(float(np.percentile(d, q)), 2) for q in (10, 50, 90)],
               "by_xcd": {}}
        for x in range(8):
            m = xcc[k] == x
            if m.any():
                rec["by_xcd"][x] = {"wgs": int(m.sum()), "end_max_us": round(float(re_[k][m].max()), 2),
                                    "dur_p50_us": round(float(np.median(d[m])), 2),
                                    "busy_us": round(float(d[m].sum()) / max(1, len(np.unique(cu_key[k][m]))), 2),
                                    "cus": int(len(np.unique(cu_key[k][m])))}
        # first-generation workgroups: how many start within 2 us of the first
        rec["wgs_started_first_2us"] = int((rs[k] < 2.0).sum())
        per.append(rec)
    # block -> XCD map of the first launch (block b on XCD b % 8?)
    blk_xcd_ok = float((xcc[0] == (np.arange(grid) % 8)).mean())
    res = {
        "pid": os.getpid(), "GBps": round(gbps, 1), "ms": round(ms, 5),
        "GBps_long_window": round(b.algo_bytes / ms2 / 1e6, 1), "metrics_under_load": box.get("m"),
        "probe_window_c4_GBps": round(nb / pms / 1e6, 1),
        "stamped_ms": round(sms, 5), "stamped_GBps": round(b.algo_bytes / sms / 1e6, 1),
        "block_on_xcd_b_mod_8_frac": blk_xcd_ok,
        "va": {"base": va(base), "descs": va(descs), "out": va(out), "stamps": va(st)},
        "device": {"name": torch.cuda.get_device_name(dev),
                   "pci_bus_id": getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", None),
                   "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
                   "ROCR_VISIBLE_DEVICES": os.environ.get("ROCR_VISIBLE_DEVICES")},
        "launches": per,
        "median_span_us": round(float(np.median([p["span_us"] for p in per[2:]])), 2),
        "raw_launch_5": a[5].tolist(),
    }
    print(json.dumps({k: res[k] for k in ("pid", "GBps", "GBps_long_window", "probe_window_c4_GBps",
                                          "stamped_GBps", "median_span_us", "metrics_under_load",
                                          "block_on_xcd_b_mod_8_frac")}), flush=True)
    print("va", json.dumps(res["va"]), flush=True)
    print("launch 5 by xcd", json.dumps(per[5]["by_xcd"]), flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
