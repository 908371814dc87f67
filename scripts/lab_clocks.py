#!/usr/bin/env python3
"""Lab: the mixed line's process-to-process spread against the GPU's clocks.

  python scripts/lab_clocks.py out.json [windows]

One process: the mixed batch in HBM, a 250-ms settle, then `windows` windows
of ~1.5 s of back-to-back AUTO launches each.  While a window's launches run,
a thread reads `rocm-smi --showmetrics --json` (read-only: the driver's
gpu_metrics table — average gfx/soc/memory/fabric clocks, power, throttle
status), so the reading is taken under load.  Writes each window's GB/s (HIP
events) next to its metrics reading.  Run it in several processes to see
whether the slow and fast modes of DESIGN.md §5 follow a clock.
"""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))
import torch  # noqa: E402

import lvlip  # noqa: E402
import workloads  # noqa: E402


def metrics(box):
    try:
        r = subprocess.run(["rocm-smi", "--showmetrics", "--json"], capture_output=True, text=True, timeout=20)
        box["raw"] = json.loads(r.stdout) if r.stdout.strip().startswith("{") else r.stdout[-2000:]
    except Exception as e:  # noqa: BLE001 (diagnostic)
        box["raw"] = repr(e)


def main():
    out_path = sys.argv[1]
    windows = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    wl = os.environ.get("CLK_WORKLOAD", "mixed")
    dev = torch.device("cuda", 0)
    b = workloads.make(wl)
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    hint = b.algo_bytes // b.n

    mode = os.environ.get("CLK_MODE", "auto")
    if mode == "probe":
        # the bench's window read probe over the same buffer (4 KiB chunks dealt
        # round robin, 8 waves/CU: no checksum work, plain reads)
        lab = lvlip.lab()
        sink = torch.zeros(1, dtype=torch.int32, device=dev)
        nb = base.numel() & ~1023
        cus = torch.cuda.get_device_properties(dev).multi_processor_count

        def step():
            lab.lvlip_lab_probe_chunk(base.data_ptr(), nb, sink.data_ptr(), 4, 4, 1, cus * 2, s.cuda_stream)
    else:
        kern = lvlip.KERNEL_NAMES[mode]

        def step():
            lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,
                            kern, 0, 0, hint)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    res = []
    for w in range(windows):
        n = 6000
        box = {}
        th = threading.Thread(target=lambda: (time.sleep(0.4), metrics(box)))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        th.start()
        for _ in range(n):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        th.join()
        ms = e0.elapsed_time(e1) / n
        gbps = (nb if mode == "probe" else b.algo_bytes) / ms / 1e6  # probe: bytes read
        res.append({"window": w, "GBps": round(gbps, 1), "ms": round(ms, 5), "metrics": box.get("raw")})
        card = next(iter(box["raw"].values())) if isinstance(box.get("raw"), dict) else {}
        print(f"{wl} {mode} window {w}: {gbps:.1f} GB/s, gfxclk {card.get('current_gfxclk (MHz)')} "
              f"power {card.get('current_socket_power (W)')} W", flush=True)
    with open(out_path, "w") as f:
        json.dump({"workload": wl, "mode": mode, "pid": os.getpid(), "windows": res}, f)


if __name__ == "__main__":
    main()
