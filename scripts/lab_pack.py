#!/usr/bin/env python3
"""Lab: does reading MTU packets as one full and one 46 %-full wave-load each
cost streaming rate?  Times, on one tcp1500-shaped buffer (1M x 1504-B slots),
the wave-contiguous 1 KiB probe (MODE 2), the packetized probe (MODE 4: per
packet one full 1 KiB load plus one with lanes 0..29), and k_stream (AUTO),
interleaved rounds in one process (diagnostic, GPU box)."""
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
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    lab = lvlip.lab()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    b = workloads.make("tcp1500")
    base, descs, out = workloads.to_device(b, dev)
    nb = (1 << 20) * 1504
    assert base.numel() >= nb
    res = {}
    variants = [("probe m2 u4 b2", 2, 4, 2), ("probe m2 u8 b2", 2, 8, 2),
                ("pack m4 u2 b2", 4, 2, 2), ("pack m4 u3 b2", 4, 3, 2), ("pack m4 u4 b2", 4, 4, 2),
                ("pack m4 u2 b4", 4, 2, 4), ("pack m4 u3 b4", 4, 3, 4)]
    for _ in range(3):
        for name, mode, u, bpc in variants:
            f = lambda: lab.lvlip_lab_probe(base.data_ptr(), nb, sink.data_ptr(), mode, u, 1, cus * bpc,  # noqa: E731
                                            s.cuda_stream)
            assert f() == 0, name
            res.setdefault(name, []).append(nb / timed(f, s) / 1e6)
        f = lambda: lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), s.cuda_stream,  # noqa: E731
                                    lvlip.KERNEL_AUTO, 0, 0, 1500)
        res.setdefault("k_stream auto", []).append(nb / timed(f, s) / 1e6)
    for k, v in sorted(res.items(), key=lambda kv: -max(kv[1])):
        print(f"{k:18s} GB/s (slot bytes) max {max(v):7.1f}  all {[round(x) for x in v]}")


if __name__ == "__main__":
    main()
