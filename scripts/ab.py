#!/usr/bin/env python3
"""A/B of launch variants on one resident batch (GPU box).

  AB_WORKLOAD=mixed AB_VARIANTS="flat:4:0,flat:8:0,auto:0:0" python scripts/ab.py [out.json]

A variant is kernel:unroll:waves_per_cu[:len_hint] (kernel names as bench.py's
--kernel; len_hint defaults to the batch's average length).  A variant prefixed
"alt/" runs through the library AB_ALT_LIB instead (another revision of the
product, built by scripts/build_ab.sh), so two builds compare in one process;
"splitP/" runs the batch as P launches back to back on the stream.  After a clock
settle, interleaved rounds in one process (AB_ROUNDS, default 5) each time every
variant over 20 launches with HIP events; prints the median GB/s of algorithmic
bytes per variant, and checks that every variant computes the same checksums.
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
    wl = os.environ.get("AB_WORKLOAD", "tcp1500")
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    dev = torch.device("cuda", 0)
    b = workloads.make(wl, n=int(os.environ["AB_N"]) if os.environ.get("AB_N") else None)
    base, descs, out = workloads.to_device(b, dev)
    s = torch.cuda.current_stream(dev)
    hint = b.algo_bytes // b.n
    alt = None
    if os.environ.get("AB_ALT_LIB"):
        import ctypes
        alt = ctypes.CDLL(os.path.abspath(os.environ["AB_ALT_LIB"]))
        alt.lvlip_csum_batch_dev_ex.restype = ctypes.c_int
        alt.lvlip_csum_batch_dev_ex.argtypes = lvlip.SIGNATURES["lvlip_csum_batch_dev_ex"][1]
    variants = []
    for v in os.environ.get("AB_VARIANTS", "auto:0:0").split(","):
        f = v.split(":")
        variants.append((v, f[0], int(f[1], 0), int(f[2]), int(f[3]) if len(f) > 3 else hint))

    def mk(k, u, w, h):
        if k.startswith("split"):  # splitP/kernel: the batch as P launches back to back
            parts, kk = int(k[5:k.index("/")]), k[k.index("/") + 1:]
            cuts = [b.n * q // parts for q in range(parts + 1)]

            def f():
                for lo, hi in zip(cuts[:-1], cuts[1:]):
                    lvlip.batch_dev(base.data_ptr(), descs.data_ptr() + 16 * lo, hi - lo,
                                    out.data_ptr() + 2 * lo, s.cuda_stream, lvlip.KERNEL_NAMES[kk],
                                    u, w, h)
            return f
        if k.startswith("alt/"):
            cfg = lvlip.LaunchCfg(lvlip.KERNEL_NAMES[k[4:]], u, w, h)

            def f():
                rc = alt.lvlip_csum_batch_dev_ex(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),
                                                 s.cuda_stream, ctypes.byref(cfg))
                assert rc == 0, rc
            return f
        return lambda: lvlip.batch_dev(base.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(),
                                       s.cuda_stream, lvlip.KERNEL_NAMES[k], u, w, h)
    timed(mk("auto", 0, 0, hint), s, reps=int(os.environ.get("AB_SETTLE", "400")))  # clock settle
    ref, res = None, {}
    # ablation variants (wrong results by design) are timed, not checked
    nocheck = set(filter(None, os.environ.get("AB_NOCHECK", "").split(",")))
    for rnd in range(rounds):
        for key, k, u, w, h in variants:
            ms = timed(mk(k, u, w, h), s)
            res.setdefault(key, []).append(b.algo_bytes / ms / 1e6)
            if rnd == 0:
                got = out.cpu().numpy().copy()
                ref = got if ref is None else ref
                if key not in nocheck:
                    assert np.array_equal(got, ref), key
    summary = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    for k, v in sorted(summary.items(), key=lambda kv: -kv[1]):
        print(f"{wl} {k:24s} {v:8.1f} GB/s   rounds {[round(x) for x in res[k]]}", flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"workload": wl, "median_GBps": summary, "rounds": res}, f, indent=1)


if __name__ == "__main__":
    main()
