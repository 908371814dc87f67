"""Lab (diagnostic, not the product): the echo reply's store form (f4,
lvlip_icmp_echo_reply_dev[_ex]) on the mixed config's 2M frames in HBM.
Both reply kernels write the reply's type byte and checksum field into each
request frame; fr_store_echo_reply (flat_src.h) does it as three byte stores
(variant 0) or as two u16 stores with a cache policy (2 sc0, 3 sc1, 4 sc0 sc1,
5 nt sc1, 6 nt sc0 sc1); for flags 0 also as one 16-B store of the patched
window chunk (1 plain, 7 nontemporal; k_echo_reply's echo_reply_chunk_store).
The first run (profiles/r05_echo_store.json) timed 0 and 2-6; this one 0, 2
and the chunk stores.  Modes: 4 = LVLIP_ECHO_FULL on the flat sweep, 5 =
flags 0 (k_echo_reply, the field from the request's field).  Each launch is
timed alone with HIP events after the request bytes are restored, as
bench.py's echo_reply_timing does; rounds interleave the variants.  Every
variant's frames are checked equal to variant 0's from the same pristine
frames first.

    python scripts/lab_echo_store.py OUT.json [ROUNDS]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "level-ip_amd")]

VARIANTS = {4: (0,), 5: (0, 8)}  # 1 / 7 (mode 5): the chunk store, last in commit 72b8c4f; 8: three-chunk window


def main(path, rounds=5):
    import torch

    import bench
    import lvlip

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    base, fd, pay = bench.mixed_frames_hbm(lvlip, torch, dev)
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).to(dev)
    lvlip.tx_checksum_dev(base, fdt, stream=stream)  # valid frames, as bench.py --frames
    icmp = pay["start_sum"] == 0
    t_off = torch.from_numpy((fd["offset"][icmp] + 34).astype(np.int64)).to(dev)
    base[t_off] = 8
    base[t_off + 1] = 0
    torch.cuda.synchronize()
    pristine = base.clone()
    msg_bytes = int(pay["len"][icmp].sum())
    n = fd.size
    res = {"frames": n, "icmp_frames": int(icmp.sum()), "icmp_bytes": msg_bytes, "parity": {}, "us": {}}
    for mode in (4, 5):
        want = None
        for v in VARIANTS[mode]:
            base.copy_(pristine)
            lvlip.frames_variant_dev(mode, v, base, fdt, stream=stream)
            torch.cuda.synchronize()
            if want is None:
                want = base.clone()
            ok = bool(torch.equal(base, want))
            res["parity"][f"m{mode}v{v}"] = ok
            assert ok, (mode, v)
        del want
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for mode in (4, 5):
            for v in VARIANTS[mode]:
                ts = []
                for _ in range(5):
                    base[t_off] = 8
                    base[t_off + 1] = 0
                    torch.cuda.synchronize()
                    e0.record(stream)
                    lvlip.frames_variant_dev(mode, v, base, fdt, stream=stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                key = f"m{mode}v{v}"
                res["us"].setdefault(key, []).append(round(sorted(ts)[2], 1))
                print(key, res["us"][key], flush=True)
    res["median_us"] = {k: float(np.median(v)) for k, v in res["us"].items()}
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print("median", res["median_us"], flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
