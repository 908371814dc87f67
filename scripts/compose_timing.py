"""Times level-ip's own stack per burst / flush, batched and unbatched
(VERDICT r05 Next #3): where batch-and-dispatch makes level-ip cheaper.

  RX + replies  tests/ref_scale_child.py in time mode: bursts of n echo
                requests (n = 8 .. 32 768, 64-1 400 B payloads, all answered)
                through libref_rxq.so (level-ip as it is) and libref_rxtxq.so
                (one RX verify, the dispatch, one TX flush) with the library's
                default threshold and with threshold 0 (always the GPU)
  TX            tests/ref_tx_batch_child.py in time mode: one tcp_send of
                W bytes (smss 536) sent by tcp_send_next, then the flush,
                for W = 4 KiB .. 32 MiB, unbatched and batched (both thresholds)
  hold_*        the same batched stacks with the TX queue holding each skb by
                reference instead of copying it (oracle/ref_txq.c's hold mode)

The tap is /dev/null; each figure is the best of 3 after an untimed run of
the same size (RX), or one run per process (TX).  Prints one JSON object.

    python scripts/compose_timing.py > gpurun_out/r06_compose.json
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
BURSTS = [8, 64, 512, 4096, 8192, 16384, 32768, 65536, 131072]
WRITES = [4 << 10, 64 << 10, 1 << 20, 8 << 20, 32 << 20]


def env_for(cpu_max):
    env = {k: v for k, v in os.environ.items() if k != "LVLIP_CPU_MAX"}
    if cpu_max is not None:
        env["LVLIP_CPU_MAX"] = str(cpu_max)
    return env


def rx(lib, mode, cpu_max=None, slab=0, hold=False, **extra_env):
    env = env_for(cpu_max)
    env.update({k: str(v) for k, v in extra_env.items()})
    opts = {"time": BURSTS, "kinds": "ok", "seed": 3}
    if slab:
        opts["slab"] = slab
    if hold:
        opts["hold"] = 1
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "o.json")
        subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_scale_child.py"), out,
                        os.path.join(REF, lib), mode, json.dumps(opts)],
                       check=True, stdin=subprocess.DEVNULL, env=env, timeout=900)
        with open(out) as f:
            return json.load(f)["time"]


def tx(lib, mode, w, cpu_max=None, hold=False, slab=0, **extra_env):
    env = env_for(cpu_max)
    env.update({k: str(v) for k, v in extra_env.items()})
    with tempfile.TemporaryDirectory() as d:
        req, out = os.path.join(d, "r.json"), os.path.join(d, "o.json")
        with open(req, "w") as f:
            json.dump([], f)
        subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_tx_batch_child.py"), req, out,
                        os.path.join(REF, lib), mode, json.dumps({"write_bytes": w, "send_next": 0, "time": True, "hold": hold,
                                                             "slab": slab})],
                       check=True, stdin=subprocess.DEVNULL, env=env, timeout=900)
        with open(out) as f:
            o = json.load(f)
        r = {"wall_us": round(o["time"]["tcp_wall_s"] * 1e6, 1), "cpu_us": round(o["time"]["tcp_cpu_s"] * 1e6, 1),
             "frames": (w + 535) // 536 + 4}
        if o.get("reports"):
            r["flush"] = o["reports"][0]
        return r


def main():
    res = {"rx_bursts": BURSTS, "rx": {}, "tx_writes": WRITES, "tx": {}}
    res["rx"]["unbatched"] = rx("libref_rxq.so", "unbatched")
    print("rx unbatched", res["rx"]["unbatched"], file=sys.stderr, flush=True)
    for tag, cm in (("batched_default", None), ("batched_gpu", 0), ("batched_cpu", 1 << 30)):
        res["rx"][tag] = rx("libref_rxtxq.so", "batched", cm)
        print("rx", tag, res["rx"][tag], file=sys.stderr, flush=True)
    # the skbs' buffers from one registered slab (oracle/ref_slab.c): the copy
    # engine moves the bursts, no gather on the CPU
    for tag, cm in (("slab_default", None), ("slab_gpu", 0), ("slab_cpu", 1 << 30)):
        res["rx"][tag] = rx("libref_rxtxq_slab.so", "batched", cm, slab=1 << 30)
        print("rx", tag, res["rx"][tag], file=sys.stderr, flush=True)
    # the replies held by reference, not copied into the TX queue
    for tag, lib, cm, slab in (("hold_default", "libref_rxtxq.so", None, 0), ("hold_gpu", "libref_rxtxq.so", 0, 0),
                               ("hold_cpu", "libref_rxtxq.so", 1 << 30, 0),
                               ("slab_hold_default", "libref_rxtxq_slab.so", None, 1 << 30),
                               ("slab_hold_gpu", "libref_rxtxq_slab.so", 0, 1 << 30),
                               ("slab_hold_cpu", "libref_rxtxq_slab.so", 1 << 30, 1 << 30)):
        res["rx"][tag] = rx(lib, "batched", cm, slab=slab, hold=True)
        print("rx", tag, res["rx"][tag], file=sys.stderr, flush=True)
    for tag, lib, mode, cm, ex in (("unbatched", "libref_fixclock.so", "unbatched", None, {}),
                                   ("batched_default", "libref_txq.so", "gpu", None, {}),
                                   ("batched_gpu", "libref_txq.so", "gpu", 0, {}),
                                   ("batched_cpu", "libref_txq.so", "gpu", 1 << 30, {}),
                                   ("hold_default", "libref_txq.so", "gpu", None, {"hold": True}),
                                   ("hold_gpu", "libref_txq.so", "gpu", 0, {"hold": True}),
                                   ("hold_cpu", "libref_txq.so", "gpu", 1 << 30, {"hold": True}),
                                   # every skb buffer from one registered slab, on both sides
                                   ("unbatched_slab", "libref_fixclock_slab.so", "unbatched", None,
                                    {"slab": 1 << 30}),
                                   ("slab_hold_default", "libref_txq_slab.so", "gpu", None,
                                    {"hold": True, "slab": 1 << 30}),
                                   ("slab_hold_gpu", "libref_txq_slab.so", "gpu", 0, {"hold": True, "slab": 1 << 30}),
                                   ("slab_hold_cpu", "libref_txq_slab.so", "gpu", 1 << 30,
                                    {"hold": True, "slab": 1 << 30})):
        res["tx"][tag] = {str(w): tx(lib, mode, w, cm, **ex) for w in WRITES}
        print("tx", tag, res["tx"][tag], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
