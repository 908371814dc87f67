"""Child process: an RX burst through level-ip's own stack, as it is and with
both batch-and-dispatch steps (VERDICT r05 Next #3).

    python tests/ref_scale_child.py OUT.json LIB MODE OPTIONS

LIB and MODE:
  oracle/_ref/libref_rxq.so    unbatched  level-ip as it is: netdev_rx_loop's
                                          skbs (alloc_skb(BUFLEN), the frame at
                                          skb->data) through netdev_receive ->
                                          ip_rcv -> icmpv4_reply -> ip_output ->
                                          tun_write, one at a time, every
                                          checksum on the CPU
                                          (lvlip_rxq_receive_all, C)
  oracle/_ref/libref_rxtxq.so  batched    the same skbs in one sk_buff_head: ONE
                                          lvlip_rx_verify_skb_list through a
                                          context, the dispatch loop
                                          (lvlip_rxq_dispatch: ip_rcv with its
                                          header sum answered by the verdict,
                                          ARP to arp_rcv, drops freed), the
                                          replies' three checksums deferred and
                                          their frames queued, then ONE flush
                                          (lvlip_txq_fill) and the sends
                                          (oracle/ref_rxq.c, oracle/ref_txq.c)
  oracle/_ref/libref_rxtxq.so  oracle     the batched composition with the CPU
                                          oracle's verdicts and TX fill

The context follows LVLIP_CPU_MAX from the environment (unset: the library's
default threshold; 0: every call on the GPU).

With oracle/_ref/libref_rxtxq_slab.so and the option "slab": bytes, every
skb's buffer comes from one slab (oracle/ref_slab.c) that the context
registers LVLIP_REG_DMA, the allocator INTEGRATION.md §2b'' recommends: the
batch calls then move the burst's frames with the copy engine instead of
gathering them on the CPU.

With the option "hold", the TX queue holds each reply's skb (the RX skb
icmpv4_reply answered in) by reference instead of copying it
(lvlip_txq_set_hold, oracle/ref_txq.c): the flush fills the held frames with
ONE lvlip_tx_checksum, sends them and frees the skbs.

OPTIONS (JSON): {"n": frames in the burst (after one ARP request), "seed",
"kinds": "all" (every ip_rcv drop reason, tests/ref_rx_cases.py) or "ok" (echo
requests only), "flags": the RX verify flags, "device": the context's device (an
invalid index: no context, both calls on the CPU), "time": [burst sizes] (tap =
/dev/null; each size timed after an untimed burst of the same size; the
context made and warmed first)}.

OUT.json: {"frames": sha1 of every frame the stack wrote, in order;
"verdicts": counts per verdict; "cpu_header_sums" / "batch_header_sums" (ip_rcv's
header sums on the CPU / answered by the batch); "reports": per flush the TX
fill's report and the context's counters; "time": per burst size the wall and
CPU time of the whole burst (verify, dispatch, replies, flush, sends)}."""
import ctypes
import hashlib
import json
import os
import socket
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "level-ip_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import ref_rx_cases  # noqa: E402

END = b"--end-of-run--"
ARP = (b"\xff" * 6 + ref_rx_cases.TAP_MAC + b"\x08\x06" + bytes.fromhex("0001080006040001") +
       ref_rx_cases.TAP_MAC + ref_rx_cases.TAP_IP + bytes(6) + ref_rx_cases.STACK_IP)


class SkBuffHead(ctypes.Structure):  # include/skbuff.h:25-29
    _fields_ = [("next", ctypes.c_void_p), ("prev", ctypes.c_void_p), ("qlen", ctypes.c_uint32)]


class TxqReport(ctypes.Structure):  # oracle/ref_batch.h: struct lvlip_txq_report
    _fields_ = [("frames", ctypes.c_int), ("rc", ctypes.c_int), ("cpu", ctypes.c_int), ("dropped", ctypes.c_int)]


class BurstReport(ctypes.Structure):  # oracle/ref_batch.h: struct lvlip_rxtxq_report
    _fields_ = [("rx_cpu", ctypes.c_int), ("queued", ctypes.c_int), ("sent", ctypes.c_int), ("tx", TxqReport)]


def burst(n, seed, kinds):
    rng = np.random.default_rng(seed)
    ks = list(ref_rx_cases.KINDS) if kinds == "all" else ["ok"]
    frames = [ARP] + [ref_rx_cases.echo_frame(ks[int(rng.integers(0, len(ks)))], rng, i % 16384) for i in range(n)]
    off = np.zeros(len(frames), np.uint64)
    ln = np.array([len(f) for f in frames], np.uint32)
    off[1:] = np.cumsum(ln[:-1])
    return np.frombuffer(b"".join(frames), np.uint8).copy(), off, ln


def main(out_path, so_path, mode, opts_json):
    opts = json.loads(opts_json)
    lib = ctypes.CDLL(so_path)
    got = []
    th = None
    if opts.get("time"):
        os.dup2(os.open(os.devnull, os.O_WRONLY), 0)
    else:
        a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
        os.dup2(a.fileno(), 0)

        def reader():
            while True:
                d = b.recv(65536)
                if d == END:
                    return
                got.append(hashlib.sha1(d).hexdigest())

        th = threading.Thread(target=reader, daemon=True)
        th.start()
    if opts.get("slab"):
        lib.lvlip_slab_init.argtypes = [ctypes.c_size_t]
        lib.lvlip_slab_base.restype = ctypes.c_void_p
        assert lib.lvlip_slab_init(int(opts["slab"])) == 0
    lib.netdev_init()
    lib.route_init()
    for fn in ("lvlip_rxq_fill",):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.lvlip_rxq_receive_all.argtypes = [ctypes.c_void_p]
    lib.lvlip_rxq_computed.restype = ctypes.c_ulong
    lib.lvlip_rxq_skipped.restype = ctypes.c_ulong
    batched = mode != "unbatched"
    flags = int(opts.get("flags", 0))
    ctx = None
    out_ctx_error = None
    hist, reports = {}, []
    if batched:
        import lvlip

        lib.lvlip_rxq_dispatch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.lvlip_rxq_verify.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]
        lib.lvlip_txq_fill.argtypes = [ctypes.c_void_p, ctypes.POINTER(TxqReport)]
        lib.lvlip_txq_send.restype = ctypes.c_int
        lib.lvlip_txq_len.restype = ctypes.c_int
        lib.lvlip_txq_frames.argtypes = [ctypes.POINTER(lvlip.Frame), ctypes.c_int]
        lib.lvlip_txq_set_ctx.argtypes = [ctypes.c_void_p]
        lib.lvlip_rxtxq_burst.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.POINTER(BurstReport)]
        if opts.get("hold"):
            assert lib.lvlip_txq_set_hold(1) == 0
        if mode == "batched":
            try:
                ctx = lvlip.Context(int(opts.get("device", 0)))
            except lvlip.LvlipError as e:  # no device: both calls fall back to the CPU
                ctx, out_ctx_error = None, e.rc
            if ctx is not None:
                lib.lvlip_txq_set_ctx(ctx._h)
            if ctx is not None and opts.get("slab"):
                assert lvlip.lib().lvlip_csum_register(ctx._h, lib.lvlip_slab_base(), int(opts["slab"]),
                                                       lvlip.REG_DMA) == 0
            if ctx is not None and opts.get("time"):  # warm the GPU path before any clock
                import workloads

                cm = ctx.cpu_max
                ctx.set_cpu_max(0)
                fr = workloads.frames(64, seed=1)
                ctx.tx_checksum(fr)
                ctx.rx_verify(fr, flags)
                ctx.set_cpu_max(cm)

    def run_burst(blob, off, ln):
        """One burst: the skbs queued (untimed, netdev_rx_loop's reads), then
        the stack over them, as ONE C call in either form (level-ip as it is:
        lvlip_rxq_receive_all; batched: lvlip_rxtxq_burst, oracle/ref_rxtxq.c);
        returns (wall s, CPU s, (verdicts, report) or None)."""
        q = SkBuffHead()
        q.next = q.prev = ctypes.addressof(q)
        n = len(ln)
        assert lib.lvlip_rxq_fill(ctypes.addressof(q), blob.ctypes.data, off.ctypes.data, ln.ctypes.data, n) == n
        v = np.zeros(n, np.uint8)
        if mode == "batched":
            s0 = ctx.stats() if ctx is not None else None
            br = BurstReport()
            t0, c0 = time.perf_counter(), time.process_time()
            m = lib.lvlip_rxtxq_burst(ctx._h if ctx is not None else None, ctypes.addressof(q), flags,
                                      v.ctypes.data, n, ctypes.byref(br))
            wall, cpu = time.perf_counter() - t0, time.process_time() - c0
            assert m == n, m
            assert br.sent == br.tx.frames
            r = {"queued": br.queued, "frames": br.tx.frames, "rc": br.tx.rc, "cpu": br.tx.cpu,
                 "dropped": br.tx.dropped, "rx_cpu_fallback": br.rx_cpu}
            if s0 is not None:
                s1 = ctx.stats()
                r.update({k: s1[k] - s0[k] for k in ("gpu_calls", "cpu_calls", "pieces", "h2d_bytes")})
            return wall, cpu, (v, r)
        t0, c0 = time.perf_counter(), time.process_time()
        if not batched:
            assert lib.lvlip_rxq_receive_all(ctypes.addressof(q)) == n
            return time.perf_counter() - t0, time.process_time() - c0, None
        # mode "oracle": the oracle's verdicts and TX fill (the harness's own check on the CPU)
        import skb_oracle

        # the walker's frame: skb->data .. skb->end (BUFLEN, the read's zero tail)
        frames = [bytes(blob[int(o):int(o) + int(ln_)]) + bytes(1600 - int(ln_)) for o, ln_ in zip(off, ln)]
        v[:] = [skb_oracle.rx_verdict(f, flags) for f in frames]
        assert lib.lvlip_rxq_dispatch(ctypes.addressof(q), v.ctypes.data, 1) == n
        nq = lib.lvlip_txq_len()
        arr = (lvlip.Frame * max(nq, 1))()
        assert lib.lvlip_txq_frames(arr, nq) == nq
        for k in range(nq):
            f = bytearray(ctypes.string_at(arr[k].head, arr[k].len))
            skb_oracle.tx_fill(f)
            ctypes.memmove(arr[k].head, bytes(f), len(f))
        assert lib.lvlip_txq_send() == nq
        wall, cpu = time.perf_counter() - t0, time.process_time() - c0
        r = {"queued": nq, "frames": nq, "rc": 0, "cpu": 0, "dropped": 0, "rx_cpu_fallback": 0}
        return wall, cpu, (v, r)

    out = {}
    if opts.get("time"):
        res = {}
        for n in opts["time"]:
            blob, off, ln = burst(n, int(opts.get("seed", 1)), opts.get("kinds", "ok"))
            run_burst(blob, off, ln)  # untimed: the same size once
            walls, cpus = [], []
            for _ in range(int(opts.get("reps", 3))):
                w, c, extra = run_burst(blob, off, ln)
                walls.append(w)
                cpus.append(c)
            res[str(n)] = {"wall_us": round(min(walls) * 1e6, 1), "cpu_us": round(min(cpus) * 1e6, 1),
                           "wall_us_per_frame": round(min(walls) * 1e6 / (n + 1), 3),
                           "cpu_us_per_frame": round(min(cpus) * 1e6 / (n + 1), 3)}
            if extra is not None:
                res[str(n)]["flush"] = extra[1]
        out["time"] = res
    else:
        blob, off, ln = burst(int(opts["n"]), int(opts.get("seed", 1)), opts.get("kinds", "all"))
        _, _, extra = run_burst(blob, off, ln)
        if extra is not None:
            v, r = extra
            hist = {int(k): int(c) for k, c in zip(*np.unique(v, return_counts=True))}
            reports.append(r)
        os.write(0, END)
        th.join(timeout=120)
        if th.is_alive():
            raise SystemExit("reader did not see the end marker")
    if ctx is not None:
        lib.lvlip_txq_set_ctx(None)  # the harness keeps no pointer to a destroyed context
        ctx.close()
    if out_ctx_error is not None:
        out["context_error"] = out_ctx_error
    out.update({"frames": got, "verdicts": hist, "reports": reports,
                "cpu_header_sums": int(lib.lvlip_rxq_computed()), "batch_header_sums": int(lib.lvlip_rxq_skipped())})
    with open(out_path, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main(*sys.argv[1:5])
