"""Child process: level-ip's TX path with and without the batch-and-dispatch
step, on the reference stack itself.

    python tests/ref_tx_batch_child.py REQUESTS.json OUT.json LIB MODE [OPTIONS]

LIB and MODE:
  oracle/_ref/libref_fixclock.so  unbatched  level-ip as it is (its ISS clock
                                             fixed, oracle/ref_clock.c): every
                                             frame checksummed on the CPU at
                                             tcp_transmit_skb / icmpv4_reply /
                                             ip_output and written at once
  oracle/_ref/libref_txq.so       gpu        the same objects with the three TX
                                             checksums deferred and ip_output's
                                             dst_neigh_output queueing the frame
                                             (oracle/ref_txq.c); each flush fills
                                             the whole queue with ONE
                                             lvlip_txq_fill (lvlip_tx_checksum_
                                             skb_list through a context: on the
                                             GPU above the context's cpu_max
                                             frames, LVLIP_CPU_MAX from the
                                             environment; the CPU fill when the
                                             call fails), then hands every skb
                                             to the real dst_neigh_output
  oracle/_ref/libref_txq.so       oracle     the same, the queue's fields filled
                                             by the CPU oracle (skb_oracle.tx_fill)

OPTIONS (JSON, all optional):
  write_bytes  bytes of the one tcp_send (default 2001; smss is 536,
               src/tcp.c:115, so 2 MiB make ~3 900 segments)
  send_next    tcp_send_next's amount (default 5: the SYN again and four
               segments; 0 = every queued skb)
  inject       queue a malformed frame (IPv4 version 6) after tcp_send_next:
               the gpu mode first checks that the batch call refuses the queue
               with LVLIP_EINVAL leaving every queued byte untouched, then the
               flush drops that one frame and fills the rest
  device       the context's device (default 0; an invalid index makes
               lvlip_csum_ctx_create fail, so the flush fills on the CPU)
  hashes       report frames as sha1 hex digests instead of their bytes
  slab         bytes: with oracle/_ref/libref_{txq,fixclock}_slab.so, every
               skb buffer from one slab (oracle/ref_slab.c), which the batched
               run's context registers LVLIP_REG_DMA
  hold         the queue holds each skb by reference instead of copying it
               (lvlip_txq_set_hold, oracle/ref_txq.c): the flush fills the
               frame array with ONE lvlip_tx_checksum, and a retransmit
               (skb_reset_header) flushes a held frame before rewriting it
  time         the tap is /dev/null and OUT.json gets the wall and CPU time
               of the TCP phase (sends + flush) and the echo phase; the
               context is made (and its GPU path warmed) before the clock
               starts

The stack runs: an ARP request (the reply teaches nothing to batch: arp_rcv
writes it directly, src/arp.c); a TCP connect (SYN with options,
src/tcp.c:156-168), write_bytes queued (src/tcp_output.c:445-478),
tcp_send_next (the SYN again and segments, src/tcp_output.c:198-225), a bare ACK
and a RST (src/tcp_output.c:247-267, :480-498), then flush; then the echo
requests of REQUESTS.json into ip_rcv (-> icmpv4_reply -> ip_output), then
flush.  fd 0 (the stack's tun fd, a zeroed static, src/tuntap_if.c:5) is one
end of a socketpair; a reader thread collects every frame the stack writes, in
order.  OUT.json: {"frames": frames in tap order (hex, or sha1 with hashes),
"batches": frames per flush, "deferred": CPU checksum computations the TX path
deferred per flush, "reports": per flush the fill's report and the context's
counters, "untouched": the malformed queue's check, "early_frames" / "reheld": the
frames the hold mode sent before a retransmit rewrote them, and those it lost
(0), "time": the timings}.
"""
import ctypes
import json
import os
import socket
import struct
import sys
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(HERE, "golden"), HERE, os.path.join(ROOT, "level-ip_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import make_golden  # noqa: E402  (SkBuff, _frame_to_skb: test infrastructure)

END = b"--end-of-run--"


class TxqReport(ctypes.Structure):  # oracle/ref_txq.c: struct lvlip_txq_report
    _fields_ = [("frames", ctypes.c_int), ("rc", ctypes.c_int), ("cpu", ctypes.c_int), ("dropped", ctypes.c_int)]


def main(req_path: str, out_path: str, so_path: str, mode: str, opts_json: str = "{}"):
    import hashlib
    import time

    opts = json.loads(opts_json)
    write_bytes = int(opts.get("write_bytes", 2001))
    send_next = int(opts.get("send_next", 5))
    timing = bool(opts.get("time", False))
    with open(req_path) as f:
        requests = [bytes.fromhex(h) for h in json.load(f)]
    lib = ctypes.CDLL(so_path)
    got = []
    if timing:
        nul = os.open(os.devnull, os.O_WRONLY)
        os.dup2(nul, 0)
        th = None
    else:
        a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
        os.dup2(a.fileno(), 0)

        def reader():
            while True:
                d = b.recv(65536)
                if d == END:
                    return
                got.append(hashlib.sha1(d).hexdigest() if opts.get("hashes") else d.hex())

        th = threading.Thread(target=reader, daemon=True)
        th.start()
    if opts.get("slab"):
        lib.lvlip_slab_init.argtypes = [ctypes.c_size_t]
        lib.lvlip_slab_base.restype = ctypes.c_void_p
        assert lib.lvlip_slab_init(int(opts["slab"])) == 0
    lib.netdev_init()
    lib.route_init()
    lib.arp_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    lib.ip_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    tap_mac = bytes.fromhex("0a1b2c3d4e5f")
    tap_ip, stack_ip = (10, 0, 0, 5), (10, 0, 0, 4)
    arp = (b"\xff" * 6 + tap_mac + b"\x08\x06" +
           struct.pack("!HHBBH", 1, 0x0800, 6, 4, 1) + tap_mac + bytes(tap_ip) + bytes(6) + bytes(stack_ip))
    lib.arp_rcv(make_golden._frame_to_skb(lib, arp))

    batched = mode != "unbatched"
    batches, deferred, reports = [], [], []
    out = {}
    if batched:
        import lvlip

        lib.lvlip_txq_len.restype = ctypes.c_int
        lib.lvlip_txq_frames.argtypes = [ctypes.POINTER(lvlip.Frame), ctypes.c_int]
        lib.lvlip_txq_fill.argtypes = [ctypes.c_void_p, ctypes.POINTER(TxqReport)]
        lib.lvlip_txq_deferred.restype = ctypes.c_ulong
        lib.lvlip_txq_queue.restype = ctypes.c_void_p
        lib.lvlip_txq_inject.argtypes = [ctypes.c_char_p, ctypes.c_uint]
        lib.lvlip_txq_set_ctx.argtypes = [ctypes.c_void_p]
        lib.lvlip_txq_flush.argtypes = [ctypes.c_void_p, ctypes.POINTER(TxqReport)]
        lib.lvlip_txq_early_frames.restype = ctypes.c_ulong
        lib.lvlip_txq_reheld.restype = ctypes.c_ulong
        if opts.get("hold"):
            assert lib.lvlip_txq_set_hold(1) == 0
    ctxs = []

    def context():
        """The flush's context, made at the first flush (after the TCP sends:
        the HIP runtime's start-up draws from rand(), which generate_iss,
        src/tcp.c:153, must see unseeded as in the unbatched run); None when
        it cannot be made (an invalid device: the flush fills on the CPU)."""
        if not ctxs:
            try:
                ctxs.append(lvlip.Context(int(opts.get("device", 0))))
                lib.lvlip_txq_set_ctx(ctxs[0]._h)
                if opts.get("slab"):
                    assert lvlip.lib().lvlip_csum_register(ctxs[0]._h, lib.lvlip_slab_base(), int(opts["slab"]),
                                                           lvlip.REG_DMA) == 0
            except lvlip.LvlipError as e:
                out["context_error"] = e.rc
                ctxs.append(None)
        return ctxs[0]

    def queued_bytes():
        n = lib.lvlip_txq_len()
        arr = (lvlip.Frame * max(n, 1))()
        assert lib.lvlip_txq_frames(arr, n) == n
        return [ctypes.string_at(arr[k].head, arr[k].len) for k in range(n)]

    timed_stats = {}

    def flush():
        if not batched:
            return
        if timing and mode == "gpu":
            # the clock is running: ONE C call (fill, then send); the report
            # and the context's counters are read after the clock stops
            ctx = context()
            rep = TxqReport()
            sent = lib.lvlip_txq_flush(ctx._h if ctx is not None else None, ctypes.byref(rep))
            if sent < 0:
                raise SystemExit(f"lvlip_txq_flush: {sent}")
            reports.append({"frames": rep.frames, "rc": rep.rc, "cpu": rep.cpu, "dropped": rep.dropped})
            batches.append(sent)
            return
        n = lib.lvlip_txq_len()
        if mode == "gpu":
            ctx = context()
            if opts.get("inject") and "untouched" not in out and ctx is not None:
                # the batch call itself on the queue with its malformed frame
                before = queued_bytes()
                if opts.get("hold"):
                    arr = (lvlip.Frame * n)()
                    assert lib.lvlip_txq_frames(arr, n) == n
                    rc = lvlip.lib().lvlip_tx_checksum(ctx._h, arr, n)
                else:
                    rc = lvlip.lib().lvlip_tx_checksum_skb_list(ctx._h, lib.lvlip_txq_queue())
                out["untouched"] = {"rc": rc, "same": queued_bytes() == before}
            s0 = ctx.stats() if ctx is not None else None
            rep = TxqReport()
            rc = lib.lvlip_txq_fill(ctx._h if ctx is not None else None, ctypes.byref(rep))
            if rc < 0:
                raise SystemExit(f"lvlip_txq_fill: {rc} (queue {n})")
            r = {"frames": rep.frames, "rc": rep.rc, "cpu": rep.cpu, "dropped": rep.dropped}
            if s0 is not None:
                s1 = ctx.stats()
                r.update({k: s1[k] - s0[k] for k in ("gpu_calls", "cpu_calls", "pieces", "h2d_bytes")})
            reports.append(r)
            n -= rep.dropped
        else:
            import skb_oracle

            arr = (lvlip.Frame * max(n, 1))()
            assert lib.lvlip_txq_frames(arr, n) == n
            for k in range(n):
                buf = (ctypes.c_char * arr[k].len).from_address(arr[k].head)
                f = bytearray(buf.raw)
                skb_oracle.tx_fill(f)
                ctypes.memmove(arr[k].head, bytes(f), len(f))
        assert lib.lvlip_txq_send() == n
        batches.append(n)
        deferred.append(int(lib.lvlip_txq_deferred()))

    if timing and batched and mode == "gpu":
        # warm: the context and its GPU path (pinned pages, kernel load) before the clock
        ctx = context()
        if ctx is not None:
            import workloads

            cm = ctx.cpu_max
            ctx.set_cpu_max(0)
            ctx.tx_checksum(workloads.frames(64, seed=1))
            ctx.set_cpu_max(cm)

    # TCP (tests/ref_stack_child.py's sequence)
    lib.sk_alloc.restype = ctypes.c_void_p
    lib.sk_alloc.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.sock_init_data.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.tcp_v4_connect.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.tcp_send.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
    lib.tcp_send_next.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.tcp_send_ack.argtypes = [ctypes.c_void_p]
    lib.tcp_send_reset.argtypes = [ctypes.c_void_p]
    tcp_ops = ctypes.addressof(ctypes.c_char.in_dll(lib, "tcp_ops"))
    sk = lib.sk_alloc(tcp_ops, 6)
    sock = ctypes.create_string_buffer(1024)  # struct socket (include/socket.h:59-71), zeroed
    lib.sock_init_data(ctypes.addressof(sock), sk)
    addr = struct.pack("=H", socket.AF_INET) + struct.pack("!H", 8000) + bytes(tap_ip) + bytes(8)
    addr_buf = ctypes.create_string_buffer(addr, len(addr))
    lib.tcp_v4_connect(sk, ctypes.addressof(addr_buf), 16, 0)
    payload = ((np.arange(write_bytes, dtype=np.uint64) * 7 + 3) & 0xFF).astype(np.uint8).tobytes()
    if timing and batched and mode == "gpu" and ctxs and ctxs[0] is not None:
        timed_stats["s0"] = ctxs[0].stats()
    t0, c0 = time.perf_counter(), time.process_time()
    lib.tcp_send(sk, payload, len(payload))
    lib.tcp_send_next(sk, send_next if send_next > 0 else (write_bytes // 536 + 8))
    if opts.get("inject") and batched:
        # a frame ip_output could never have built: IPv4 version 6
        n = lib.lvlip_txq_len()
        arr = (lvlip.Frame * max(n, 1))()
        lib.lvlip_txq_frames(arr, n)
        bad = bytearray(ctypes.string_at(arr[n - 1].head, arr[n - 1].len))
        bad[14] = 0x65
        assert lib.lvlip_txq_inject(bytes(bad), len(bad)) == 0
    lib.tcp_send_ack(sk)
    lib.tcp_send_reset(sk)
    flush()
    t_tcp = (time.perf_counter() - t0, time.process_time() - c0)
    if "s0" in timed_stats:  # the TCP phase's counters (the flush before the SYN retransmit included)
        s1 = ctxs[0].stats()
        reports[-1].update({k: s1[k] - timed_stats["s0"][k] for k in ("gpu_calls", "cpu_calls", "pieces", "h2d_bytes")})
    # echo requests -> icmpv4_reply
    skbs = [make_golden._frame_to_skb(lib, req) for req in requests]
    t0, c0 = time.perf_counter(), time.process_time()
    for skb in skbs:
        lib.ip_rcv(skb)
    flush()
    t_echo = (time.perf_counter() - t0, time.process_time() - c0)
    if th is not None:
        os.write(0, END)
        th.join(timeout=120)
        if th.is_alive():
            raise SystemExit("reader did not see the end marker")
    for c in ctxs:
        if c is not None:
            lib.lvlip_txq_set_ctx(None)  # the harness keeps no pointer to a destroyed context
            c.close()
    out.update({"frames": got, "batches": batches, "deferred": deferred, "reports": reports})
    if batched:
        out.update({"early_frames": int(lib.lvlip_txq_early_frames()), "reheld": int(lib.lvlip_txq_reheld())})
    if timing:
        out["time"] = {"tcp_wall_s": t_tcp[0], "tcp_cpu_s": t_tcp[1], "echo_wall_s": t_echo[0],
                       "echo_cpu_s": t_echo[1]}
    with open(out_path, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main(*sys.argv[1:6])
