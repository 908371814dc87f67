"""Child process: level-ip's TX path with and without the batch-and-dispatch
step, on the reference stack itself.

    python tests/ref_tx_batch_child.py REQUESTS.json OUT.json LIB MODE

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
                                             lvlip_tx_checksum_skb_list on the
                                             GPU, then hands every skb to the
                                             real dst_neigh_output
  oracle/_ref/libref_txq.so       oracle     the same, the queue's fields filled
                                             by the CPU oracle (skb_oracle.tx_fill)

The stack runs: an ARP request (the reply teaches nothing to batch: arp_rcv
writes it directly, src/arp.c); a TCP connect (SYN with options,
src/tcp.c:156-168), 2 001 B queued (src/tcp_output.c:445-478), tcp_send_next
(the SYN again and four data segments, src/tcp_output.c:198-225), a bare ACK
and a RST (src/tcp_output.c:247-267, :480-498), then flush; then the echo
requests of REQUESTS.json into ip_rcv (-> icmpv4_reply -> ip_output), then
flush.  fd 0 (the stack's tun fd, a zeroed static, src/tuntap_if.c:5) is one
end of a socketpair; a reader thread collects every frame the stack writes, in
order.  OUT.json: {"frames": hex frames in tap order, "batches": frames per
flush, "deferred": CPU checksum computations the TX path deferred per flush}.
"""
import ctypes
import json
import os
import socket
import struct
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(HERE, "golden"), HERE, os.path.join(ROOT, "level-ip_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import make_golden  # noqa: E402  (SkBuff, _frame_to_skb: test infrastructure)

END = b"--end-of-run--"


def main(req_path: str, out_path: str, so_path: str, mode: str):
    with open(req_path) as f:
        requests = [bytes.fromhex(h) for h in json.load(f)]
    lib = ctypes.CDLL(so_path)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    os.dup2(a.fileno(), 0)
    got = []

    def reader():
        while True:
            d = b.recv(65536)
            if d == END:
                return
            got.append(d.hex())

    th = threading.Thread(target=reader, daemon=True)
    th.start()
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
    batches, deferred = [], []
    if batched:
        import lvlip

        lib.lvlip_txq_len.restype = ctypes.c_int
        lib.lvlip_txq_frames.argtypes = [ctypes.POINTER(lvlip.Frame), ctypes.c_int]
        lib.lvlip_txq_fill_gpu.argtypes = [ctypes.c_void_p]
        lib.lvlip_txq_deferred.restype = ctypes.c_ulong
    ctxs = []

    def flush():
        if not batched:
            return
        n = lib.lvlip_txq_len()
        if mode == "gpu":
            # created at the first flush, after the TCP sends: the HIP
            # runtime's start-up draws from rand(), which generate_iss
            # (src/tcp.c:153) must see unseeded as in the unbatched run
            if not ctxs:
                ctxs.append(lvlip.Context(0))
            rc = lib.lvlip_txq_fill_gpu(ctxs[0]._h)
            if rc != n:
                raise SystemExit(f"lvlip_txq_fill_gpu: {rc} (queue {n})")
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
    payload = bytes(((7 * i + 3) & 0xFF) for i in range(2001))
    lib.tcp_send(sk, payload, len(payload))
    lib.tcp_send_next(sk, 5)
    lib.tcp_send_ack(sk)
    lib.tcp_send_reset(sk)
    flush()
    # echo requests -> icmpv4_reply
    for req in requests:
        lib.ip_rcv(make_golden._frame_to_skb(lib, req))
    flush()
    os.write(0, END)
    th.join(timeout=30)
    if th.is_alive():
        raise SystemExit("reader did not see the end marker")
    for c in ctxs:
        c.close()
    with open(out_path, "w") as f:
        json.dump({"frames": got, "batches": batches, "deferred": deferred}, f)


if __name__ == "__main__":
    main(*sys.argv[1:5])
