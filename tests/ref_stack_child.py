"""Child process for tests/test_ref_stack_dropin.py: drives level-ip's own TCP
transmit path on a given build of the stack and writes every frame it sends.

    python tests/ref_stack_child.py OUT.json path/to/libref_dropin.so

fd 0 becomes one end of a socketpair, which the stack's tun fd (a zero static,
src/tuntap_if.c:5) writes to (src/tuntap_if.c:68-71).  After an ARP request
teaches the stack the peer's MAC (src/arp.c:74-128), a TCP sock is made the way
inet_create does it (sk_alloc + sock_init_data, src/inet.c:58-61) and:
  tcp_v4_connect   SYN with MSS/SACK/WS options       (src/tcp.c:156-168)
  tcp_send         2 001 B queued as 536-B segments    (src/tcp_output.c:445-478)
  tcp_send_next    SYN again + the 4 data segments     (src/tcp_output.c:198-225)
  tcp_send_ack     bare ACK                            (src/tcp_output.c:247-267)
  tcp_send_reset   RST                                 (src/tcp_output.c:480-498)
Every one goes through tcp_transmit_skb -> tcp_v4_checksum -> checksum()
(src/tcp_output.c:126, src/tcp.c:97) and ip_output -> ip_send_check
(src/ip_output.c:53).  Sequence numbers and the port are random (time-seeded,
src/tcp.c:138-154), so the parent checks the checksums rather than the bytes."""
import ctypes
import json
import os
import socket
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden  # noqa: E402  (SkBuff, _frame_to_skb: test infrastructure)


def main(out_path: str, so_path: str):
    lib = ctypes.CDLL(so_path)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    os.dup2(a.fileno(), 0)
    lib.netdev_init()
    lib.route_init()
    lib.arp_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    tap_mac = bytes.fromhex("0a1b2c3d4e5f")
    tap_ip, stack_ip = (10, 0, 0, 5), (10, 0, 0, 4)
    arp = (b"\xff" * 6 + tap_mac + b"\x08\x06" +
           struct.pack("!HHBBH", 1, 0x0800, 6, 4, 1) + tap_mac + bytes(tap_ip) + bytes(6) + bytes(stack_ip))
    lib.arp_rcv(make_golden._frame_to_skb(lib, arp))
    b.recv(2048)  # the ARP reply

    lib.sk_alloc.restype = ctypes.c_void_p
    lib.sk_alloc.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.sock_init_data.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for fn in ("tcp_v4_connect",):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
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

    frames = []
    b.settimeout(2.0)

    def drain(k):
        for _ in range(k):
            frames.append(b.recv(4096).hex())

    lib.tcp_v4_connect(sk, ctypes.addressof(addr_buf), 16, 0)
    drain(1)
    payload = bytes(((7 * i + 3) & 0xFF) for i in range(2001))
    lib.tcp_send(sk, payload, len(payload))  # queued: the SYN is in flight
    lib.tcp_send_next(sk, 5)
    drain(5)
    lib.tcp_send_ack(sk)
    drain(1)
    lib.tcp_send_reset(sk)
    drain(1)
    with open(out_path, "w") as f:
        json.dump({"frames": frames, "payload_hex": payload.hex()}, f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
