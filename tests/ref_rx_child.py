"""Child process for tests/test_skb_gpu.py::test_rx_verify_agrees_with_reference_ip_rcv:
feeds frames to level-ip's own ip_rcv (src/ip_input.c:17-66, compiled from the
reference by oracle/Makefile) one at a time, and records for each whether the
stack answered.

    python tests/ref_rx_child.py FRAMES.json OUT.json path/to/libref.so

FRAMES.json holds hex Ethernet/IPv4 frames carrying ICMPv4 echo requests from
the tap (10.0.0.5) to the stack (10.0.0.4).  ip_rcv either drops a frame
(version, ihl, ttl, header checksum at src/ip_input.c:38, unknown protocol) or
hands it to icmpv4_incoming, which answers an echo request through
icmpv4_reply -> ip_output -> tun_write (src/icmpv4.c:31-54).  The stack's tun
fd is a zeroed static (src/tuntap_if.c:5), so fd 0 is made one end of a
socketpair and a reply shows up on the other end before ip_rcv returns.
OUT.json: per frame, the reply's hex or null."""
import ctypes
import json
import os
import socket
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden  # noqa: E402  (SkBuff, _frame_to_skb: test infrastructure)


def main(frames_path: str, out_path: str, so_path: str):
    with open(frames_path) as f:
        frames = [bytes.fromhex(h) for h in json.load(f)]
    lib = ctypes.CDLL(so_path)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    os.dup2(a.fileno(), 0)
    lib.netdev_init()
    lib.route_init()
    lib.arp_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    lib.ip_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    tap_mac = bytes.fromhex("0a1b2c3d4e5f")
    tap_ip, stack_ip = (10, 0, 0, 5), (10, 0, 0, 4)
    arp = (b"\xff" * 6 + tap_mac + b"\x08\x06" +
           struct.pack("!HHBBH", 1, 0x0800, 6, 4, 1) + tap_mac + bytes(tap_ip) + bytes(6) + bytes(stack_ip))
    lib.arp_rcv(make_golden._frame_to_skb(lib, arp))
    b.recv(2048)  # the ARP reply
    b.setblocking(False)
    replies = []
    for fr in frames:
        lib.ip_rcv(make_golden._frame_to_skb(lib, fr))
        try:
            replies.append(b.recv(4096).hex())
        except BlockingIOError:
            replies.append(None)
    with open(out_path, "w") as f:
        json.dump(replies, f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
