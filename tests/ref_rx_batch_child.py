"""Child process: level-ip's RX path with and without the batch-and-dispatch step
(INTEGRATION.md §2b), on the reference stack itself
(oracle/_ref/libref.so, compiled from /root/reference by oracle/Makefile).

    python tests/ref_rx_batch_child.py FRAMES.json OUT.json libref.so MODE

FRAMES.json holds hex Ethernet frames arriving on the tap.  Every frame goes
into its own skb as netdev_rx_loop puts it there (alloc_skb(BUFLEN), then the
read into skb->data, src/netdev.c:86-101).  MODE:

  unbatched   level-ip as it is: each skb straight to netdev_receive's
              dispatch (src/netdev.c:63-84): ARP -> arp_rcv, IPv4 -> ip_rcv,
              anything else freed
  batched[:F] the optional batch-and-dispatch path: all skbs linked into one
              sk_buff_head as skb_queue_tail links them (include/skbuff.h:55-59),
              ONE lvlip_rx_verify_skb_list call on the GPU (flags F, default 0)
              over the queue, then per skb in list order: LVLIP_RX_OK -> ip_rcv,
              LVLIP_RX_NOT_IP -> netdev_receive's other branches (ARP ->
              arp_rcv), anything else -> free_skb (ip_rcv's drop_pkt)
  oracle[:F]  the same composition with the verdicts from the CPU oracle
              (oracle/skb_oracle.py) instead of the GPU: the harness's own
              check on a machine without one

The stack's tun fd is a zeroed static (src/tuntap_if.c:5), so fd 0 is made one
end of a socketpair and whatever the stack transmits shows up on the other end.
OUT.json: {"replies": per frame the bytes the stack wrote in response (hex,
several frames joined by "|"), or null; "verdicts": the batch's verdicts (null
for unbatched)}.

On oracle/_ref/libref_rxq.so (ip_rcv's header checksum at src/ip_input.c:38
gated on the batch verdict, oracle/ref_rxq.c) the batched modes mark every
accepted skb's IPv4 header before ip_rcv, so :38 takes the batch's result
instead of summing it again; OUT.json then also holds "cpu_header_sums" (the
header sums ip_rcv ran on the CPU) and "batch_header_sums" (the ones the
batch answered).
"""
import ctypes
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(HERE, "golden"), HERE, os.path.join(ROOT, "level-ip_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import make_golden  # noqa: E402  (SkBuff: struct sk_buff on LP64)
from test_skb_list import Queue  # noqa: E402  (skb_queue_tail's linking)

BUFLEN = 1600  # include/netdev.h:8
ETH_P_ARP, ETH_P_IP = 0x0806, 0x0800


def main(frames_path: str, out_path: str, so_path: str, mode: str):
    with open(frames_path) as f:
        frames = [bytes.fromhex(h) for h in json.load(f)]
    lib = ctypes.CDLL(so_path)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    os.dup2(a.fileno(), 0)
    lib.netdev_init()
    lib.route_init()
    lib.alloc_skb.restype = ctypes.POINTER(make_golden.SkBuff)
    lib.alloc_skb.argtypes = [ctypes.c_uint]
    lib.free_skb.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    lib.arp_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    lib.ip_rcv.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    b.setblocking(False)

    def sent():
        out = []
        while True:
            try:
                out.append(b.recv(4096).hex())
            except BlockingIOError:
                return "|".join(out) if out else None

    def netdev_receive(skb, frame):  # src/netdev.c:63-84
        et = int.from_bytes(frame[12:14], "big")
        if et == ETH_P_ARP:
            lib.arp_rcv(skb)
        elif et == ETH_P_IP:
            lib.ip_rcv(skb)
        else:
            lib.free_skb(skb)

    skbs = []
    for fr in frames:  # netdev_rx_loop: alloc_skb(BUFLEN), tun_read into skb->data
        skb = lib.alloc_skb(BUFLEN)
        ctypes.memmove(skb.contents.data, fr, len(fr))
        skbs.append(skb)
    replies, verdicts = [], None
    gated = hasattr(lib, "lvlip_rxq_accept")
    if gated:
        lib.lvlip_rxq_accept.argtypes = [ctypes.c_void_p]
        lib.lvlip_rxq_computed.restype = ctypes.c_ulong
        lib.lvlip_rxq_skipped.restype = ctypes.c_ulong
    if mode == "unbatched":
        for skb, fr in zip(skbs, frames):
            netdev_receive(skb, fr)
            replies.append(sent())
    else:
        kind, _, fl = mode.partition(":")
        flags = int(fl or "0", 0)
        q = Queue()
        for skb in skbs:
            q.tail(skb)
        if kind == "batched":
            import numpy as np

            import lvlip
            v = np.zeros(len(skbs), np.uint8)
            with lvlip.Context(0) as ctx:
                m = lvlip.lib().lvlip_rx_verify_skb_list(ctx._h, q.ptr(), flags, v.ctypes.data, len(skbs))
            if m != len(skbs):
                raise SystemExit(f"lvlip_rx_verify_skb_list returned {m}")
            verdicts = [int(x) for x in v]
        elif kind == "oracle":
            import skb_oracle
            # the frame the list walker hands over: skb->data .. skb->end
            verdicts = [skb_oracle.rx_verdict(ctypes.string_at(s.contents.data, BUFLEN), flags) for s in skbs]
        else:
            raise SystemExit(f"unknown mode {mode}")
        import lvlip  # noqa: F811 (constants only on the oracle path)
        for skb, fr, vd in zip(skbs, frames, verdicts):
            if vd == lvlip.RX_OK:
                if gated:  # ip_hdr(skb) = skb->head + ETH_HDR_LEN (include/ip.h:47-50)
                    assert lib.lvlip_rxq_accept(skb.contents.head + 14) == 0
                # the checks are taken; ip_rcv repeats them (same outcome), and
                # on libref_rxq.so skips the header sum (:38) the batch made
                lib.ip_rcv(skb)
            elif vd == lvlip.RX_NOT_IP:
                netdev_receive(skb, fr)
            else:
                lib.free_skb(skb)  # ip_rcv's drop_pkt
            replies.append(sent())
    out = {"replies": replies, "verdicts": verdicts}
    if gated:
        out["cpu_header_sums"] = int(lib.lvlip_rxq_computed())
        out["batch_header_sums"] = int(lib.lvlip_rxq_skipped())
    with open(out_path, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main(*sys.argv[1:5])
