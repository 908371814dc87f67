"""The skb-queue entries of include/lvlip_skb.h (lvlip_rx_verify_skb_list,
lvlip_tx_checksum_skb_list) on level-ip's own sk_buff queues: the skbs are
allocated and shaped by the reference's own skbuff.c (alloc_skb, skb_reserve,
skb_push from oracle/_ref/libref.so, src/skbuff.c:5-43) and linked into an
sk_buff_head as skb_queue_tail does (include/skbuff.h:55-59); verdicts and
filled frames are compared with the oracle's restatement of ip_rcv's and the
TX path's decisions (oracle/skb_oracle.py)."""
import ctypes
import os
import sys

import numpy as np
import pytest

import lvlip
import ref_rx_cases
import skb_oracle
import workloads

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden  # noqa: E402  (SkBuff: struct sk_buff on LP64, test infrastructure)

BUFLEN = 1600  # include/netdev.h:8


class SkBuffHead(ctypes.Structure):
    # struct sk_buff_head (include/skbuff.h:25-29): list_head + qlen
    _fields_ = [("next", ctypes.c_void_p), ("prev", ctypes.c_void_p), ("qlen", ctypes.c_uint32)]


def _ref():
    if not os.path.exists(ref_rx_cases.REF_SO):
        pytest.skip("oracle/_ref/libref.so not built")
    lib = ctypes.CDLL(ref_rx_cases.REF_SO)
    lib.alloc_skb.restype = ctypes.POINTER(make_golden.SkBuff)
    lib.alloc_skb.argtypes = [ctypes.c_uint]
    lib.skb_reserve.restype = ctypes.c_void_p
    lib.skb_reserve.argtypes = [ctypes.POINTER(make_golden.SkBuff), ctypes.c_uint]
    lib.skb_push.restype = ctypes.c_void_p
    lib.skb_push.argtypes = [ctypes.POINTER(make_golden.SkBuff), ctypes.c_uint]
    lib.free_skb.argtypes = [ctypes.POINTER(make_golden.SkBuff)]
    return lib


class Queue:
    """An sk_buff_head with skb_queue_tail's linking (list_add_tail, include/list.h)."""

    def __init__(self):
        self.q = SkBuffHead()
        a = ctypes.addressof(self.q)
        self.q.next = self.q.prev = a
        self.skbs = []

    def tail(self, skb):
        node, head = ctypes.addressof(skb.contents), ctypes.addressof(self.q)
        last = self.q.prev
        s = skb.contents
        s.next, s.prev = head, last
        if last == head:
            self.q.next = node
        else:
            make_golden.SkBuff.from_address(last).next = node
        self.q.prev = node
        self.q.qlen += 1
        self.skbs.append(skb)

    def ptr(self):
        return ctypes.addressof(self.q)


def test_skb_list_arguments_without_gpu():
    L = lvlip.lib()
    q = Queue()
    v = np.zeros(4, np.uint8)
    assert L.lvlip_rx_verify_skb_list(None, q.ptr(), 0, v.ctypes.data, 4) == lvlip.EINVAL
    assert L.lvlip_tx_checksum_skb_list(None, q.ptr()) == lvlip.EINVAL
    assert L.lvlip_tx_checksum_skb_list(None, None) == lvlip.EINVAL


@pytest.mark.gpu
def test_rx_verify_skb_list_on_reference_skbs():
    """3 000 frames of every kind, each read into an skb as netdev_rx_loop does
    (alloc_skb(BUFLEN), the frame at skb->data, src/netdev.c:88-91): the
    verdicts, in list order, equal the oracle's on the skb's whole buffer; the
    queue is untouched; a short verdict array gets LVLIP_ERANGE."""
    ref = _ref()
    fr = workloads.frames(3000, seed=81, max_l4=1500)
    for f in fr[::2]:
        skb_oracle.tx_fill(f)
    rng = np.random.default_rng(82)
    for i in rng.choice(len(fr), 300, replace=False):
        f = fr[int(i)]
        f[14 + int(rng.integers(0, 40))] ^= 1 << int(rng.integers(0, 8))
    q = Queue()
    for f in fr:
        skb = ref.alloc_skb(BUFLEN)
        ctypes.memmove(skb.contents.data, bytes(f), len(f))
        q.tail(skb)
    before = [ctypes.string_at(s.contents.data, BUFLEN) for s in q.skbs]
    with lvlip.Context(0, arena_bytes=4 << 20) as ctx:
        for flags in (0, lvlip.RX_VERIFY_L4):
            v = np.zeros(len(fr), np.uint8)
            n = lvlip.lib().lvlip_rx_verify_skb_list(ctx._h, q.ptr(), flags, v.ctypes.data, len(fr))
            assert n == len(fr)
            want = [skb_oracle.rx_verdict(b, flags) for b in before]
            assert v.tolist() == want, flags
        v = np.zeros(10, np.uint8)
        assert lvlip.lib().lvlip_rx_verify_skb_list(ctx._h, q.ptr(), 0, v.ctypes.data, 10) == lvlip.ERANGE
        empty = Queue()
        assert lvlip.lib().lvlip_rx_verify_skb_list(ctx._h, empty.ptr(), 0, None, 0) == 0
    assert [ctypes.string_at(s.contents.data, BUFLEN) for s in q.skbs] == before
    assert len({w for w in want}) >= 3
    for s in q.skbs:
        ref.free_skb(s)


@pytest.mark.gpu
def test_tx_checksum_skb_list_on_reference_skbs():
    """2 000 TCP/ICMP segments built the way level-ip's TX path builds them
    (alloc_skb, skb_reserve to the end, skb_push of the segment and of the IPv4
    header, src/skbuff.c:31-43; 14 bytes of Ethernet header left in front for
    netdev_transmit): after lvlip_tx_checksum_skb_list every skb's IPv4 header
    and segment equal the oracle's fill (tcp_transmit_skb + ip_send_check,
    src/tcp_output.c:126, src/ip_output.c:53), and nothing else changed."""
    ref = _ref()
    fr = workloads.frames(2000, seed=83, max_l4=1460)
    q = Queue()
    for f in fr:
        body = bytes(f[14:])  # IPv4 header + segment (+ padding past ip.len)
        skb = ref.alloc_skb(14 + len(body) + 16)
        ref.skb_reserve(skb, 14 + len(body))
        ref.skb_push(skb, len(body))
        ctypes.memmove(skb.contents.data, body, len(body))
        q.tail(skb)
    want = [bytearray(f) for f in fr]
    for w in want:
        skb_oracle.tx_fill(w)
    with lvlip.Context(0, arena_bytes=4 << 20) as ctx:
        assert lvlip.lib().lvlip_tx_checksum_skb_list(ctx._h, q.ptr()) == len(fr)
    for s, w in zip(q.skbs, want):
        got = ctypes.string_at(s.contents.data, s.contents.len)
        assert got == bytes(w[14:])
    for s in q.skbs:
        ref.free_skb(s)
