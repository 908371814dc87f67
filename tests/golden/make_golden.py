#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Runs only in the build container, where /root/reference exists: it loads
oracle/_ref/libref.so (level-ip's own src/*.c compiled by oracle/Makefile) and
records inputs + the reference's outputs as data files.  The tests then check
the oracle and the GPU path against these files with no reference present.

  kat.json     SURVEY.md §8c known-answer tests, re-computed by the reference
  vectors.npz  seeded random + adversarial checksum() cases (any offset/len/seed)
  tcp.npz      tcp_udp_checksum() cases (src/tcp.c:87-98), incl. the lost carry
  iphdr.npz    ip_send_check() cases (src/ip_output.c:8-12), ihl 5..15
  echo.json    config #1: ICMPv4 echo request -> reply frames produced by the
               reference stack (ip_rcv -> icmpv4_reply -> ip_output ->
               netdev_transmit -> tun_write) through an in-memory fake TAP
               (a socketpair dup'ed onto the stack's tun fd)
  tcp_frames.json  TCP frames the reference stack transmits (SYN with options,
               retransmit, 536/536/536/393-B data segments, ACK, RST) through
               the same fake TAP (tests/ref_stack_child.py on libref.so)

usage: python tests/golden/make_golden.py   (from the repo root)
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "level-ip_amd"))

import pyoracle  # noqa: E402
import workloads  # noqa: E402


def ref():
    lib = pyoracle.reflib()
    if lib is None:
        raise SystemExit("oracle/_ref/libref.so missing: run `make -C oracle` with /root/reference present")
    return lib


def i32(x):
    return ctypes.c_int(ctypes.c_uint32(x & 0xFFFFFFFF).value).value


def rcsum(lib, data: bytes, count: int, start: int) -> int:
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    return int(lib.checksum(buf, count, i32(start)))


def htonl_ip(a, b, c, d):
    # network-order u32 as the stack passes it (htonl(sk->saddr), src/tcp_output.c:126)
    return struct.unpack("<I", bytes([a, b, c, d]))[0]


# --------------------------------------------------------------------- KATs --

def make_kats(lib):
    ramp = lambda n: bytes(((7 * i + 3) & 0xFF) for i in range(n))  # noqa: E731
    iphdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    iphdr_filled = iphdr[:10] + bytes.fromhex("b861") + iphdr[12:]
    cases = [
        # name, data, count, start, survey value or None
        ("empty", b"", 0, 0, 0xFFFF),
        ("zeros20", bytes(20), 20, 0, 0xFFFF),
        ("odd3", bytes([0x12, 0x34, 0x56]), 3, 0, 0xCB97),
        ("rfc1071_s3", bytes.fromhex("0001f203f4f5f6f7"), 8, 0, 0x0D22),
        ("ipv4_hdr", iphdr, 20, 0, 0x61B8),
        ("ipv4_hdr_verify", iphdr_filled, 20, 0, 0x0000),
        ("ff1500", b"\xff" * 1500, 1500, 0, 0x0000),
        ("ff9000_seed", b"\xff" * 9000, 9000, 0x0A000014, 0xF5EB),
        ("ff9000_wrap", b"\xff" * 9000, 9000, 0xFFFFFF00, 0x0100),
        ("ramp1501", ramp(1501), 1501, 0, 0xE15F),
        ("ramp1500", ramp(1500), 1500, 0, 0xE166),
        ("neg_count", b"\x01\x02", -5, 0, None),
        ("one_byte", b"\xab", 1, 0, None),
        ("ramp65535", ramp(65535), 65535, 0, None),
        ("ramp65535_odd_seed", ramp(65535), 65535, 0xFFFFFFFF, None),
    ]
    out = []
    for name, data, count, start, survey in cases:
        v = rcsum(lib, data, count, start)
        if survey is not None and v != survey:
            raise SystemExit(f"reference disagrees with SURVEY KAT {name}: {v:#06x} != {survey:#06x}")
        out.append({"name": name, "data_hex": data.hex() if len(data) <= 64 else None,
                    "data_gen": None if len(data) <= 64 else _gen_desc(name), "count": count,
                    "start_sum": start & 0xFFFFFFFF, "expected": v})
    tcp = []
    for name, s, d, survey in [("tcp_10.0.0.4_to_5", (10, 0, 0, 4), (10, 0, 0, 5), 0xDCEB),
                               ("tcp_carry_lost", (10, 0, 0, 200), (10, 0, 0, 100), 0xB9EB)]:
        data = ctypes.create_string_buffer(20)
        v = int(lib.tcp_udp_checksum(htonl_ip(*s), htonl_ip(*d), 6, data, 20)) & 0xFFFF
        if v != survey:
            raise SystemExit(f"reference disagrees with SURVEY KAT {name}")
        tcp.append({"name": name, "saddr": htonl_ip(*s), "daddr": htonl_ip(*d), "proto": 6,
                    "data_hex": bytes(20).hex(), "len": 20, "expected": v})
    return {"source": "level-ip src/utils.c:22-55, src/tcp.c:87-98 compiled by oracle/Makefile",
            "checksum": out, "tcp_udp_checksum": tcp}


def _gen_desc(name):
    if name.startswith("ff"):
        return {"kind": "fill", "byte": 255, "n": int(name[2:].split("_")[0])}
    if name.startswith("ramp"):
        return {"kind": "ramp", "mul": 7, "add": 3, "n": int(name[4:].split("_")[0])}
    raise ValueError(name)


# ------------------------------------------------------------ random vectors --

def make_vectors(lib, rng):
    """checksum() over a 1 MiB seeded blob at many offsets, lengths and seeds."""
    blob = workloads.fill_bytes(1 << 20, seed=0xC0FFEE)
    # adversarial regions: runs of 0x00 and 0xff
    blob[1000:11000] = 0
    blob[20000:90000] = 0xFF
    cases = []
    lens = (list(range(0, 70)) + [127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 1459, 1460,
                                  1499, 1500, 1501, 2047, 2048, 4096, 8999, 9000, 9001,
                                  16383, 65534, 65535, 65536, 131069, 131070, 131071, 200001])
    for ln in lens:
        for _ in range(6):
            off = int(rng.integers(0, blob.size - ln)) if ln < blob.size else 0
            start = int(rng.choice([0, int(rng.integers(0, 2**32)), 0xFFFFFFFF, 0xFFFF0000,
                                    int(rng.integers(2**32 - 2**20, 2**32))]))
            cases.append((off, ln, start))
    # every byte alignment x tail parity, long and short
    for off_mod in range(16):
        for ln in (1, 2, 3, 15, 16, 17, 31, 33, 1000, 1001):
            off = 4096 * int(rng.integers(1, 200)) + off_mod
            cases.append((off, ln, int(rng.integers(0, 2**32))))
    # adversarial blocks, including the ones that wrap T = start + W
    for (off, ln) in [(1000, 10000), (20000, 70000), (20000, 1500), (20001, 9000), (1000, 1)]:
        for start in (0, 1, 0xFFFF, 0x10000, 0xFFFFFFFF, 0xFFFFFF00, 0x80000000):
            cases.append((off, ln, start))
    # ragged random
    for _ in range(2000):
        ln = int(rng.integers(0, 3000))
        off = int(rng.integers(0, blob.size - ln))
        cases.append((off, ln, int(rng.integers(0, 2**32))))
    off = np.array([c[0] for c in cases], dtype=np.uint64)
    ln = np.array([c[1] for c in cases], dtype=np.int32)
    st = np.array([c[2] for c in cases], dtype=np.uint32)
    exp = np.empty(len(cases), dtype=np.uint16)
    base = (ctypes.c_uint8 * blob.size).from_buffer(blob)
    addr = ctypes.addressof(base)
    for i in range(len(cases)):
        exp[i] = lib.checksum(ctypes.c_void_p(addr + int(off[i])), int(ln[i]), i32(int(st[i])))
    # negative counts are legal in the reference (utils.c:27,34): append a few
    neg = np.array([-1, -2, -100, -(2**31)], dtype=np.int32)
    for n_ in neg:
        off = np.append(off, np.uint64(12345))
        ln = np.append(ln, n_)
        st = np.append(st, np.uint32(0x1234))
        exp = np.append(exp, np.uint16(lib.checksum(ctypes.c_void_p(addr + 12345), int(n_), 0x1234)))
    return dict(blob=blob, offset=off, len=ln, start_sum=st, expected=exp)


def make_tcp(lib, rng):
    n = 600
    blob = workloads.fill_bytes(1 << 17, seed=0xBEEF)
    saddr = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    daddr = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    saddr[:50] = 0xFFFFFFFF  # force the lost carry
    daddr[:50] = rng.integers(1, 2**32, 50, dtype=np.uint64).astype(np.uint32)
    proto = np.where(rng.random(n) < 0.8, 6, 17).astype(np.uint8)
    ln = rng.integers(0, 65536, n).astype(np.uint32)
    ln[:200] = rng.integers(20, 1501, 200)
    off = np.array([int(rng.integers(0, blob.size - int(x))) if x < blob.size else 0 for x in ln],
                   dtype=np.uint64)
    ln = np.minimum(ln, blob.size - off).astype(np.uint32)
    exp = np.empty(n, dtype=np.uint16)
    base = (ctypes.c_uint8 * blob.size).from_buffer(blob)
    addr = ctypes.addressof(base)
    for i in range(n):
        exp[i] = int(lib.tcp_udp_checksum(int(saddr[i]), int(daddr[i]), int(proto[i]),
                                          ctypes.c_void_p(addr + int(off[i])), int(ln[i]))) & 0xFFFF
    return dict(blob=blob, saddr=saddr, daddr=daddr, proto=proto, offset=off, len=ln, expected=exp)


def make_iphdr(lib, rng):
    n = 300
    hdrs = np.zeros((n, 60), dtype=np.uint8)
    after = np.zeros((n, 60), dtype=np.uint8)
    for i in range(n):
        ihl = 5 if i < 200 else int(rng.integers(5, 16))
        h = bytearray(rng.integers(0, 256, 60, dtype=np.uint8).tobytes())
        h[0] = 0x40 | ihl
        if i % 3 == 0:
            h[10:12] = b"\x00\x00"  # ip_output zeroes csum first (src/ip_output.c:42)
        buf = ctypes.create_string_buffer(bytes(h), 60)
        lib.ip_send_check(buf)
        hdrs[i] = np.frombuffer(bytes(h), dtype=np.uint8)
        after[i] = np.frombuffer(buf.raw, dtype=np.uint8)
    return dict(hdr=hdrs, after=after)


# ------------------------------------------------------- config #1 (echo) --

class SkBuff(ctypes.Structure):
    # mirror of struct sk_buff (include/skbuff.h:9-23) on x86-64
    _fields_ = [("next", ctypes.c_void_p), ("prev", ctypes.c_void_p), ("rt", ctypes.c_void_p),
                ("dev", ctypes.c_void_p), ("refcnt", ctypes.c_int), ("protocol", ctypes.c_uint16),
                ("len", ctypes.c_uint32), ("dlen", ctypes.c_uint32), ("seq", ctypes.c_uint32),
                ("end_seq", ctypes.c_uint32), ("end", ctypes.c_void_p), ("head", ctypes.c_void_p),
                ("data", ctypes.c_void_p), ("payload", ctypes.c_void_p)]


def _frame_to_skb(lib, frame: bytes):
    lib.alloc_skb.restype = ctypes.POINTER(SkBuff)
    lib.alloc_skb.argtypes = [ctypes.c_uint]
    skb = lib.alloc_skb(1600)  # BUFLEN, include/netdev.h:8 (netdev_rx_loop, src/netdev.c:89)
    ctypes.memmove(skb.contents.data, frame, len(frame))
    return skb


def _ip_hdr(src, dst, proto, payload_len, ident):
    h = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + payload_len, ident, 0x4000, 64, proto,
                              0, bytes(src), bytes(dst)))
    c = pyoracle.checksum(bytes(h), 20, 0)
    h[10:12] = c.to_bytes(2, "little")
    return bytes(h)


def echo_child(out_path: str, so_path: str = pyoracle.REF_SO):
    """Runs in a subprocess: fd 0 becomes one end of a socketpair (the stack's
    tun fd is a zero-initialised static, src/tuntap_if.c:5, so tun_write writes
    to fd 0, src/tuntap_if.c:68-71).  `so_path` is the reference stack to drive:
    libref.so for the fixtures, libref_dropin.so (the same objects on the
    product library's checksum) for tests/test_ref_stack_dropin.py."""
    lib = ctypes.CDLL(so_path)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    os.dup2(a.fileno(), 0)
    lib.netdev_init()           # 10.0.0.4 / 00:0c:29:6d:50:25 (src/netdev.c:34-38)
    lib.route_init()            # src/route.c:39-44
    lib.arp_rcv.argtypes = [ctypes.POINTER(SkBuff)]
    lib.ip_rcv.argtypes = [ctypes.POINTER(SkBuff)]
    tap_mac = bytes.fromhex("0a1b2c3d4e5f")
    stack_mac = bytes.fromhex("000c296d5025")
    tap_ip, stack_ip = (10, 0, 0, 5), (10, 0, 0, 4)
    # ARP request tap -> stack, so the stack learns the tap's MAC (src/arp.c:74-128)
    arp = (b"\xff" * 6 + tap_mac + b"\x08\x06" +
           struct.pack("!HHBBH", 1, 0x0800, 6, 4, 1) + tap_mac + bytes(tap_ip) + bytes(6) + bytes(stack_ip))
    lib.arp_rcv(_frame_to_skb(lib, arp))
    arp_reply = b.recv(2048)
    results = {"arp_reply_hex": arp_reply.hex(), "echo": []}
    for data_len, ident, seq in [(56, 0x1234, 1), (64, 0x4321, 2), (57, 0x0101, 3), (1472, 0x7777, 4)]:
        payload = bytes(((i * 31 + seq) & 0xFF) for i in range(data_len))
        icmp = bytearray(struct.pack("!BBHHH", 8, 0, 0, ident, seq) + payload)
        c = pyoracle.checksum(bytes(icmp), len(icmp), 0)
        icmp[2:4] = c.to_bytes(2, "little")
        iph = _ip_hdr(tap_ip, stack_ip, 1, len(icmp), 0x1000 + seq)
        frame = stack_mac + tap_mac + b"\x08\x00" + iph + bytes(icmp)
        lib.ip_rcv(_frame_to_skb(lib, frame))
        reply = b.recv(4096)
        results["echo"].append({"data_len": data_len, "request_hex": frame.hex(),
                                "reply_hex": reply.hex()})
    with open(out_path, "w") as f:
        json.dump(results, f, indent=1)


def main():
    lib = ref()
    rng = np.random.default_rng(0x1E7E1C5)
    kats = make_kats(lib)
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump(kats, f, indent=1)
    np.savez_compressed(os.path.join(OUT, "vectors.npz"), **make_vectors(lib, rng))
    np.savez_compressed(os.path.join(OUT, "tcp.npz"), **make_tcp(lib, rng))
    np.savez_compressed(os.path.join(OUT, "iphdr.npz"), **make_iphdr(lib, rng))
    subprocess.run([sys.executable, __file__, "--echo-child", os.path.join(OUT, "echo.json")],
                   check=True, stdin=subprocess.DEVNULL)
    subprocess.run([sys.executable, os.path.join(os.path.dirname(OUT), "ref_stack_child.py"),
                    os.path.join(OUT, "tcp_frames.json"), pyoracle.REF_SO],
                   check=True, stdin=subprocess.DEVNULL)
    for fn in sorted(os.listdir(OUT)):
        print(fn, os.path.getsize(os.path.join(OUT, fn)))


if __name__ == "__main__":
    if len(sys.argv) in (3, 4) and sys.argv[1] == "--echo-child":
        echo_child(*sys.argv[2:])
    else:
        main()
