"""Echo-request frames with every ip_rcv drop reason, and what level-ip's own
RX path does with them (tests/ref_rx_child.py on oracle/_ref/libref.so).

Used by the CPU test that pins the RX oracle to the reference
(tests/test_ref_rx.py) and by the GPU test that pins the batch verdicts to it
(tests/test_skb_gpu.py).  Test infrastructure only."""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

import pyoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
STACK_MAC, TAP_MAC = bytes.fromhex("000c296d5025"), bytes.fromhex("0a1b2c3d4e5f")
TAP_IP, STACK_IP = bytes((10, 0, 0, 5)), bytes((10, 0, 0, 4))

# kind -> the ip_rcv decision it exercises (src/ip_input.c:17-60)
KINDS = ("ok", "ok_options", "ip_csum", "version", "ihl", "ttl0", "proto", "icmp_csum")


def _csum_into(b: bytearray, lo: int, n: int, field: int) -> None:
    b[field:field + 2] = b"\0\0"
    b[field:field + 2] = pyoracle.checksum(bytes(b[lo:lo + n]), n, 0).to_bytes(2, "little")


def echo_frame(kind: str, rng: np.random.Generator, seq: int) -> bytes:
    data_len = int(rng.integers(0, 1400))
    icmp = bytearray(struct.pack("!BBHHH", 8, 0, 0, 0x4000 + seq, seq) +
                     rng.integers(0, 256, data_len, dtype=np.uint8).tobytes())
    _csum_into(icmp, 0, len(icmp), 2)
    if kind == "icmp_csum":
        icmp[2] ^= 0x5A  # the reference never verifies ICMP on RX (src/icmpv4.c:11)
    ihl = int(rng.integers(6, 16)) if kind == "ok_options" else 5
    # options: level-ip's icmpv4_incoming reads the ICMP type at the fixed
    # iphdr->data (byte 20 of the header, src/icmpv4.c:9), i.e. the first option
    # byte; starting the options with 8 keeps the frame an "echo request" there,
    # so an accepted frame is still answered and the test can see it
    opts = bytes([8, 0] + [1] * ((ihl - 5) * 4 - 2)) if ihl > 5 else b""
    ih = bytearray(struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, 0, ihl * 4 + len(icmp), 0x1000 + seq,
                               0x4000, 64, 1, 0, TAP_IP, STACK_IP) + opts)
    if kind == "version":
        ih[0] = 0x60 | ihl
    elif kind == "ttl0":
        ih[8] = 0
    elif kind == "proto":
        ih[9] = 17
    _csum_into(ih, 0, ihl * 4, 10)  # a valid header checksum for what is there ...
    if kind == "ip_csum":
        ih[4] ^= 0x01  # ... except here
    elif kind == "ihl":
        ih[0] = 0x44  # ihl 4: dropped before the checksum is looked at
    return STACK_MAC + TAP_MAC + b"\x08\x00" + bytes(ih) + bytes(icmp)


def frames(seed: int, per_kind: int = 24):
    """(frames, kinds): per_kind frames of every kind, shuffled."""
    rng = np.random.default_rng(seed)
    ks = [k for k in KINDS for _ in range(per_kind)]
    rng.shuffle(ks)
    return [bytearray(echo_frame(k, rng, i)) for i, k in enumerate(ks)], ks


def reference_replies(frs, so_path: str = REF_SO):
    """Runs the frames through level-ip's ip_rcv in a child process; per frame
    the stack's reply (bytes) or None when it dropped the frame."""
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "frames.json"), os.path.join(d, "replies.json")
        with open(fin, "w") as f:
            json.dump([bytes(x).hex() for x in frs], f)
        subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_rx_child.py"), fin, fout,
                        so_path], check=True, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, timeout=120)
        with open(fout) as f:
            return [bytes.fromhex(h) if h is not None else None for h in json.load(f)]
