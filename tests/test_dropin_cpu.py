"""Group 1 of include/lvlip_csum.h — the per-call drop-in for src/utils.c:22-55 —
against the reference's outputs, plus BASELINE config #1 (ICMPv4 echo through
the reference stack with a fake TAP, CPU only)."""
import ctypes

import numpy as np
import pytest

import golden_io
import lvlip
import pyoracle


def test_kats():
    cases, tcp = golden_io.kats()
    for name, data, count, start, expected in cases:
        assert lvlip.checksum(data if data else b"\0", count, start) == expected, name
    for t in tcp:
        got = lvlip.tcp_udp_checksum(t["saddr"], t["daddr"], t["proto"],
                                     bytes.fromhex(t["data_hex"]), t["len"])
        assert got == t["expected"], t["name"]


def test_vectors():
    v = golden_io.vectors()
    blob = v["blob"]
    for off, ln, st, exp in zip(v["offset"], v["len"], v["start_sum"], v["expected"]):
        off, ln = int(off), int(ln)
        got = lvlip.checksum(blob[off:], ln, int(st))
        assert got == int(exp), (off, ln, int(st))


def test_sum_every_16bits_matches_definition():
    rng = np.random.default_rng(3)
    for ln in list(range(0, 40)) + [255, 256, 257, 4095, 65535, 262145, 1 << 20]:
        a = rng.integers(0, 256, max(ln, 1), dtype=np.uint8)
        words = a[: ln & ~1].view("<u2").astype(np.uint64).sum()
        if ln & 1:
            words += int(a[ln - 1])
        assert lvlip.sum_every_16bits(a, ln) == int(words) & 0xFFFFFFFF
    # a sum that overflows u32 (the reference wraps silently)
    big = np.full(70000 * 2 * 32, 0xFF, dtype=np.uint8)
    n = big.size
    assert lvlip.sum_every_16bits(big, n) == (0xFFFF * (n // 2)) & 0xFFFFFFFF


def test_tcp_vectors():
    t = golden_io.tcp()
    for i in range(t["len"].size):
        off, ln = int(t["offset"][i]), int(t["len"][i])
        got = lvlip.tcp_udp_checksum(int(t["saddr"][i]), int(t["daddr"][i]), int(t["proto"][i]),
                                     t["blob"][off:off + max(ln, 1)], ln)
        assert got == int(t["expected"][i]), i


def test_ip_send_check():
    h = golden_io.iphdr()
    for hdr, after in zip(h["hdr"], h["after"]):
        b = bytearray(hdr.tobytes())
        lvlip.ip_send_check(b)
        assert bytes(b) == after.tobytes()


def test_echo_config1_cpu():
    """Config #1: the reference stack's replies re-derived with the drop-in.

    For each request frame: the IPv4 header verifies to 0 (src/ip_input.c:38);
    the reply's ICMP checksum equals checksum(icmp with csum=0)
    (src/icmpv4.c:46-47) and its IPv4 header checksum equals ip_send_check's
    (src/ip_output.c:42,53) — both compared with the bytes the reference wrote."""
    e = golden_io.echo()
    assert len(e["echo"]) >= 2
    for case in e["echo"]:
        req = bytes.fromhex(case["request_hex"])
        rep = bytearray(bytes.fromhex(case["reply_hex"]))
        assert lvlip.checksum(req[14:34], 20, 0) == 0
        iplen = int.from_bytes(rep[16:18], "big")
        icmp = bytearray(rep[34:14 + iplen])
        want_icmp = int.from_bytes(icmp[2:4], "little")
        icmp[2:4] = b"\0\0"
        assert icmp[0] == 0  # echo reply
        assert lvlip.checksum(bytes(icmp), len(icmp), 0) == want_icmp
        hdr = bytearray(rep[14:34])
        want_ip = bytes(hdr[10:12])
        hdr[10:12] = b"\0\0"
        lvlip.ip_send_check(hdr)
        assert bytes(hdr[10:12]) == want_ip
        # and the full reply verifies
        assert lvlip.checksum(bytes(rep[14:34]), 20, 0) == 0
        assert lvlip.checksum(bytes(rep[34:14 + iplen]), iplen - 20, 0) == 0


class SkBuff(ctypes.Structure):
    # struct sk_buff, include/skbuff.h:9-23, LP64 (the layout tcp_v4_checksum reads)
    _fields_ = [("next", ctypes.c_void_p), ("prev", ctypes.c_void_p), ("rt", ctypes.c_void_p),
                ("dev", ctypes.c_void_p), ("refcnt", ctypes.c_int), ("protocol", ctypes.c_uint16),
                ("len", ctypes.c_uint32), ("dlen", ctypes.c_uint32), ("seq", ctypes.c_uint32),
                ("end_seq", ctypes.c_uint32), ("end", ctypes.c_void_p), ("head", ctypes.c_void_p),
                ("data", ctypes.c_void_p), ("payload", ctypes.c_void_p)]


def test_tcp_v4_checksum_skb():
    """The exported tcp_v4_checksum (src/tcp.c:100-103) reads skb->data/len at
    the reference's offsets: golden TCP vectors through an sk_buff, and (where
    oracle/_ref is built) the reference's own tcp_v4_checksum on the same skb."""
    assert ctypes.sizeof(SkBuff) == 88 and SkBuff.len.offset == 40 and SkBuff.data.offset == 72
    t = golden_io.tcp()
    ref = pyoracle.reflib()
    if ref is not None:
        ref.tcp_v4_checksum.restype = ctypes.c_int
        ref.tcp_v4_checksum.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    n = 0
    for i in range(t["len"].size):
        if int(t["proto"][i]) != 6:
            continue
        off, ln = int(t["offset"][i]), int(t["len"][i])
        seg = np.ascontiguousarray(t["blob"][off:off + max(ln, 1)])
        skb = SkBuff(len=ln, data=seg.ctypes.data, head=seg.ctypes.data, refcnt=1)
        s, d = int(t["saddr"][i]), int(t["daddr"][i])
        got = lvlip.lib().tcp_v4_checksum(ctypes.byref(skb), s, d)
        assert got == int(t["expected"][i]), i
        if ref is not None:
            assert ref.tcp_v4_checksum(ctypes.byref(skb), s, d) == got, i
        n += 1
    assert n > 100


def test_ip_send_check_symbol_matches_reference():
    h = golden_io.iphdr()
    ref = pyoracle.reflib()
    for hdr in h["hdr"][:50]:
        a = bytearray(hdr.tobytes())
        b = bytearray(a)
        lvlip.ip_send_check(a)
        if ref is not None:
            c = (ctypes.c_char * len(b)).from_buffer(b)
            ref.ip_send_check(ctypes.addressof(c))
            del c
            assert a == b


def _word_sum(a: np.ndarray, ln: int) -> int:
    w = int(a[: ln & ~1].view("<u2").astype(np.uint64).sum())
    if ln & 1:
        w += int(a[ln - 1])
    return w & 0xFFFFFFFF


def test_sum_every_alignment_and_length():
    """Every alignment 0-63 x lengths 0-300 and the config sizes (the SIMD loop,
    its scalar tail and the portable loop all see their edges)."""
    rng = np.random.default_rng(17)
    buf = rng.integers(0, 256, 1 << 15, dtype=np.uint8)
    for off in range(64):
        for ln in list(range(0, 301)) + [1499, 1500, 1501, 9000, 9001]:
            a = buf[off:off + ln]
            assert lvlip.sum_every_16bits(a if ln else b"\0", ln) == _word_sum(a, ln), (off, ln)


def _cpu_flags():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


@pytest.mark.parametrize("path", ["scalar", "avx2", "avx512"])
def test_each_sum_path(path):
    """LVLIP_CPU_SUM caps the per-call word sum at the portable loop, AVX2 or
    AVX-512 (masked-load tail); every path gives the same results at every
    length 0-299 and 16 alignments (subprocess: the choice is made once per
    process).  A path the CPU lacks is skipped."""
    import os
    import subprocess
    import sys

    need = {"scalar": set(), "avx2": {"avx2"}, "avx512": {"avx512f", "avx512bw"}}[path]
    if not need <= _cpu_flags():
        pytest.skip(f"CPU lacks {sorted(need)}")

    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, lvlip\n"
        "rng = np.random.default_rng(5); b = rng.integers(0, 256, 300000, dtype=np.uint8)\n"
        "for off in range(17):\n"
        "  for ln in list(range(0, 300)) + [1500, 9000, 262145, 299000]:\n"
        "    a = b[off:off + ln]\n"
        "    w = int(a[: ln & ~1].view('<u2').astype(np.uint64).sum()) + (int(a[-1]) if ln & 1 else 0)\n"
        "    assert lvlip.sum_every_16bits(a if ln else b'\\0', ln) == w & 0xFFFFFFFF, (off, ln)\n"
        "print('ok')\n" % os.path.dirname(lvlip.__file__))
    env = dict(os.environ, LVLIP_CPU_SUM=path)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr
