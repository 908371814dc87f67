"""Property-based differential test of Group 1 (the per-call drop-in,
level-ip_amd/csrc/csum_cpu.c) against level-ip's own compiled functions
(oracle/_ref/libref.so: src/utils.c:22-55, src/tcp.c:87-98,
src/ip_output.c:8-12), on inputs hypothesis draws: any bytes at any alignment,
counts including 0 and negative ones (src/utils.c:27 loops `while (count > 1)`,
:34 adds the odd byte only `if (count > 0)`), any 32-bit `start_sum` pattern
(the reference's `int`), and any pseudo-header address and protocol.  CPU only; skipped where oracle/_ref was not
built (the GPU box keeps the prebuilt file, so it runs there too)."""
import ctypes

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import lvlip
import pyoracle

REF = pyoracle.reflib()
pytestmark = pytest.mark.skipif(REF is None, reason="oracle/_ref/libref.so not built")

# every call below runs both libraries on the same pointer (signatures: lvlip.SIGNATURES)
SETTINGS = settings(max_examples=600, deadline=None, suppress_health_check=[HealthCheck.too_slow])
_product = lvlip.lib()


def _buf(data: bytes, align: int):
    """data placed `align` bytes past a 64-B boundary (the drop-in's SIMD
    loops, their masked or scalar tails and the portable loop see every
    alignment)."""
    raw = np.zeros(len(data) + 128, np.uint8)
    base = (-raw.ctypes.data) % 64 + align
    raw[base:base + len(data)] = np.frombuffer(data, np.uint8)
    return raw, raw.ctypes.data + base


def _i32(u: int) -> int:
    return ctypes.c_int32(u & 0xFFFFFFFF).value


@SETTINGS
@given(data=st.binary(min_size=0, max_size=3000), align=st.integers(0, 63),
       cut=st.integers(-8, 3000), seed=st.integers(0, 0xFFFFFFFF))
def test_checksum_matches_reference(data, align, cut, seed):
    raw, p = _buf(data, align)
    count = min(cut, len(data))
    s = _i32(seed)
    assert _product.sum_every_16bits(p, count) == REF.sum_every_16bits(p, count)
    assert _product.checksum(p, count, s) == REF.checksum(p, count, s)
    del raw


@SETTINGS
@given(fill=st.sampled_from([0x00, 0xFF]), n=st.integers(0, 9001), align=st.integers(0, 63),
       seed=st.sampled_from([0, 1, 0xFFFF, 0x10000, 0x7FFFFFFF, 0x80000000, 0xFFFF0000, 0xFFFFFF00,
                             0xFFFFFFFF]))
def test_checksum_adversarial_fills(fill, n, align, seed):
    """All-0x00 / all-0xff packets with the seeds at the fold's and the u32
    wrap's edges (SURVEY.md §8c KATs generalised)."""
    raw, p = _buf(bytes([fill]) * n, align)
    s = _i32(seed)
    assert _product.checksum(p, n, s) == REF.checksum(p, n, s)
    del raw


@SETTINGS
@given(data=st.binary(min_size=0, max_size=2000), align=st.integers(0, 63),
       saddr=st.integers(0, 0xFFFFFFFF), daddr=st.integers(0, 0xFFFFFFFF),
       proto=st.integers(0, 255), cut=st.integers(0, 2000))
def test_tcp_udp_checksum_matches_reference(data, align, saddr, daddr, proto, cut):
    """The pseudo-header sum as whole u32 words with the carry lost
    (src/tcp.c:92-95), for any addresses, protocol and length."""
    raw, p = _buf(data, align)
    ln = min(cut, len(data))
    got = _product.tcp_udp_checksum(saddr, daddr, proto, p, ln)
    assert got == REF.tcp_udp_checksum(saddr, daddr, proto, p, ln)
    del raw


@SETTINGS
@given(hdr=st.binary(min_size=60, max_size=60), ihl=st.integers(5, 15), align=st.integers(0, 63))
def test_ip_send_check_matches_reference(hdr, ihl, align):
    """ip_send_check sums ihl*4 bytes with the field as it stands and stores
    the result raw at offset 10 (src/ip_output.c:8-12)."""
    b = bytearray(hdr)
    b[0] = 0x40 | ihl
    raw_a, pa = _buf(bytes(b), align)
    raw_b, pb = _buf(bytes(b), align)
    _product.ip_send_check(pa)
    REF.ip_send_check(pb)
    off = (-raw_a.ctypes.data) % 64 + align
    off_b = (-raw_b.ctypes.data) % 64 + align
    assert raw_a[off:off + 60].tobytes() == raw_b[off_b:off_b + 60].tobytes()
