"""f1/f2 frame batches (include/lvlip_skb.h), host side: the plan and apply steps
that lvlip_rx_verify / lvlip_tx_checksum wrap around their one GPU batch.

The batch in the middle is replaced here by the oracle over exactly the
(ptr, len, start_sum) entries the plan produced, so these tests check which
bytes are summed with which seed and how results land; the GPU tests
(test_skb_gpu.py) run the same frames through the real batch.  Expected
values come from oracle/skb_oracle.py (ip_rcv / TX restatement over the
pinned checksum oracle) and, for config #1, from the reference stack's own
echo replies (tests/golden/echo.json)."""
import ctypes
import struct

import numpy as np

import golden_io
import lvlip
import pyoracle
import skb_oracle
import workloads


def oracle_batch(entries):
    out = np.empty(len(entries), dtype=np.uint16)
    for k, (ptr, ln, st) in enumerate(entries):
        data = ctypes.string_at(ptr, ln) if ln else b""
        out[k] = pyoracle.checksum(data if data else b"\0", ln, st)
    return out


def tx_via_plan(frames):
    plan = lvlip.tx_plan(frames)
    assert plan is not None
    entries, field = plan
    lvlip.tx_apply(field, oracle_batch(entries))


def rx_via_plan(frames, flags):
    verdict, entries, tag = lvlip.rx_plan(frames, flags)
    return lvlip.rx_apply(verdict, tag, oracle_batch(entries))


def test_pseudo_sum_rfc():
    rng = np.random.default_rng(5)
    for _ in range(2000):
        s, d = (int(x) for x in rng.integers(0, 1 << 32, 2, dtype=np.uint64))
        p, ln = int(rng.integers(0, 256)), int(rng.integers(0, 1 << 16))
        assert lvlip.pseudo_sum_rfc(s, d, p, ln) == skb_oracle.pseudo_sum_rfc(s, d, p, ln)
    # where the reference's u32 seed loses a carry the two differ by exactly that
    s = d = 0xFFFF_FFFF
    assert lvlip.pseudo_sum(s, d, 6, 40) != lvlip.pseudo_sum_rfc(s, d, 6, 40)


def test_tx_plan_matches_reference_tx():
    fr = workloads.frames(400, seed=11)
    before = [bytes(f) for f in fr]
    plan = lvlip.tx_plan(fr)
    assert [bytes(f) for f in fr] == before  # the plan does not write frames
    assert len(plan[0]) == 2 * len(fr)
    want = [bytearray(f) for f in before]
    for f in want:
        skb_oracle.tx_fill(f)
    tx_via_plan(fr)
    for i, (a, b) in enumerate(zip(fr, want)):
        assert bytes(a) == bytes(b), i


def test_tx_fields_any_prior_value():
    """The seed compensation is exact whatever the field held (incl. 0 and 0xffff)."""
    base = workloads.frames(8, seed=12, max_l4=300)
    for v in (b"\0\0", b"\xff\xff", b"\x00\xff", b"\x12\x34"):
        fr = [bytearray(f) for f in base]
        for f in fr:
            ihl = f[14] & 0xF
            f[24:26] = v
            off = 14 + ihl * 4 + (16 if f[23] == 6 else 2)
            f[off:off + 2] = v
        want = [bytearray(f) for f in fr]
        for f in want:
            skb_oracle.tx_fill(f)
        tx_via_plan(fr)
        assert [bytes(f) for f in fr] == [bytes(f) for f in want]


def test_tx_echo_reply_golden():
    """Config #1 TX: the reference stack's echo replies, checksum fields
    scrambled, refilled by plan/apply == the bytes the reference wrote."""
    e = golden_io.echo()["echo"]
    fr = []
    for case in e:
        rep = bytearray(bytes.fromhex(case["reply_hex"]))
        rep[24:26] = b"\xde\xad"
        rep[36:38] = b"\xbe\xef"
        fr.append(rep)
    tx_via_plan(fr)
    for f, case in zip(fr, e):
        assert bytes(f) == bytes.fromhex(case["reply_hex"])


def _scrambled_tcp_frames():
    want = golden_io.tcp_frames()
    fr = []
    for k, w in enumerate(want):
        f = bytearray(w)
        f[24:26] = (b"\0\0", b"\xff\xff", b"\xde\xad")[k % 3]
        f[34 + 16:34 + 18] = (b"\xff\xff", b"\0\0", b"\xbe\xef")[k % 3]
        fr.append(f)
    return fr, want


def test_tx_tcp_stack_frames_golden():
    """f2 on the frames level-ip's own TCP transmit path wrote
    (tests/golden/tcp_frames.json: SYN with MSS/SACK/WS options, data segments
    of 536/536/536/393 B, ACK, RST): fields scrambled, refilled by plan/apply ==
    the reference's bytes; and RX verify (header + L4) accepts them."""
    fr, want = _scrambled_tcp_frames()
    tx_via_plan(fr)
    assert [bytes(f) for f in fr] == want
    for flags in (0, lvlip.RX_VERIFY_L4):
        assert rx_via_plan(fr, flags).tolist() == [lvlip.RX_OK] * len(fr)


def test_tx_tcp_golden_segments():
    """TCP TX over the segments of tests/golden/tcp.npz (reference
    tcp_udp_checksum outputs): with the field restored to the value the golden
    checksum was computed over, the compensated seed reproduces it."""
    t = golden_io.tcp()
    n = 0
    for i in range(t["len"].size):
        ln = int(t["len"][i])
        if int(t["proto"][i]) != 6 or ln < 20 or ln > 65535 - 20:
            continue
        off = int(t["offset"][i])
        seg = bytearray(t["blob"][off:off + ln].tobytes())
        f = bytearray(14) + bytearray(20) + seg
        f[12:14] = b"\x08\x00"
        f[14], f[22], f[23] = 0x45, 64, 6
        f[16:18] = (20 + ln).to_bytes(2, "big")
        f[26:34] = struct.pack("<II", int(t["saddr"][i]), int(t["daddr"][i]))
        # golden = checksum(seg, ln, seed) with seg's own field value g; the
        # plan computes checksum(seg with field 0, seed).  Find that via the
        # oracle and compare; then check the golden one through start_sum.
        entries, field = lvlip.tx_plan([f])
        ptr, l4len, st = entries[0]
        assert l4len == ln and ctypes.string_at(ptr, ln) == bytes(seg)
        g = struct.unpack_from("<H", seg, 16)[0]
        assert pyoracle.checksum(bytes(seg), ln, (st + g) & 0xFFFFFFFF) == int(t["expected"][i])
        n += 1
    assert n > 100


def test_tx_malformed_refused():
    good = workloads.frames(3, seed=13, max_l4=100)
    bad = [bytearray(f) for f in good]
    bad[1][14] = 0x65  # version 6
    assert lvlip.tx_plan(bad) is None
    short = [bytearray(f) for f in good]
    short[2] = short[2][:30]
    assert lvlip.tx_plan(short) is None
    trunc = [bytearray(f) for f in good]
    iplen = int.from_bytes(trunc[0][16:18], "big")
    trunc[0] = trunc[0][:14 + iplen - 1]
    assert lvlip.tx_plan(trunc) is None
    assert lvlip.tx_plan(good) is not None


def _rx_cases(seed):
    rng = np.random.default_rng(seed)
    base = workloads.frames(60, seed=seed, max_l4=700, protos=(6, 1))
    for f in base:
        skb_oracle.tx_fill(f)  # valid header checksum; L4 valid unless the seed lost a carry
    cases = []
    for f in base:
        cases.append(bytearray(f))
        g = bytearray(f)
        kind = int(rng.integers(0, 11))
        ihl = g[14] & 0xF
        if kind == 0:
            g[14] = 0x60 | ihl
        elif kind == 1:
            g[14] = 0x40 | int(rng.integers(0, 5))
        elif kind == 2:
            g[22] = 0
        elif kind == 3:
            g[14 + int(rng.integers(0, ihl * 4))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 4:
            j = 14 + ihl * 4 + int(rng.integers(0, len(g) - 14 - ihl * 4))
            g[j] ^= 0x40
        elif kind == 5:
            g[12:14] = b"\x08\x06"
        elif kind == 6:
            g = g[: int(rng.integers(0, 34))]
        elif kind == 7:
            g = g[: 14 + ihl * 4 - 1] if ihl > 5 else g[:33]
        elif kind == 8:
            iplen = int.from_bytes(g[16:18], "big")
            g = g[: 14 + iplen - 1]
        elif kind == 9:
            g[23] = 17  # UDP: not handled by ip_rcv; header checksum refilled
            skb_oracle.tx_fill(g)
        else:
            g[23] = 17  # unknown proto AND a stale header checksum
        cases.append(g)
    return cases


def test_rx_plan_matches_ip_rcv():
    fr = _rx_cases(21)
    before = [bytes(f) for f in fr]
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = rx_via_plan(fr, flags)
        want = [skb_oracle.rx_verdict(f, flags) for f in fr]
        assert [bytes(f) for f in fr] == before
        assert got.tolist() == want, flags
    # every verdict kind is exercised
    seen = set(rx_via_plan(fr, lvlip.RX_VERIFY_L4).tolist()) | set(rx_via_plan(fr, 0).tolist())
    assert seen >= set(range(1, 10)), seen


def test_rx_echo_requests_ok():
    e = golden_io.echo()["echo"]
    fr = [bytearray(bytes.fromhex(c["request_hex"])) for c in e]
    for flags in (0, lvlip.RX_VERIFY_L4):
        assert rx_via_plan(fr, flags).tolist() == [lvlip.RX_OK] * len(fr)


def test_rx_rfc_tcp_verify():
    """A TCP segment whose checksum an RFC-correct peer filled verifies as OK
    even where the reference's own u32 seed would lose a carry."""
    fr = workloads.frames(40, seed=22, max_l4=400, protos=(6,))
    for f in fr:
        skb_oracle.tx_fill(f)
        f[26:34] = b"\xff" * 8  # saddr = daddr = 255.255.255.255: the u32 seed overflows
        ihl = f[14] & 0xF
        l4 = 14 + ihl * 4
        iplen = int.from_bytes(f[16:18], "big")
        f[l4 + 16:l4 + 18] = b"\0\0"
        seed = skb_oracle.pseudo_sum_rfc(0xFFFFFFFF, 0xFFFFFFFF, 6, iplen - ihl * 4)
        c = pyoracle.checksum(bytes(f[l4:14 + iplen]), iplen - ihl * 4, seed)
        f[l4 + 16:l4 + 18] = struct.pack("<H", c)
        f[24:26] = b"\0\0"
        f[24:26] = struct.pack("<H", pyoracle.checksum(bytes(f[14:14 + ihl * 4]), ihl * 4, 0))
    assert rx_via_plan(fr, lvlip.RX_VERIFY_L4).tolist() == [lvlip.RX_OK] * len(fr)


def test_empty_batches():
    v, entries, tag = lvlip.rx_plan([], 0)
    assert v.size == 0 and entries == [] and tag.size == 0
    entries, field = lvlip.tx_plan([])
    assert entries == [] and field.size == 0


# ------------------------------------------------------------ f4: RFC 1624 --

def _echo_request(payload: bytes, ident=0x1234, seq=1, alt_zero=False):
    """Ethernet + IPv4 + ICMP echo request with a valid ICMP checksum (oracle)."""
    icmp = bytearray(b"\x08\x00\x00\x00" + ident.to_bytes(2, "big") + seq.to_bytes(2, "big") + payload)
    c = pyoracle.checksum(bytes(icmp), len(icmp), 0)
    if alt_zero and c == 0:
        c = 0xFFFF  # the other one's-complement zero: verifies too
    icmp[2:4] = struct.pack("<H", c)
    f = bytearray(14) + bytearray(20) + icmp
    f[12:14] = b"\x08\x00"
    f[14], f[22], f[23] = 0x45, 64, 1
    f[16:18] = (20 + len(icmp)).to_bytes(2, "big")
    skb_oracle.tx_fill(bytearray(f))  # (shape check only)
    assert pyoracle.checksum(bytes(icmp), len(icmp), 0) == 0 or alt_zero
    return f


def _reply_full(frame: bytearray) -> bytes:
    """src/icmpv4.c:44-47: type = 0, csum = 0, csum = checksum(icmp, icmp_len, 0)."""
    g = bytearray(frame)
    ihl = g[14] & 0xF
    iplen = int.from_bytes(g[16:18], "big")
    o = 14 + ihl * 4
    g[o] = 0
    g[o + 2:o + 4] = b"\0\0"
    g[o + 2:o + 4] = struct.pack("<H", pyoracle.checksum(bytes(g[o:14 + iplen]), iplen - ihl * 4, 0))
    return bytes(g)


def test_icmp_incremental_random():
    rng = np.random.default_rng(61)
    frames = []
    for _ in range(3000):
        ln = int(rng.integers(0, 1473))
        frames.append(_echo_request(rng.integers(0, 256, ln, dtype=np.uint8).tobytes(),
                                    int(rng.integers(0, 1 << 16)), int(rng.integers(0, 1 << 16))))
    want = [_reply_full(f) for f in frames]
    n_re = lvlip.icmp_echo_reply_fill(frames)
    assert [bytes(f) for f in frames] == want
    assert n_re <= 3  # ~1/65535 per frame


def test_icmp_incremental_edges():
    cases = [
        _echo_request(b"", ident=0, seq=0),                    # reply all zero: 0xffff
        _echo_request(b"", ident=0xF7FF, seq=0),               # request sum 0xffff, field 0
        _echo_request(b"", ident=0xF7FF, seq=0, alt_zero=True),  # same, field 0xffff
        _echo_request(b"\xff\xff", ident=0, seq=0),            # reply sum 0xffff: 0x0000
        _echo_request(b"\x00" * 64, ident=0, seq=0),
        _echo_request(b"\xff" * 9, ident=0xFFFF, seq=0xFFFF),  # odd length
    ]
    assert cases[1][36:38] == b"\0\0" and cases[2][36:38] == b"\xff\xff"
    want = [_reply_full(f) for f in cases]
    assert lvlip.icmp_echo_reply_fill([bytearray(f) for f in cases]) == 3  # cases 0, 3, 4
    lvlip.icmp_echo_reply_fill(cases)
    assert [bytes(f) for f in cases] == want
    assert int.from_bytes(want[0][36:38], "little") == 0xFFFF
    assert lvlip.icmp_echo_reply_csum(0xFFF7) == lvlip.CSUM_RECOMPUTE


def test_icmp_incremental_echo_golden():
    """Config #1 requests -> the ICMP part of the replies the reference stack wrote."""
    e = golden_io.echo()["echo"]
    fr = [bytearray(bytes.fromhex(c["request_hex"])) for c in e]
    lvlip.icmp_echo_reply_fill(fr)
    for f, c in zip(fr, e):
        rep = bytes.fromhex(c["reply_hex"])
        iplen = int.from_bytes(rep[16:18], "big")
        assert bytes(f[34:14 + iplen]) == rep[34:14 + iplen]


def test_icmp_incremental_refuses_non_requests():
    fr = [_echo_request(b"abc"), bytearray(workloads.frames(1, seed=62, protos=(6,))[0])]
    before = [bytes(f) for f in fr]
    import pytest
    with pytest.raises(ValueError):
        lvlip.icmp_echo_reply_fill(fr)
    assert [bytes(f) for f in fr] == before


def test_frame_calls_refuse_oversized_batches():
    """A frame yields up to two checksums, so the host frame calls take at most
    LVLIP_MAX_BATCH / 2 frames, like the _dev calls (csum_kernels.hip): larger n is
    LVLIP_EINVAL before the context, the frames or any allocation are touched
    (the dummy pointers below are never dereferenced)."""
    L = lvlip.lib()
    dummy = ctypes.create_string_buffer(64)
    p = ctypes.cast(dummy, ctypes.c_void_p)
    fp = ctypes.cast(dummy, ctypes.POINTER(lvlip.Frame))
    too_many = 0xFFFFFFF0 // 2 + 1
    assert L.lvlip_rx_verify(p, fp, too_many, 0, p) == lvlip.EINVAL
    assert L.lvlip_tx_checksum(p, fp, too_many) == lvlip.EINVAL
    # NULL context: EINVAL too, for any n
    assert L.lvlip_rx_verify(None, fp, 1, 0, p) == lvlip.EINVAL
    assert L.lvlip_tx_checksum(None, fp, 1) == lvlip.EINVAL
