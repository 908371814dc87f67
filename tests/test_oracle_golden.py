"""The oracle (oracle/csum_oracle.c) pinned against the reference's own outputs.

Fixtures in tests/golden/ were produced by level-ip's src/utils.c and src/tcp.c
compiled from /root/reference (tests/golden/make_golden.py).  When the compiled
reference is present (the build container) the oracle is additionally
cross-checked against it on fresh random inputs.
"""
import numpy as np
import pytest

import golden_io
import pyoracle


def test_kats_match_reference_outputs():
    cases, tcp = golden_io.kats()
    assert len(cases) >= 11
    for name, data, count, start, expected in cases:
        got = pyoracle.checksum(data if data else b"\0", count, start)
        assert got == expected, name
    for t in tcp:
        data = bytes.fromhex(t["data_hex"])
        seed = pyoracle.pseudo_sum(t["saddr"], t["daddr"], t["proto"], t["len"])
        assert pyoracle.checksum(data, t["len"], seed) == t["expected"], t["name"]


def test_lost_carry_is_reproduced():
    # 10.0.0.200 -> 10.0.0.100 over 20 zero bytes gives 0xb9eb in the
    # reference, one off the RFC-correct value because the pseudo-header carry is lost.
    s = int.from_bytes(bytes([10, 0, 0, 200]), "little")
    d = int.from_bytes(bytes([10, 0, 0, 100]), "little")
    seed = pyoracle.pseudo_sum(s, d, 6, 20)
    assert seed < s  # wrapped
    assert pyoracle.checksum(bytes(20), 20, seed) == 0xB9EB


def test_vectors_match_reference():
    v = golden_io.vectors()
    blob = v["blob"]
    descs = np.zeros(v["offset"].size, dtype=[("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    descs["offset"], descs["len"], descs["start_sum"] = v["offset"], v["len"], v["start_sum"]
    got = pyoracle.batch(blob, descs)
    bad = np.nonzero(got != v["expected"])[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}"
    assert got.size > 2500


def test_tcp_vectors_match_reference():
    t = golden_io.tcp()
    for i in range(t["len"].size):
        off, ln = int(t["offset"][i]), int(t["len"][i])
        seed = pyoracle.pseudo_sum(int(t["saddr"][i]), int(t["daddr"][i]), int(t["proto"][i]), ln)
        got = pyoracle.checksum(t["blob"][off:off + max(ln, 1)], ln, seed)
        assert got == int(t["expected"][i]), i


def test_ip_send_check_vectors():
    h = golden_io.iphdr()
    for hdr, after in zip(h["hdr"], h["after"]):
        buf = hdr.copy()
        ihl = buf[0] & 0xF
        c = pyoracle.checksum(buf[: ihl * 4], ihl * 4, 0)
        buf[10:12] = np.frombuffer(int(c).to_bytes(2, "little"), dtype=np.uint8)
        assert np.array_equal(buf, after)


def test_O0_build_agrees():
    v = golden_io.vectors()
    descs = np.zeros(v["offset"].size, dtype=[("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    descs["offset"], descs["len"], descs["start_sum"] = v["offset"], v["len"], v["start_sum"]
    got = pyoracle.batch(v["blob"], descs, threads=4, opt=0)
    assert np.array_equal(got, v["expected"])


@pytest.mark.skipif(pyoracle.reflib() is None, reason="compiled reference not present")
def test_oracle_vs_live_reference_random():
    ref = pyoracle.reflib()
    rng = np.random.default_rng(7)
    blob = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    descs = np.zeros(3000, dtype=[("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
    descs["len"] = rng.integers(-3, 5000, 3000)
    descs["offset"] = [int(rng.integers(0, blob.size - max(int(l), 0))) for l in descs["len"]]
    descs["start_sum"] = rng.integers(0, 2**32, 3000, dtype=np.uint64).astype(np.uint32)
    ours = pyoracle.batch(blob, descs)
    theirs = pyoracle.batch(blob, descs, threads=3, use_reference=True)
    assert np.array_equal(ours, theirs)
    # and sum_every_16bits directly
    for i in range(200):
        off, ln = int(descs["offset"][i]), int(descs["len"][i])
        a = blob[off:]
        assert pyoracle.sum_every_16bits(a, ln) == ref.sum_every_16bits(a.ctypes.data, ln)
