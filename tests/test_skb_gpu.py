"""f1/f2 on the GPU: lvlip_rx_verify / lvlip_tx_checksum (include/lvlip_skb.h)
run their checksums as one GPU batch; every frame is compared with the
oracle's restatement of the reference's RX/TX decisions (oracle/skb_oracle.py)
and, for config #1, with the reference stack's own echo replies."""
import os

import numpy as np
import pytest

import golden_io
import lvlip
import ref_rx_cases
import skb_oracle
import workloads
from test_skb_cpu import _rx_cases, _scrambled_tcp_frames

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or lvlip.device_count() == 0:
        pytest.fail("GPU tests need a HIP device (run them on the MI355X box)")


@pytest.fixture(scope="module")
def ctx():
    with lvlip.Context(0, arena_bytes=4 << 20) as c:
        yield c


def test_tx_checksum_frames(ctx):
    fr = workloads.frames(5000, seed=31)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    ctx.tx_checksum(fr)
    bad = [i for i, (a, b) in enumerate(zip(fr, want)) if bytes(a) != bytes(b)]
    assert not bad, bad[:10]


def test_tx_checksum_jumbo_and_tiny(ctx):
    fr = workloads.frames(300, seed=32, max_l4=9000 - 60) + workloads.frames(300, seed=33, max_l4=8)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    ctx.tx_checksum(fr)
    assert [bytes(f) for f in fr] == [bytes(f) for f in want]


def test_tx_echo_reply_golden(ctx):
    e = golden_io.echo()["echo"]
    fr = []
    for case in e:
        rep = bytearray(bytes.fromhex(case["reply_hex"]))
        rep[24:26] = b"\x00\x00"
        rep[36:38] = b"\xff\xff"
        fr.append(rep)
    ctx.tx_checksum(fr)
    assert [bytes(f) for f in fr] == [bytes.fromhex(c["reply_hex"]) for c in e]


def test_tx_tcp_stack_frames_golden(ctx):
    """The reference TCP transmit path's frames (tests/golden/tcp_frames.json),
    fields scrambled, refilled by the GPU batch == the reference's bytes, on the
    host-resident path and on the device-resident one; RX verify accepts them."""
    fr, want = _scrambled_tcp_frames()
    ctx.tx_checksum(fr)
    assert [bytes(f) for f in fr] == want
    assert ctx.rx_verify(fr, lvlip.RX_VERIFY_L4).tolist() == [lvlip.RX_OK] * len(fr)
    fr, _ = _scrambled_tcp_frames()
    buf, fd = lvlip.pack_frames(fr, align_mod=16, seed=3)
    base = _dev(buf)
    assert lvlip.tx_checksum_dev(base, fd).cpu().numpy().tolist() == [1] * len(fr)
    out = base.cpu().numpy()
    got = [out[int(d["offset"]):int(d["offset"]) + int(d["len"])].tobytes() for d in fd]
    assert got == want
    v = lvlip.rx_verify_dev(base, fd, lvlip.RX_VERIFY_L4).cpu().numpy()
    assert v.tolist() == [lvlip.RX_OK] * len(fr)


def test_tx_malformed_untouched(ctx):
    fr = workloads.frames(10, seed=34, max_l4=200)
    fr[7][14] = 0x35  # version 3
    before = [bytes(f) for f in fr]
    with pytest.raises(lvlip.LvlipError) as ei:
        ctx.tx_checksum(fr)
    assert ei.value.rc == lvlip.EINVAL
    assert [bytes(f) for f in fr] == before


def test_rx_verify_matches_ip_rcv(ctx):
    fr = _rx_cases(41) + _rx_cases(42)
    before = [bytes(f) for f in fr]
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = ctx.rx_verify(fr, flags)
        want = [skb_oracle.rx_verdict(f, flags) for f in fr]
        assert got.tolist() == want, flags
    assert [bytes(f) for f in fr] == before


def test_rx_verify_large_batch(ctx):
    """A batch bigger than the arena: valid TX output verifies OK (header), and
    flipped bytes are caught exactly where the oracle catches them."""
    fr = workloads.frames(20000, seed=43, max_l4=1460)
    ctx.tx_checksum(fr)
    rng = np.random.default_rng(44)
    for i in rng.choice(len(fr), 2000, replace=False):
        f = fr[int(i)]
        f[14 + int(rng.integers(0, len(f) - 14))] ^= 0x10
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = ctx.rx_verify(fr, flags)
        want = np.array([skb_oracle.rx_verdict(f, flags) for f in fr], dtype=np.uint8)
        assert np.array_equal(got, want), flags


def test_rx_echo_requests_ok(ctx):
    e = golden_io.echo()["echo"]
    fr = [bytearray(bytes.fromhex(c["request_hex"])) for c in e]
    assert ctx.rx_verify(fr, lvlip.RX_VERIFY_L4).tolist() == [lvlip.RX_OK] * len(fr)


def test_empty(ctx):
    assert ctx.rx_verify([], 0).size == 0
    ctx.tx_checksum([])


# ------------------------------------- host frames: every source (round 5) --
#
# The host frame calls parse on the device (frames_host.cpp): scattered frames
# are gathered whole into the pinned arena, frames in a registered region are
# DMA'd as spans (LVLIP_REG_DMA, and LVLIP_REG_ZEROCOPY when the frames lie
# densely in it) or read in place (LVLIP_REG_ZEROCOPY, frames spread thinly
# over the region: "zerocopy_sparse", one frame per 4 KiB).  The same frames
# through every source must give the oracle's verdicts and fill.

SOURCES = ("scattered", "slab", "dma", "zerocopy", "zerocopy_sparse")


def _frames_in(source, frames, seed):
    """(views, buf): the frames as separate bytearrays ("scattered"), or as
    numpy views into one slab (frames at every offset mod 16, in shuffled
    order), unregistered or to be registered."""
    if source == "scattered":
        return [bytearray(f) for f in frames], None
    if source == "zerocopy_sparse":
        # one frame per 4 KiB (jumbo frames take more), at a random offset mod
        # 16: the region's span is well over twice the frames' bytes
        rng = np.random.default_rng(seed)
        offs, pos = [], 0
        for f in frames:
            o = pos + int(rng.integers(0, 16))
            offs.append(o)
            pos = (o + len(f) + 4095) // 4096 * 4096
        buf = np.zeros(pos + 64, dtype=np.uint8)
        views = []
        for o, f in zip(offs, frames):
            buf[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
            views.append(buf[o:o + len(f)])
        return views, buf
    buf, fd = lvlip.pack_frames(frames, align_mod=16, seed=seed)
    views = [buf[int(d["offset"]):int(d["offset"]) + int(d["len"])] for d in fd]
    return views, buf


def _registered(ctx, source, buf):
    if source in ("dma", "zerocopy", "zerocopy_sparse"):
        ctx.register(buf, lvlip.REG_DMA if source == "dma" else lvlip.REG_ZEROCOPY)


def _unregister(ctx, source, buf):
    if source in ("dma", "zerocopy", "zerocopy_sparse"):
        ctx.unregister(buf)


@pytest.mark.parametrize("source", SOURCES)
def test_host_frames_every_source_matches_oracle(ctx, source):
    """20 000 frames (options, odd lengths, 300 jumbo) filled by the TX call,
    then 2 000 bit flips and 200 truncations plus every ip_rcv drop reason:
    TX fill == the oracle's fill and the RX verdicts (header, header + L4) ==
    the oracle's, through each source, the order shuffled so the DMA spans
    run out of address order."""
    fr = workloads.frames(20000, seed=81, max_l4=1460) + workloads.frames(300, seed=82, max_l4=8900)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    views, buf = _frames_in(source, fr, seed=83)
    rng = np.random.default_rng(84)
    perm = rng.permutation(len(views))
    _registered(ctx, source, buf)
    try:
        ctx.tx_checksum([views[int(i)] for i in perm])
        got = [bytes(v) for v in views]
        bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != bytes(w)]
        assert not bad, bad[:10]
        for i in rng.choice(len(views), 2000, replace=False):
            v = views[int(i)]
            v[14 + int(rng.integers(0, len(v) - 14))] ^= 0x10
        rx = [views[int(i)] for i in perm]
        for i in rng.choice(len(rx), 200, replace=False):
            rx[int(i)] = rx[int(i)][: int(rng.integers(0, 80))]
        cases = _rx_cases(85)
        for flags in (0, lvlip.RX_VERIFY_L4):
            v = ctx.rx_verify(rx, flags)
            w = np.array([skb_oracle.rx_verdict(bytes(f), flags) for f in rx], dtype=np.uint8)
            assert np.array_equal(v, w), (flags, np.nonzero(v != w)[0][:5])
            # the drop reasons, scattered, in the same call as slab frames
            v = ctx.rx_verify(rx[:3000] + cases, flags)
            w = [skb_oracle.rx_verdict(bytes(f), flags) for f in rx[:3000] + cases]
            assert v.tolist() == w, flags
    finally:
        _unregister(ctx, source, buf)


@pytest.mark.parametrize("source", SOURCES)
def test_host_tx_malformed_untouched_every_source(ctx, source):
    """One malformed frame (version 6) among 20 000, in a late piece: the
    host has already stored the fields of the earlier pieces (the apply runs
    per piece) and must restore them: LVLIP_EINVAL and every frame byte
    unchanged, whichever source the frames come from."""
    fr = workloads.frames(20000, seed=86, max_l4=1460)
    views, buf = _frames_in(source, fr, seed=87)
    views[17500][14] = 0x65
    before = [bytes(v) for v in views]
    _registered(ctx, source, buf)
    try:
        with pytest.raises(lvlip.LvlipError) as ei:
            ctx.tx_checksum(views)
        assert ei.value.rc == lvlip.EINVAL
        assert [bytes(v) for v in views] == before
    finally:
        _unregister(ctx, source, buf)


@pytest.mark.parametrize("source", ("dma", "zerocopy"))
def test_host_frames_region_not_16b_aligned(ctx, source):
    """A region registered from an address 13 B past a 16-B boundary, its
    first frame at its first byte: the DMA spans are rounded from the region's
    start (never before it), zero-copy reads in place; fill and verdicts ==
    the oracle's (the ASan harness poisons the bytes before such a region)."""
    fr = workloads.frames(3000, seed=97, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    total = sum(len(f) for f in fr)
    raw = np.zeros(total + 64, dtype=np.uint8)
    lead = (13 - raw.ctypes.data) % 16
    region = raw[lead:lead + total]
    assert region.ctypes.data % 16 == 13
    views, o = [], 0
    for f in fr:
        region[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        views.append(region[o:o + len(f)])
        o += len(f)
    ctx.register(region, lvlip.REG_DMA if source == "dma" else lvlip.REG_ZEROCOPY)
    try:
        ctx.tx_checksum(views)
        assert [bytes(v) for v in views] == [bytes(w) for w in want]
        for flags in (0, lvlip.RX_VERIFY_L4):
            v = ctx.rx_verify(views, flags)
            w = np.array([skb_oracle.rx_verdict(bytes(f), flags) for f in views], dtype=np.uint8)
            assert np.array_equal(v, w), flags
    finally:
        ctx.unregister(region)


def test_rx_verify_skb_buffers_longer_than_frames(ctx):
    """RX skbs as netdev_rx_loop fills them: every frame at the start of a
    BUFLEN (1600 B) buffer whose end is the frame's end (src/netdev.c:89-91),
    the bytes past the IP total length garbage.  The gather moves only
    max(74, 14 + total length) bytes of each; the verdicts == the oracle's on
    the whole buffers, with total lengths below, at and above the buffer."""
    rng = np.random.default_rng(88)
    fr = workloads.frames(6000, seed=89, max_l4=1400)
    for f in fr:
        skb_oracle.tx_fill(f)
    for i in rng.choice(len(fr), 600, replace=False):
        f = fr[int(i)]
        f[14 + int(rng.integers(0, len(f) - 14))] ^= 0x04
    for i in rng.choice(len(fr), 100, replace=False):  # total length past the buffer
        fr[int(i)][16:18] = int(rng.integers(1600 - 14 + 1, 65536)).to_bytes(2, "big")
    bufs = []
    for f in fr:
        b = bytearray(rng.integers(0, 256, 1600, dtype=np.uint8).tobytes())
        b[:len(f)] = f
        bufs.append(b)
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = ctx.rx_verify(bufs, flags)
        want = np.array([skb_oracle.rx_verdict(bytes(b), flags) for b in bufs], dtype=np.uint8)
        assert np.array_equal(got, want), (flags, np.nonzero(got != want)[0][:5])
    assert (got == lvlip.RX_OK).sum() > 3500


# ------------------------------------------------- device-resident frames --

def _dev(buf):
    t = torch.zeros(buf.size, dtype=torch.uint8, device="cuda")
    t[:] = torch.from_numpy(buf)
    return t


def test_rx_verify_dev_matches_ip_rcv():
    fr = _rx_cases(51) + _rx_cases(52)
    buf, fd = lvlip.pack_frames(fr, align_mod=16, seed=1)  # frames at every alignment
    base = _dev(buf)
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = lvlip.rx_verify_dev(base, fd, flags).cpu().numpy()
        want = [skb_oracle.rx_verdict(f, flags) for f in fr]
        assert got.tolist() == want, flags
    assert np.array_equal(base.cpu().numpy(), buf)  # frames not modified


def test_tx_checksum_dev_matches_reference_tx():
    fr = workloads.frames(6000, seed=53) + workloads.frames(200, seed=54, max_l4=8900)
    bad = [bytearray(b"\x00" * 20), bytearray(workloads.frames(1, seed=55)[0])]
    bad[1][14] = 0x65  # version 6: left untouched, status 0
    allf = fr + bad
    buf, fd = lvlip.pack_frames(allf, align_mod=16, seed=2)
    base = _dev(buf)
    status = lvlip.tx_checksum_dev(base, fd).cpu().numpy()
    assert status.tolist() == [1] * len(fr) + [0, 0]
    out = base.cpu().numpy()
    for i, f in enumerate(allf):
        o, ln = int(fd[i]["offset"]), int(fd[i]["len"])
        want = bytearray(f)
        if i < len(fr):
            skb_oracle.tx_fill(want)
        assert out[o:o + ln].tobytes() == bytes(want), i
    # nothing between frames was written
    mask = np.ones(buf.size, dtype=bool)
    for d in fd:
        mask[int(d["offset"]):int(d["offset"]) + int(d["len"])] = False
    assert np.array_equal(out[mask], buf[mask])


def test_tx_checksum_dev_plain_and_nt_stores_agree():
    """The device TX fill with every field-store kind (the product's `nt sc0
    sc1`; the lab's nontemporal, plain, sc0, sc1, sc0 sc1, nt sc1 and whole
    32-B / 64-B blocks) and the lab's other shapes (8 loads per round, block
    order): identical frames, equal to the oracle's fill, odd and even field
    addresses (frames at every alignment)."""
    fr = workloads.frames(3000, seed=58) + workloads.frames(100, seed=59, max_l4=8900)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    buf, fd = lvlip.pack_frames(fr, align_mod=16, seed=5)
    # product (nt sc0 sc1 field stores), then the lab's: plain, 8 loads per
    # round, block order, U 8 blocks plain, whole 32-B / 64-B blocks, and the
    # field stores' cache policies sc0 .. nt sc0 sc1 (round 4)
    for kind in ("nt", "plain", 2, 4, 6, 7, 16, 32, 64, 128, 192, 256, 320):
        base = _dev(buf)
        if kind == "nt":
            st = lvlip.tx_checksum_dev(base, fd)
        else:
            st = lvlip.frames_variant_dev(0, 1 if kind == "plain" else kind, base, fd)
        assert int(st.sum()) == len(fr), kind
        out = base.cpu().numpy()
        got = [out[int(d["offset"]):int(d["offset"]) + int(d["len"])].tobytes() for d in fd]
        assert got == [bytes(f) for f in want], kind


def test_tx_dev_then_rx_dev_roundtrip_large():
    """2^17 frames built and filled on the GPU verify OK on the GPU (header and,
    where the TCP seed kept its carry, L4), matching the host path verdicts."""
    fr = workloads.frames(1 << 17, seed=56, max_l4=1460, options=False)
    buf, fd = lvlip.pack_frames(fr, align_mod=1)
    base = _dev(buf)
    assert int(lvlip.tx_checksum_dev(base, fd).sum()) == len(fr)
    v = lvlip.rx_verify_dev(base, fd, lvlip.RX_VERIFY_L4).cpu().numpy()
    out = base.cpu().numpy()
    filled = [bytearray(out[int(d["offset"]):int(d["offset"]) + int(d["len"])].tobytes()) for d in fd]
    with lvlip.Context(0) as ctx:
        assert np.array_equal(ctx.rx_verify(filled, lvlip.RX_VERIFY_L4), v)
    assert (v == lvlip.RX_OK).mean() > 0.4 and set(np.unique(v)) <= {lvlip.RX_OK, lvlip.RX_BAD_L4}


def test_dev_frames_arguments():
    """Argument errors return LVLIP_EINVAL before any launch; n = 0 is a no-op;
    the reserved workspace may be NULL (its size is 0)."""
    lib = lvlip.lib()
    assert lib.lvlip_frames_workspace_bytes(1000) == 0
    fr = workloads.frames(8, seed=57)
    buf, fd = lvlip.pack_frames(fr, align_mod=1)
    base = _dev(np.concatenate([buf, np.zeros(32, np.uint8)]))
    fdt = torch.from_numpy(fd.view(np.uint8).copy()).cuda()
    out = torch.zeros(8, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    p, f, o = base.data_ptr(), fdt.data_ptr(), out.data_ptr()
    assert lib.lvlip_rx_verify_dev(p + 1, f, 8, 0, o, None, s) == lvlip.EINVAL  # base not 16-B aligned
    assert lib.lvlip_rx_verify_dev(p, None, 8, 0, o, None, s) == lvlip.EINVAL
    assert lib.lvlip_rx_verify_dev(p, f, 8, 0, None, None, s) == lvlip.EINVAL  # verdict required
    assert lib.lvlip_tx_checksum_dev(None, f, 8, o, None, s) == lvlip.EINVAL
    assert lib.lvlip_rx_verify_dev(p, f, 0, 0, None, None, s) == lvlip.OK      # n = 0
    assert lib.lvlip_tx_checksum_dev(p, f, 8, None, None, s) == lvlip.OK       # status optional
    torch.cuda.synchronize()
    assert lib.lvlip_rx_verify_dev(p, f, 8, 0, o, None, s) == lvlip.OK  # headers filled above
    torch.cuda.synchronize()
    assert out.cpu().numpy().tolist() == [lvlip.RX_OK] * 8


# ------------------------------------------- against level-ip's own ip_rcv --

@pytest.mark.skipif(not os.path.exists(ref_rx_cases.REF_SO), reason="oracle/_ref/libref.so not built")
def test_rx_verify_agrees_with_reference_ip_rcv(ctx):
    """Batch-and-dispatch in front of level-ip's RX path: the
    GPU batch accepts exactly the frames the reference's own ip_rcv accepts
    (tests/ref_rx_child.py on oracle/_ref/libref.so: every drop reason, IP
    options), host- and device-resident; and handing the stack only the frames
    the batch accepted produces the same replies as handing it all of them."""
    frs, kinds = ref_rx_cases.frames(8)
    replies = ref_rx_cases.reference_replies(frs)
    got = ctx.rx_verify(frs, 0)
    assert [int(v) == lvlip.RX_OK for v in got] == [r is not None for r in replies]
    got_l4 = ctx.rx_verify(frs, lvlip.RX_VERIFY_L4)
    for v, k, r in zip(got_l4, kinds, replies):
        if v == lvlip.RX_OK:
            assert r is not None, k
        if k == "icmp_csum":  # answered by the reference, caught by the L4 check
            assert v == lvlip.RX_BAD_L4 and r is not None
    buf, fd = lvlip.pack_frames(frs, align_mod=16, seed=3)
    dev = lvlip.rx_verify_dev(_dev(buf), fd, 0).cpu().numpy()
    assert np.array_equal(dev, got)
    accepted = [f for f, v in zip(frs, got) if v == lvlip.RX_OK]
    assert ref_rx_cases.reference_replies(accepted) == [r for r, v in zip(replies, got)
                                                        if v == lvlip.RX_OK]


def test_rx_header_lane_and_flat_agree():
    """The header-only RX call on both of its kernels (k_rx_hdr, one lane per
    frame, the product; k_flat2 with a frame source, the lab variant, in its
    shapes):
    20 000 frames at every alignment, 20 % with IP options (ihl 6-15, the
    window's last words and the byte-load tail), a tenth with a flipped bit in
    the header or beyond, some truncated; every verdict == the oracle's."""
    fr = workloads.frames(20000, seed=61, max_l4=1460)
    for f in fr:
        skb_oracle.tx_fill(f)
    rng = np.random.default_rng(62)
    for i in rng.choice(len(fr), 2000, replace=False):
        f = fr[int(i)]
        ihl = f[14] & 0xF
        f[14 + int(rng.integers(0, ihl * 4 + 8))] ^= 1 << int(rng.integers(0, 8))
    for i in rng.choice(len(fr), 200, replace=False):
        fr[int(i)] = fr[int(i)][: int(rng.integers(0, 80))]
    want = [skb_oracle.rx_verdict(f, 0) for f in fr]
    buf, fd = lvlip.pack_frames(fr, align_mod=16, seed=4)
    base = _dev(buf)
    for kern in ("lane", 0, 2, 4, 6):
        if kern == "lane":
            got = lvlip.rx_verify_dev(base, fd, 0).cpu().numpy()
        else:
            got = lvlip.frames_variant_dev(1, kern, base, fd).cpu().numpy()
        bad = np.nonzero(got != np.array(want, dtype=np.uint8))[0]
        assert bad.size == 0, (kern, bad[:5])
    assert len(set(want)) >= 3


# ------------------------------------------------ f4: echo reply in HBM --

def _icmp_reply_ref(frame: bytes) -> bytes:
    """icmpv4_reply's ICMP part (src/icmpv4.c:44-47) on a request frame: type 0,
    checksum field zeroed, checksum over icmp_len = ip.len - ihl*4 bytes (the
    oracle restatement of src/utils.c:40-55), stored raw."""
    import pyoracle

    f = bytearray(frame)
    ihl = f[14] & 0xF
    l4, n = 14 + ihl * 4, int.from_bytes(f[16:18], "big") - ihl * 4
    f[l4] = 0
    f[l4 + 2:l4 + 4] = b"\x00\x00"
    f[l4 + 2:l4 + 4] = pyoracle.checksum(bytes(f[l4:l4 + n]), n, 0).to_bytes(2, "little")
    return bytes(f)


def _echo_requests(rng, n, ihl_max=5):
    """n verified ICMP echo requests (random payload lengths, odd ones
    included) with the RFC 1624 corner cases mixed in: request checksum field
    0xffff (the other zero: the message sums to 0xffff), and the undecidable
    replies (S' = 0xffff: an all-zero echo body, whose reply field is 0xffff,
    and an all-0xff body, whose reply field is 0x0000)."""
    import pyoracle

    out, kinds = [], []
    for i in range(n):
        kind = ("random", "random", "random", "ffff", "zero", "ones")[int(rng.integers(0, 6))] \
            if i >= 4 else ("ffff", "zero", "ones", "random")[i]
        ihl = 5 if ihl_max == 5 or rng.random() < 0.5 else int(rng.integers(6, ihl_max + 1))
        plen = int(rng.integers(0, 1473 - 4 * (ihl - 5)))
        if kind == "ones":
            plen &= ~1
        body = bytearray(4 + plen)  # id, seq, payload
        if kind == "random" or kind == "ffff":
            body[:] = rng.integers(0, 256, len(body), dtype=np.uint8).tobytes()
        elif kind == "ones":
            body[:] = b"\xff" * len(body)
        icmp = bytearray(b"\x08\x00\x00\x00") + body
        if kind == "ffff":
            # make the message (field zeroed) sum to 0xffff: fix the id word
            icmp[4:6] = b"\x00\x00"
            s = 0xFFFF & ~pyoracle.checksum(bytes(icmp), len(icmp), 0)  # one's-complement sum
            w = (0xFFFF - s) & 0xFFFF  # s + w == 0xffff (one's complement)
            icmp[4:6] = w.to_bytes(2, "little")
        c = pyoracle.checksum(bytes(icmp), len(icmp), 0)
        icmp[2:4] = c.to_bytes(2, "little")
        if kind == "ffff":
            assert c == 0
            icmp[2:4] = b"\xff\xff"  # the other representation, still verifies
        assert pyoracle.checksum(bytes(icmp), len(icmp), 0) == 0, kind
        iplen = ihl * 4 + len(icmp)
        ih = bytearray(rng.integers(0, 256, ihl * 4, dtype=np.uint8).tobytes())
        ih[0] = 0x40 | ihl
        ih[2:4] = iplen.to_bytes(2, "big")
        ih[8] = 64
        ih[9] = 1
        pad = bytes(rng.integers(0, 256, int(rng.integers(0, 4)), dtype=np.uint8).tobytes())
        eth = bytes(rng.integers(0, 256, 12, dtype=np.uint8).tobytes()) + b"\x08\x00"
        out.append(bytearray(eth + bytes(ih) + bytes(icmp) + pad))
        kinds.append(kind)
    return out, kinds


def _run_echo_dev(frames, flags=0):
    buf, fd = lvlip.pack_frames(frames, align_mod=16, seed=9)
    base = _dev(buf)
    st = lvlip.icmp_echo_reply_dev(base, fd, flags=flags).cpu().numpy()
    out = base.cpu().numpy()
    got = [out[int(d["offset"]):int(d["offset"]) + int(d["len"])].tobytes() for d in fd]
    rest = np.ones(buf.size, dtype=bool)
    for d in fd:
        rest[int(d["offset"]):int(d["offset"]) + int(d["len"])] = False
    assert np.array_equal(out[rest], buf[rest])  # nothing outside the frames written
    return st, got


def test_icmp_echo_reply_dev_golden_echo():
    """Config #1's echo requests (tests/golden/echo.json, recorded from the
    reference stack): the device reply's ICMP part equals the reference stack's
    own reply byte for byte."""
    e = golden_io.echo()["echo"]
    reqs = [bytearray(bytes.fromhex(c["request_hex"])) for c in e]
    st, got = _run_echo_dev(reqs)
    for c, g, s in zip(e, got, st):
        rep = bytes.fromhex(c["reply_hex"])
        ihl = g[14] & 0xF
        n = int.from_bytes(g[16:18], "big") - ihl * 4
        assert g[34:34 + n] == rep[34:34 + n]
        assert s in (1, 2)


def test_icmp_echo_reply_dev_random_and_corner_cases():
    """20 000 verified requests (ihl 5-15: the parse window's field and the byte
    loads past it) plus non-requests (replies, other ICMP types, TCP, short
    frames): every frame equals the oracle's icmpv4_reply recomputation, the
    corner fields included; the status says which lanes recomputed."""
    rng = np.random.default_rng(71)
    fr, kinds = _echo_requests(rng, 20000, ihl_max=15)
    others = workloads.frames(600, seed=72)  # TCP and ICMP type 8 with garbage fields
    for f in others:
        if f[23] == 1:
            f[14 + (f[14] & 0xF) * 4] = int(rng.choice([0, 3, 11]))  # not a request
    short = [bytearray(f[:int(rng.integers(0, 40))]) for f in fr[:50]]
    allf = fr + others + short
    st, got = _run_echo_dev(allf)
    for i, (f, g) in enumerate(zip(fr, got)):
        assert g == _icmp_reply_ref(f), (i, kinds[i])
    st_req = st[:len(fr)]
    und = np.array([k in ("zero", "ones") for k in kinds])
    assert (st_req[und] == 2).all() and (st_req[~und] == 1).all()
    for f, g, s in zip(others + short, got[len(fr):], st[len(fr):]):
        assert s == 0 and g == bytes(f)
    assert {"ffff", "zero", "ones"} <= set(kinds)


@pytest.mark.skipif(not os.path.exists(ref_rx_cases.REF_SO), reason="oracle/_ref/libref.so not built")
def test_icmp_echo_reply_dev_agrees_with_reference_stack():
    """2 000 random requests (ihl 5, as icmpv4_reply assumes: it reads the ICMP
    message at head + 34, src/icmpv4.c:38-43) through level-ip's own ip_rcv ->
    icmpv4_reply (oracle/_ref/libref.so): the device reply's ICMP part equals
    the stack's reply for every one, the 0xffff and undecidable fields
    included."""
    rng = np.random.default_rng(73)
    fr, kinds = _echo_requests(rng, 2000)
    for f in fr:  # the stack checks the IPv4 header and answers 10.0.0.4 only
        f[14 + 12:14 + 16] = bytes([10, 0, 0, 5])
        f[14 + 16:14 + 20] = bytes([10, 0, 0, 4])
        f[14 + 6:14 + 8] = b"\x40\x00"
        f[14 + 10:14 + 12] = b"\x00\x00"
        c = lvlip.checksum(bytes(f[14:34]), 20, 0)
        f[24:26] = c.to_bytes(2, "little")
        f[0:6] = bytes.fromhex("000c296d5025")
    replies = ref_rx_cases.reference_replies(fr)
    st, got = _run_echo_dev(fr)
    assert all(r is not None for r in replies)
    for i, (g, r) in enumerate(zip(got, replies)):
        n = int.from_bytes(g[16:18], "big") - 20
        assert g[34:34 + n] == r[34:34 + n], (i, kinds[i])
    assert {"ffff", "zero", "ones"} <= set(kinds)


def _corrupt_icmp(frames, rng):
    """Echo requests whose ICMP checksum field no longer verifies."""
    out = []
    for f in frames:
        g = bytearray(f)
        l4 = 14 + (g[14] & 0xF) * 4
        old = bytes(g[l4 + 2:l4 + 4])
        while bytes(g[l4 + 2:l4 + 4]) == old or g[l4 + 2:l4 + 4] in (b"\x00\x00", b"\xff\xff"):
            g[l4 + 2:l4 + 4] = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()
        out.append(g)
    return out


def test_icmp_echo_reply_dev_corrupted_requests_pin_both_modes():
    """a request whose ICMP checksum does not verify.  level-ip
    answers it with icmpv4_reply's full recomputation (src/icmpv4.c:11 never
    verifies, :45-47 recompute).  flags 0 (the documented precondition is
    broken): the lane writes the RFC 1624 field from the request's field, which
    differs from the reference's for these frames, status 1.  LVLIP_ECHO_FULL:
    the reference's bytes for every frame, status 2."""
    rng = np.random.default_rng(74)
    good, _ = _echo_requests(rng, 3000, ihl_max=15)
    bad = _corrupt_icmp(good, rng)
    st0, got0 = _run_echo_dev(bad)
    stf, gotf = _run_echo_dev(bad, flags=lvlip.ECHO_FULL)
    differ = 0
    for f, g0, gf, s0 in zip(bad, got0, gotf, st0):
        ref = _icmp_reply_ref(f)
        assert gf == ref
        l4 = 14 + (f[14] & 0xF) * 4
        hc = int.from_bytes(f[l4 + 2:l4 + 4], "little")
        inc = lvlip.icmp_echo_reply_csum(hc)
        if inc != lvlip.CSUM_RECOMPUTE:
            assert s0 == 1 and int.from_bytes(g0[l4 + 2:l4 + 4], "little") == inc
            assert g0[l4] == 0 and g0[:l4 + 2] == ref[:l4 + 2] and g0[l4 + 4:] == ref[l4 + 4:]
        differ += g0 != ref
    assert (stf == 2).all()
    assert differ > 2900  # the incremental field is wrong for (almost) every corrupted request


def test_icmp_echo_reply_dev_full_equals_oracle():
    """LVLIP_ECHO_FULL on the verified requests of the corner-case test (ihl
    5-15, 0xffff fields, both undecidable kinds) and on non-requests: every
    frame equals the oracle's icmpv4_reply recomputation, non-requests stay
    untouched (status 0)."""
    rng = np.random.default_rng(75)
    fr, kinds = _echo_requests(rng, 8000, ihl_max=15)
    others = workloads.frames(300, seed=76)
    for f in others:
        if f[23] == 1:
            f[14 + (f[14] & 0xF) * 4] = int(rng.choice([0, 3, 11]))
    st, got = _run_echo_dev(fr + others, flags=lvlip.ECHO_FULL)
    for i, (f, g) in enumerate(zip(fr, got)):
        assert g == _icmp_reply_ref(f), (i, kinds[i])
    assert (st[:len(fr)] == 2).all()
    for f, g, s in zip(others, got[len(fr):], st[len(fr):]):
        assert s == 0 and g == bytes(f)


@pytest.mark.skipif(not os.path.exists(ref_rx_cases.REF_SO), reason="oracle/_ref/libref.so not built")
def test_icmp_echo_reply_dev_full_agrees_with_reference_stack_on_corrupted():
    """Corrupted requests (the ICMP field garbage) through level-ip's own ip_rcv
    -> icmpv4_reply (oracle/_ref/libref.so), which answers them: the
    LVLIP_ECHO_FULL reply's ICMP part equals the stack's for every one."""
    rng = np.random.default_rng(77)
    fr, _ = _echo_requests(rng, 1000)
    fr = _corrupt_icmp(fr, rng)
    for f in fr:
        f[14 + 12:14 + 16] = bytes([10, 0, 0, 5])
        f[14 + 16:14 + 20] = bytes([10, 0, 0, 4])
        f[14 + 6:14 + 8] = b"\x40\x00"
        f[14 + 10:14 + 12] = b"\x00\x00"
        c = lvlip.checksum(bytes(f[14:34]), 20, 0)
        f[24:26] = c.to_bytes(2, "little")
        f[0:6] = bytes.fromhex("000c296d5025")
    replies = ref_rx_cases.reference_replies(fr)
    assert all(r is not None for r in replies)
    _, got = _run_echo_dev(fr, flags=lvlip.ECHO_FULL)
    for i, (g, r) in enumerate(zip(got, replies)):
        n = int.from_bytes(g[16:18], "big") - 20
        assert g[34:34 + n] == r[34:34 + n], i


def _tx_kinds():
    return [None, 7, 16, 32, 128, 320]


def test_tx_fill_dev_block_stores_every_alignment_and_packed_frames():
    """VERDICT r03 Next #1's cases for the whole-block field stores (lab
    variants 16 / 32) and the product: frames starting at every offset mod 32
    (and mod 64), 54-B TCP frames (14 + 20 + 20: both fields inside one 32-B
    sector for some offsets, the next frame's first bytes in the same block)
    packed back to back with no gap, and ICMP frames whose two fields share a
    sector.  Every variant's frames equal the oracle's fill, and no byte
    outside the frames changes."""
    rng = np.random.default_rng(90)
    fr = []
    for k in range(64 * 6):
        f = workloads.frames(1, seed=1000 + k, max_l4=int(rng.choice([20, 24, 40, 200])),
                             options=bool(k % 3 == 0), protos=(6,) if k % 2 else (1,))[0]
        fr.append(f)
    # 54-B TCP frames (no options, 20-B segment), packed back to back
    tight = workloads.frames(256, seed=91, max_l4=20, options=False, protos=(6,))
    for f in tight:
        del f[14 + 20 + 20:]
        f[16:18] = (40).to_bytes(2, "big")
    want = [bytearray(f) for f in fr + tight]
    for f in want:
        skb_oracle.tx_fill(f)
    # every frame of `fr` at its own offset mod 64: a 64-B aligned slot plus k
    slots, off = [], 0
    for k, f in enumerate(fr):
        off = (off + 63) // 64 * 64 + (k % 64)
        slots.append(off)
        off += len(f)
    for f in tight:  # back to back, from an odd offset
        slots.append(off + 1 if f is tight[0] else off)
        off = slots[-1] + len(f)
    buf = rng.integers(0, 256, (off + 64 + 15) // 16 * 16, dtype=np.uint8)
    allf = fr + tight
    for o, f in zip(slots, allf):
        buf[o:o + len(f)] = np.frombuffer(bytes(f), np.uint8)
    fd = np.zeros(len(allf), dtype=lvlip.FRAME_DESC_DTYPE)
    fd["offset"] = slots
    fd["len"] = [len(f) for f in allf]
    outside = np.ones(buf.size, bool)
    for o, f in zip(slots, allf):
        outside[o:o + len(f)] = False
    for kind in _tx_kinds():
        base = _dev(buf)
        st = lvlip.tx_checksum_dev(base, fd) if kind is None else lvlip.frames_variant_dev(0, kind, base, fd)
        assert int(st.sum()) == len(allf), kind
        out = base.cpu().numpy()
        got = [out[o:o + len(f)].tobytes() for o, f in zip(slots, allf)]
        assert got == [bytes(f) for f in want], kind
        assert np.array_equal(out[outside], buf[outside]), kind
