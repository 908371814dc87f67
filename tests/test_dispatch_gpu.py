"""The size-based dispatch of a context's host calls (include/lvlip_csum.h,
lvlip_csum_ctx_set_cpu_max; VERDICT r05 Next #1), its failure paths, and the
order-aware span rule of the registered-region paths.

Both sides of the threshold must give the same bytes, verdicts and return
codes: a call of at most cpu_max packets / frames runs on the calling thread
(the library's CPU code), a larger one on the GPU; the context's counters
(lvlip_csum_ctx_stats) say which side ran.  Everything is compared with the
oracle (oracle/skb_oracle.py, oracle/pyoracle.py)."""
import os

import numpy as np
import pytest

import lvlip
import pyoracle
import skb_oracle
import workloads
from test_skb_cpu import _rx_cases

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or lvlip.device_count() == 0:
        pytest.fail("GPU tests need a HIP device (run them on the MI355X box)")


def _side(ctx, before):
    st = ctx.stats()
    if st["cpu_calls"] > before["cpu_calls"]:
        assert st["gpu_calls"] == before["gpu_calls"]
        return "cpu"
    assert st["gpu_calls"] == before["gpu_calls"] + 1 and st["pieces"] > before["pieces"]
    return "gpu"


def test_default_threshold_from_library_and_env(monkeypatch):
    monkeypatch.delenv("LVLIP_CPU_MAX", raising=False)
    with lvlip.Context(0) as c:
        assert c.cpu_max == lvlip.CPU_MAX_DEFAULT
        c.set_cpu_max(0)
        assert c.cpu_max == 0
    monkeypatch.setenv("LVLIP_CPU_MAX", "77")
    with lvlip.Context(0) as c:
        assert c.cpu_max == 77
    with lvlip.Context(0, cpu_max=5) as c:
        assert c.cpu_max == 5
    assert lvlip.lib().lvlip_csum_ctx_set_cpu_max(None, 1) == lvlip.EINVAL


@pytest.mark.parametrize("n", [1, 3, 8, 64, 511, 512, 513])
def test_frames_both_sides_of_threshold(n):
    """TX fill and RX verdicts (header, header + L4) for n frames with the
    threshold at 512: n <= 512 on the CPU, above on the GPU; both equal the
    oracle, and the counters show the side."""
    fr = workloads.frames(n, seed=100 + n, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    with lvlip.Context(0, arena_bytes=1 << 20, cpu_max=512) as ctx:
        s0 = ctx.stats()
        ctx.tx_checksum(fr)
        assert _side(ctx, s0) == ("cpu" if n <= 512 else "gpu")
        assert [bytes(f) for f in fr] == [bytes(w) for w in want]
        rx = (fr + _rx_cases(100 + n))[:n]
        for flags in (0, lvlip.RX_VERIFY_L4):
            s0 = ctx.stats()
            v = ctx.rx_verify(rx, flags)
            assert _side(ctx, s0) == ("cpu" if n <= 512 else "gpu")
            assert v.tolist() == [skb_oracle.rx_verdict(bytes(f), flags) for f in rx], flags


@pytest.mark.parametrize("cpu_max", [0, 1 << 30])
def test_frames_same_bytes_either_side(cpu_max):
    """The same 3 000 frames (every ip_rcv drop reason among them) forced to
    the GPU (cpu_max 0) and to the CPU (cpu_max 2^30): identical fills and
    verdicts, and identical refusals (a malformed frame: LVLIP_EINVAL, batch
    untouched; a frame longer than the arena: LVLIP_ERANGE)."""
    fr = workloads.frames(3000, seed=110, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    side = "gpu" if cpu_max == 0 else "cpu"
    with lvlip.Context(0, arena_bytes=1 << 20, cpu_max=cpu_max) as ctx:
        s0 = ctx.stats()
        ctx.tx_checksum(fr)
        assert _side(ctx, s0) == side
        assert [bytes(f) for f in fr] == [bytes(w) for w in want]
        rx = fr[:2500] + _rx_cases(111)
        for flags in (0, lvlip.RX_VERIFY_L4):
            assert ctx.rx_verify(rx, flags).tolist() == [skb_oracle.rx_verdict(bytes(f), flags) for f in rx]
        bad = [bytearray(f) for f in fr]
        bad[2900][14] = 0x65
        before = [bytes(f) for f in bad]
        with pytest.raises(lvlip.LvlipError) as e:
            ctx.tx_checksum(bad)
        assert e.value.rc == lvlip.EINVAL and [bytes(f) for f in bad] == before
    with lvlip.Context(0, arena_bytes=4096, cpu_max=cpu_max) as ctx:
        big = workloads.frames(4, seed=112, max_l4=5000)
        big[2] = bytearray(big[2]) + bytearray(5000)
        for call in (lambda: ctx.tx_checksum(big), lambda: ctx.rx_verify(big, lvlip.RX_VERIFY_L4)):
            with pytest.raises(lvlip.LvlipError) as e:
                call()
            assert e.value.rc == lvlip.ERANGE
        ctx.rx_verify(big, 0)  # the header-only call never refuses


@pytest.mark.parametrize("n", [1, 8, 300, 301])
def test_packets_both_sides_of_threshold(n):
    """lvlip_csum_batch_host (iov) and _flat on n packets with the threshold
    at 300: equal to the oracle on both sides; empty packets and u32 seeds
    with the top bit set included; a packet larger than the arena is
    LVLIP_ERANGE on both sides."""
    rng = np.random.default_rng(120 + n)
    lens = rng.integers(0, 3000, n)
    lens[::7] = 0
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    pk = [rng.integers(0, 256, int(l), dtype=np.uint8) for l in lens]
    want = np.array([pyoracle.checksum(p.tobytes() or b"\0", int(l), int(s)) for p, l, s in zip(pk, lens, seeds)],
                    dtype=np.uint16)
    flat = np.zeros(int(lens.sum()) + n + 96, np.uint8)
    d = np.zeros(n, dtype=lvlip.DESC_DTYPE)
    o = 3
    for i, p in enumerate(pk):
        flat[o:o + p.size] = p
        d[i] = (o, p.size, int(seeds[i]))
        o += p.size + 1
    for cpu_max in (300, 0, 1 << 30):
        with lvlip.Context(0, arena_bytes=1 << 20, cpu_max=cpu_max) as ctx:
            s0 = ctx.stats()
            got = ctx.batch_host(pk, [int(s) for s in seeds])
            side = _side(ctx, s0)
            assert side == ("cpu" if n <= cpu_max else "gpu")
            assert np.array_equal(got, want)
            assert np.array_equal(ctx.batch_host_flat(flat, d), want)
    for cpu_max in (0, 1 << 30):
        with lvlip.Context(0, arena_bytes=4096, cpu_max=cpu_max) as ctx:
            with pytest.raises(lvlip.LvlipError) as e:
                ctx.batch_host([np.zeros(8, np.uint8), np.zeros(5000, np.uint8)], [0, 0])
            assert e.value.rc == lvlip.ERANGE


def test_failed_gpu_tx_undoes_then_cpu_fills():
    """LVLIP_FAIL_PIECE=3 makes the third device piece of every GPU call
    fail (LVLIP_EHIP) after the first pieces' fields were stored: the call
    restores every frame (untouched), and lvlip_tx_checksum_cpu then fills
    them, byte-identical to the oracle: no frame is left with a half-done or
    deferred field."""
    fr = workloads.frames(20000, seed=130, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    before = [bytes(f) for f in fr]
    old = os.environ.get("LVLIP_FAIL_PIECE")
    os.environ["LVLIP_FAIL_PIECE"] = "3"
    try:
        ctx = lvlip.Context(0, arena_bytes=1 << 20, cpu_max=0)
    finally:
        if old is None:
            del os.environ["LVLIP_FAIL_PIECE"]
        else:
            os.environ["LVLIP_FAIL_PIECE"] = old
    with ctx:
        with pytest.raises(lvlip.LvlipError) as e:
            ctx.tx_checksum(fr)
        assert e.value.rc == lvlip.EHIP and "LVLIP_FAIL_PIECE" in str(e.value)
        assert [bytes(f) for f in fr] == before
        assert ctx.stats()["pieces"] >= 3
        # a call of fewer pieces is not affected
        small = [bytearray(f) for f in fr[:50]]
        ctx.tx_checksum(small)
        assert [bytes(f) for f in small] == [bytes(w) for w in want[:50]]
    lvlip.tx_checksum_cpu(fr)
    assert [bytes(f) for f in fr] == [bytes(w) for w in want]


def _slab(frames, order_seed=None):
    """The frames packed in one slab (address order = list order), and the
    call order: the identity, or a permutation."""
    buf, fd = lvlip.pack_frames(frames, align_mod=16, seed=7)
    views = [buf[int(x["offset"]):int(x["offset"]) + int(x["len"])] for x in fd]
    perm = np.arange(len(views))
    if order_seed is not None:
        perm = np.random.default_rng(order_seed).permutation(len(views))
    return buf, fd, views, perm


@pytest.mark.parametrize("shuffled", [False, True])
def test_dma_region_spans_only_in_order(shuffled):
    """frames of a registered DMA slab larger than the arena, in
    address order, move as spans (the h2d bytes are about the slab's); the
    same frames in shuffled call order would cut into pieces of one or two
    frames, each moving up to a whole piece of span: they are gathered
    instead (h2d bytes about their own 16-B slots, not pieces x span).  The
    results equal the oracle either way; the packet calls (iov and flat)
    follow the same rule."""
    fr = workloads.frames(12000, seed=140, max_l4=1460)  # ~9 MB against a 1 MiB arena
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    buf, fd, views, perm = _slab(fr, 141 if shuffled else None)
    call = [views[int(i)] for i in perm]
    frame_bytes = sum(len(f) for f in fr)
    with lvlip.Context(0, arena_bytes=1 << 20, cpu_max=0) as ctx:
        ctx.register(buf, lvlip.REG_DMA)
        try:
            s0 = ctx.stats()
            ctx.tx_checksum(call)
            moved = ctx.stats()["h2d_bytes"] - s0["h2d_bytes"]
            assert frame_bytes * 0.9 <= moved <= 1.3 * frame_bytes + (1 << 20), (moved, frame_bytes)
            assert [bytes(v) for v in views] == [bytes(w) for w in want]
            # packets: each frame's L4 segment (the seed as tx_fill's TCP / ICMP)
            seg = [call[i][34:] for i in range(len(call))]
            seeds = [0] * len(seg)
            ref = np.array([pyoracle.checksum(bytes(p) or b"\0", len(p), 0) for p in seg], np.uint16)
            s0 = ctx.stats()
            assert np.array_equal(ctx.batch_host(seg, seeds), ref)
            moved = ctx.stats()["h2d_bytes"] - s0["h2d_bytes"]
            assert moved <= 1.3 * frame_bytes + (1 << 20), (moved, frame_bytes)
            d = np.zeros(len(seg), dtype=lvlip.DESC_DTYPE)
            d["offset"] = fd["offset"][perm] + 34
            d["len"] = fd["len"][perm] - 34
            s0 = ctx.stats()
            assert np.array_equal(ctx.batch_host_flat(buf, d), ref)
            moved = ctx.stats()["h2d_bytes"] - s0["h2d_bytes"]
            assert moved <= 1.3 * frame_bytes + (1 << 20), (moved, frame_bytes)
        finally:
            ctx.unregister(buf)


@pytest.mark.parametrize("inline_max", ["0", "32768"])
def test_inline_and_pool_host_steps_agree(inline_max, monkeypatch):
    """LVLIP_INLINE_MAX: the same 20 000 frames and 40 000 packets with every
    host step on the pool threads (0) and on the calling thread (the default,
    calls of up to 32 768 items): the same fills, verdicts and checksums, equal
    to the oracle, from plain memory and from a registered slab."""
    monkeypatch.setenv("LVLIP_INLINE_MAX", inline_max)
    fr = workloads.frames(20000, seed=150, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    buf, fd, views, perm = _slab(fr)
    with lvlip.Context(0, arena_bytes=4 << 20, cpu_max=0) as ctx:
        scattered = [bytearray(f) for f in fr]
        ctx.tx_checksum(scattered)
        assert [bytes(f) for f in scattered] == [bytes(w) for w in want]
        ctx.register(buf, lvlip.REG_DMA)
        try:
            ctx.tx_checksum(views)
            assert [bytes(v) for v in views] == [bytes(w) for w in want]
            for flags in (0, lvlip.RX_VERIFY_L4):
                v = ctx.rx_verify(views, flags)
                assert v.tolist() == [skb_oracle.rx_verdict(bytes(w), flags) for w in want], flags
        finally:
            ctx.unregister(buf)
        seg = [bytes(w[14:]) for w in want] * 2
        got = ctx.batch_host(seg, [0] * len(seg))
        ref = np.array([pyoracle.checksum(s or b"\0", len(s), 0) for s in seg], np.uint16)
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("ratio", ["2", "3"])
def test_span_ratio_moves_half_full_granules(ratio, monkeypatch):
    """LVLIP_SPAN_RATIO: frames each in its own 1 792-B granule of a
    registered DMA slab (level-ip's RX skbs: BUFLEN 1 600 rounded to 256 B),
    ~2.2x their bytes.  Ratio 2 (the default) gathers them (h2d bytes about
    the frames' own); ratio 3 moves the granules as spans (h2d bytes about
    the slab's).  The fills equal the oracle either way."""
    monkeypatch.setenv("LVLIP_SPAN_RATIO", ratio)
    fr = workloads.frames(4096, seed=160, max_l4=1460)
    fr = [f for f in fr if len(f) <= 1000][:2048]  # at most 1 000 B each, ~530 B on average
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    gran = 1792
    buf = np.zeros(gran * len(fr) + 64, dtype=np.uint8)
    views = []
    for i, f in enumerate(fr):
        o = i * gran + 14  # skb->data at head + 14: the frame from head
        buf[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        views.append(buf[o:o + len(f)])
    frame_bytes = sum(len(f) for f in fr)
    span = gran * len(fr)
    assert span > 2 * frame_bytes + (1 << 20) and span < 3 * frame_bytes + (1 << 20)
    with lvlip.Context(0, cpu_max=0) as ctx:
        ctx.register(buf, lvlip.REG_DMA)
        try:
            s0 = ctx.stats()
            ctx.tx_checksum(views)
            moved = ctx.stats()["h2d_bytes"] - s0["h2d_bytes"]
        finally:
            ctx.unregister(buf)
    assert [bytes(v) for v in views] == [bytes(w) for w in want]
    if ratio == "2":
        assert moved < 1.3 * frame_bytes, (moved, frame_bytes)
    else:
        assert 0.9 * span < moved < 1.1 * span, (moved, span)


@pytest.mark.parametrize("warm", ["0", "1048576"])
def test_context_without_and_with_copy_engine_warmup(warm, monkeypatch):
    """LVLIP_WARM_BYTES: a context made with no copy-engine warm-up (0) and
    with the default's; a call of several pieces (the later ones through the
    copy engine) fills the frames as the oracle does either way."""
    monkeypatch.setenv("LVLIP_WARM_BYTES", warm)
    fr = workloads.frames(6000, seed=170, max_l4=1460)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    got = [bytearray(f) for f in fr]
    with lvlip.Context(0, arena_bytes=1 << 20, cpu_max=0) as ctx:
        ctx.tx_checksum(got)
        assert ctx.stats()["pieces"] >= 3
    assert [bytes(f) for f in got] == [bytes(w) for w in want]
