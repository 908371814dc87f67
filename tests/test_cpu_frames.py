"""The context-free CPU frame calls (include/lvlip_skb.h: lvlip_rx_verify_cpu,
lvlip_tx_checksum_cpu and their _skb_list forms).  They are what a context runs
for calls of at most its cpu_max frames, and what a caller that deferred its TX
checksums falls back to when the GPU call fails.  No GPU:
checked here against the oracle (oracle/skb_oracle.py over the pinned checksum
oracle) and the reference stack's own frames (tests/golden/echo.json,
tcp_frames.json); test_dispatch_gpu.py checks that both sides of a context's
threshold give the same bytes."""
import ctypes

import numpy as np
import pytest

import golden_io
import lvlip
import skb_oracle
import workloads
from test_skb_cpu import _rx_cases, _scrambled_tcp_frames
from test_skb_list import BUFLEN, Queue, _ref


def test_tx_cpu_matches_reference_tx():
    fr = workloads.frames(400, seed=31)
    want = [bytearray(f) for f in fr]
    for f in want:
        skb_oracle.tx_fill(f)
    lvlip.tx_checksum_cpu(fr)
    assert [bytes(f) for f in fr] == [bytes(f) for f in want]


def test_tx_cpu_reference_stack_frames():
    """The frames level-ip's TCP transmit path and icmpv4_reply wrote, their
    checksum fields scrambled, refilled == the reference's bytes."""
    fr, want = _scrambled_tcp_frames()
    lvlip.tx_checksum_cpu(fr)
    assert [bytes(f) for f in fr] == want
    e = golden_io.echo()["echo"]
    rep = []
    for case in e:
        r = bytearray(bytes.fromhex(case["reply_hex"]))
        r[24:26], r[36:38] = b"\xde\xad", b"\xbe\xef"
        rep.append(r)
    lvlip.tx_checksum_cpu(rep)
    assert [bytes(f) for f in rep] == [bytes.fromhex(c["reply_hex"]) for c in e]


def test_tx_cpu_any_prior_field_value_and_aliases():
    """Whatever the fields held, and a frame listed twice: the same bytes as
    one reference fill (the seed compensation makes a second pass a no-op)."""
    base = workloads.frames(16, seed=32, max_l4=300)
    for v in (b"\0\0", b"\xff\xff", b"\x12\x34"):
        fr = [bytearray(f) for f in base]
        for f in fr:
            ihl = f[14] & 0xF
            f[24:26] = v
            off = 14 + ihl * 4 + (16 if f[23] == 6 else 2)
            f[off:off + 2] = v
        want = [bytearray(f) for f in fr]
        for f in want:
            skb_oracle.tx_fill(f)
        lvlip.tx_checksum_cpu(fr + fr[:5])
        assert [bytes(f) for f in fr] == [bytes(f) for f in want]


def test_tx_cpu_malformed_leaves_batch_untouched():
    good = workloads.frames(6, seed=33, max_l4=200)
    for k, damage in enumerate(("version", "short", "trunc", "ihl")):
        fr = [bytearray(f) for f in good]
        j = (k + 1) % len(fr)
        if damage == "version":
            fr[j][14] = 0x65
        elif damage == "short":
            fr[j] = fr[j][:30]
        elif damage == "trunc":
            fr[j] = fr[j][:14 + int.from_bytes(fr[j][16:18], "big") - 1]
        else:
            fr[j][14] = 0x44
        before = [bytes(f) for f in fr]
        with pytest.raises(lvlip.LvlipError) as e:
            lvlip.tx_checksum_cpu(fr)
        assert e.value.rc == lvlip.EINVAL
        assert [bytes(f) for f in fr] == before, damage


def test_rx_cpu_matches_ip_rcv():
    fr = _rx_cases(34)
    before = [bytes(f) for f in fr]
    seen = set()
    for flags in (0, lvlip.RX_VERIFY_L4):
        got = lvlip.rx_verify_cpu(fr, flags).tolist()
        assert got == [skb_oracle.rx_verdict(f, flags) for f in fr], flags
        seen |= set(got)
    assert [bytes(f) for f in fr] == before
    assert seen >= set(range(1, 10)), seen


def test_rx_cpu_echo_requests_and_tcp_frames_ok():
    fr = [bytearray(bytes.fromhex(c["request_hex"])) for c in golden_io.echo()["echo"]]
    fr += [bytearray(f) for f in golden_io.tcp_frames()]
    for flags in (0, lvlip.RX_VERIFY_L4):
        assert lvlip.rx_verify_cpu(fr, flags).tolist() == [lvlip.RX_OK] * len(fr)


def test_cpu_frame_calls_empty_and_bad_arguments():
    L = lvlip.lib()
    assert L.lvlip_rx_verify_cpu(None, 0, 0, None) == lvlip.OK
    assert L.lvlip_tx_checksum_cpu(None, 0) == lvlip.OK
    assert L.lvlip_rx_verify_cpu(None, 1, 0, None) == lvlip.EINVAL
    assert L.lvlip_tx_checksum_cpu(None, 1) == lvlip.EINVAL
    fp = ctypes.cast(ctypes.create_string_buffer(64), ctypes.POINTER(lvlip.Frame))
    assert L.lvlip_tx_checksum_cpu(fp, 0xFFFFFFF0 // 2 + 1) == lvlip.EINVAL
    assert L.lvlip_rx_verify_skb_list_cpu(None, 0, None, 0) == lvlip.EINVAL
    assert L.lvlip_tx_checksum_skb_list_cpu(None) == lvlip.EINVAL


def test_skb_list_cpu_forms():
    """The _skb_list_cpu walkers over skbs made by the reference's own
    skbuff.c (test_skb_list.py's shapes): TX fills what the reference
    computes, RX gives ip_rcv's verdicts on skb->data .. skb->end; an empty
    queue is 0 frames; more skbs than cap is LVLIP_ERANGE."""
    ref = _ref()
    L = lvlip.lib()
    tx = workloads.frames(40, seed=35, max_l4=1460)
    q = Queue()
    for f in tx:
        body = bytes(f[14:])
        skb = ref.alloc_skb(14 + len(body) + 16)
        ref.skb_reserve(skb, 14 + len(body))
        ref.skb_push(skb, len(body))
        ctypes.memmove(skb.contents.data, body, len(body))
        q.tail(skb)
    want = [bytearray(f) for f in tx]
    for w in want:
        skb_oracle.tx_fill(w)
    assert L.lvlip_tx_checksum_skb_list_cpu(q.ptr()) == len(tx)
    assert [ctypes.string_at(s.contents.data, s.contents.len) for s in q.skbs] == [bytes(w[14:]) for w in want]

    rx = _rx_cases(36)[:60]
    q2 = Queue()
    for f in rx:
        skb = ref.alloc_skb(BUFLEN)
        ctypes.memmove(skb.contents.data, bytes(f), len(f))
        q2.tail(skb)
    bufs = [ctypes.string_at(s.contents.data, BUFLEN) for s in q2.skbs]
    v = np.zeros(len(rx), np.uint8)
    for flags in (0, lvlip.RX_VERIFY_L4):
        assert L.lvlip_rx_verify_skb_list_cpu(q2.ptr(), flags, v.ctypes.data, len(rx)) == len(rx)
        assert v.tolist() == [skb_oracle.rx_verdict(b, flags) for b in bufs], flags
    assert L.lvlip_rx_verify_skb_list_cpu(q2.ptr(), 0, v.ctypes.data, len(rx) - 1) == lvlip.ERANGE
    assert L.lvlip_tx_checksum_skb_list_cpu(Queue().ptr()) == 0
    assert [ctypes.string_at(s.contents.data, BUFLEN) for s in q2.skbs] == bufs
    for s in q.skbs + q2.skbs:
        ref.free_skb(s)


# ------------------------------------------------- property-based (hypothesis) --

from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

SETTINGS = settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@st.composite
def _frame(draw):
    """A frame whose header fields hypothesis picks from the values that steer
    ip_rcv's decisions (ethertype, version, ihl, TTL, protocol, total length
    against the frame's length), over random bytes, with random checksum
    fields (valid or not)."""
    body = bytearray(draw(st.binary(min_size=0, max_size=1600)))
    f = bytearray(14) + body
    if len(f) >= 14:
        f[12:14] = draw(st.sampled_from([b"\x08\x00", b"\x08\x00", b"\x08\x06", b"\x86\xdd"]))
    if len(f) >= 34:
        ver = draw(st.sampled_from([4, 4, 4, 6]))
        ihl = draw(st.integers(0, 15))
        f[14] = (ver << 4) | ihl
        f[22] = draw(st.sampled_from([0, 1, 64, 255]))
        f[23] = draw(st.sampled_from([1, 6, 6, 17]))
        iplen = draw(st.one_of(st.just(len(f) - 14), st.integers(0, 0xFFFF)))
        f[16:18] = iplen.to_bytes(2, "big")
        # valid fields where the frame holds the packet its header describes
        if draw(st.booleans()) and 20 <= ihl * 4 <= iplen <= len(f) - 14:
            g = bytearray(f)
            try:
                skb_oracle.tx_fill(g)
                f = g
            except (IndexError, ValueError, struct_error):
                pass
    return f


struct_error = __import__("struct").error


@SETTINGS
@given(frames=st.lists(_frame(), min_size=0, max_size=24), flags=st.sampled_from([0, lvlip.RX_VERIFY_L4]))
def test_rx_cpu_property(frames, flags):
    """lvlip_rx_verify_cpu == the oracle's ip_rcv restatement on any frames."""
    got = lvlip.rx_verify_cpu(frames, flags).tolist()
    assert got == [skb_oracle.rx_verdict(bytes(f), flags) for f in frames]


@SETTINGS
@given(frames=st.lists(_frame(), min_size=1, max_size=24))
def test_tx_cpu_property(frames):
    """lvlip_tx_checksum_cpu: the oracle's fill on every frame when all are
    well formed (tx_plan's rule), else LVLIP_EINVAL with every frame as it
    was."""
    before = [bytes(f) for f in frames]
    ok = lvlip.tx_plan([bytearray(f) for f in frames]) is not None
    if ok:
        lvlip.tx_checksum_cpu(frames)
        want = [bytearray(b) for b in before]
        for w in want:
            skb_oracle.tx_fill(w)
        assert [bytes(f) for f in frames] == [bytes(w) for w in want]
    else:
        with pytest.raises(lvlip.LvlipError) as e:
            lvlip.tx_checksum_cpu(frames)
        assert e.value.rc == lvlip.EINVAL and [bytes(f) for f in frames] == before
