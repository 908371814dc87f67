"""The optional batch-and-dispatch RX path (BASELINE.json
north_star: src/ip_input.c "gains an optional batch-and-dispatch path over
skbuff lists") composed with level-ip's own RX code, run in running code
rather than described.

tests/ref_rx_batch_child.py drives the reference stack compiled from its own
sources (oracle/_ref/libref.so) over a socketpair tap: the same frames once as
level-ip handles them (each skb straight into netdev_receive -> ip_rcv) and
once batched (all skbs in one sk_buff_head, ONE lvlip_rx_verify_skb_list on
the GPU, then ip_rcv only for LVLIP_RX_OK, arp_rcv for the ARP frame, free_skb
for the rest).  The frames: an ARP request, then echo requests of every
ip_rcv decision (good, IP options, corrupted header checksum, bad version,
ihl < 5, TTL 0, unknown protocol, corrupted ICMP checksum; ref_rx_cases.py).
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

import lvlip
import ref_rx_cases

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = os.path.join(HERE, "ref_rx_batch_child.py")
ARP = (b"\xff" * 6 + ref_rx_cases.TAP_MAC + b"\x08\x06" + bytes.fromhex("0001080006040001") +
       ref_rx_cases.TAP_MAC + ref_rx_cases.TAP_IP + bytes(6) + ref_rx_cases.STACK_IP)

needs_ref = pytest.mark.skipif(not os.path.exists(ref_rx_cases.REF_SO), reason="oracle/_ref/libref.so not built")


REF_RXQ = os.path.join(os.path.dirname(ref_rx_cases.REF_SO), "libref_rxq.so")


def _run(frames, mode, so=ref_rx_cases.REF_SO, cpu_max="0"):
    """cpu_max: the context's LVLIP_CPU_MAX in the child (None: unset, the
    library's default threshold, under which these queues of ~100-200 skbs
    are verified on the calling thread; "0": on the GPU)."""
    env = {k: v for k, v in os.environ.items() if k != "LVLIP_CPU_MAX"}
    if cpu_max is not None:
        env["LVLIP_CPU_MAX"] = cpu_max
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "f.json"), os.path.join(d, "o.json")
        with open(fin, "w") as f:
            json.dump([bytes(x).hex() for x in frames], f)
        r = subprocess.run([sys.executable, CHILD, fin, fout, so, mode],
                           stdin=subprocess.DEVNULL, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        with open(fout) as f:
            return json.load(f)


def _frames(seed, per_kind):
    frs, kinds = ref_rx_cases.frames(seed, per_kind)
    return [ARP] + frs, ["arp"] + kinds


def _check(frames, kinds, mode, cpu_max="0"):
    ref = _run(frames, "unbatched")
    got = _run(frames, mode, cpu_max=cpu_max)
    # the ARP reply, then one echo reply per accepted request
    assert ref["replies"][0] is not None and got["replies"][0] == ref["replies"][0]
    answered = {k for k, r in zip(kinds, ref["replies"]) if r is not None}
    assert answered == {"arp", "ok", "ok_options", "icmp_csum"}, answered
    return ref, got


@needs_ref
def test_batched_rx_composition_with_oracle_verdicts():
    """The composition itself, with the CPU oracle's verdicts in place of the
    GPU (harness check on any machine): level-ip's replies are byte-identical,
    frame for frame, and the frames it drops are exactly the frames ip_rcv
    drops on its own."""
    frames, kinds = _frames(81, 12)
    ref, got = _check(frames, kinds, "oracle")
    assert got["replies"] == ref["replies"]
    dropped = [v not in (lvlip.RX_OK, lvlip.RX_NOT_IP) for v in got["verdicts"]]
    assert dropped == [r is None for r in ref["replies"]]


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("cpu_max", ["0", None])
def test_batched_rx_through_reference_stack_on_gpu(cpu_max):
    """VERDICT r03 Next #3: one lvlip_rx_verify_skb_list over the queue (on
    the GPU with threshold 0; on the calling thread with the library's default
    threshold, VERDICT r05 Next #1), then level-ip's own ip_rcv ->
    icmpv4_reply -> ip_output for the accepted skbs only.  The replies on the
    tap are byte-identical to the unbatched reference run on the same frames,
    and the dropped set equals what ip_rcv itself drops (src/ip_input.c:22-43,
    :51-60)."""
    frames, kinds = _frames(82, 24)
    ref, got = _check(frames, kinds, "batched", cpu_max)
    assert got["replies"] == ref["replies"]
    dropped = [v not in (lvlip.RX_OK, lvlip.RX_NOT_IP) for v in got["verdicts"]]
    assert dropped == [r is None for r in ref["replies"]]
    by_kind = {}
    for k, v in zip(kinds, got["verdicts"]):
        by_kind.setdefault(k, set()).add(v)
    assert by_kind["arp"] == {lvlip.RX_NOT_IP}
    assert by_kind["ip_csum"] == {lvlip.RX_BAD_CSUM} and by_kind["ttl0"] == {lvlip.RX_TTL0}
    assert by_kind["version"] == {lvlip.RX_BAD_VERSION} and by_kind["ihl"] == {lvlip.RX_BAD_IHL}
    assert by_kind["proto"] == {lvlip.RX_UNKNOWN_PROTO}


@pytest.mark.gpu
@needs_ref
def test_batched_rx_with_l4_verify_drops_corrupted_icmp():
    """With LVLIP_RX_VERIFY_L4 the batch also drops the echo requests whose
    ICMP checksum is corrupted, which level-ip answers (it never verifies ICMP
    on RX, src/icmpv4.c:11); every other frame's outcome and reply is the
    reference's."""
    frames, kinds = _frames(83, 16)
    ref, got = _check(frames, kinds, f"batched:{lvlip.RX_VERIFY_L4}")
    for k, r, g, v in zip(kinds, ref["replies"], got["replies"], got["verdicts"]):
        if k == "icmp_csum":
            assert r is not None and g is None and v == lvlip.RX_BAD_L4
        else:
            assert g == r, k


def _gated(mode):
    """The composition on libref_rxq.so, where ip_rcv's header checksum
    (src/ip_input.c:38) takes the batch's verdict for accepted frames
    (INTEGRATION.md §2b's one-line change, made at link level): per accepted
    frame, the CPU header sums the batch removes."""
    frames, kinds = _frames(84, 12)
    ref = _run(frames, "unbatched", REF_RXQ)
    got = _run(frames, mode, REF_RXQ)
    assert got["replies"] == ref["replies"]
    accepted = sum(v == lvlip.RX_OK for v in got["verdicts"])
    # unbatched: ip_rcv sums the header of every IPv4 frame that passes the
    # version / ihl / TTL checks (ok, options, bad checksum, unknown protocol,
    # bad ICMP checksum: 5 of the 8 kinds)
    reaching = sum(k in ("ok", "ok_options", "ip_csum", "proto", "icmp_csum") for k in kinds)
    assert ref["cpu_header_sums"] == reaching and ref["batch_header_sums"] == 0
    # batched: the rejected frames never reach ip_rcv, the accepted ones take
    # the batch's result: no header is summed on the CPU
    assert got["cpu_header_sums"] == 0 and got["batch_header_sums"] == accepted > 0
    return ref, got


@pytest.mark.skipif(not os.path.exists(REF_RXQ), reason="oracle/_ref/libref_rxq.so not built")
def test_gated_ip_rcv_takes_batch_verdicts_oracle():
    """CPU: the gated composition with the oracle's verdicts."""
    _gated("oracle")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_RXQ), reason="oracle/_ref/libref_rxq.so not built")
def test_gated_ip_rcv_takes_batch_verdicts_gpu():
    """GPU: one lvlip_rx_verify_skb_list, then ip_rcv with :38 answered by the
    batch; replies identical to the unbatched stack, zero CPU header sums."""
    _gated("batched")
