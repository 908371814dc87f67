"""The TX batch-and-dispatch path in running code (north_star: "src/ip_output.c
and src/tcp.c ... gain an optional batch-and-dispatch path over skbuff lists";
INTEGRATION.md §2a), on level-ip's own TX code.

tests/ref_tx_batch_child.py drives the reference stack twice, each in a fresh
process: as it is (oracle/_ref/libref_fixclock.so: every TX checksum on the
CPU at tcp_transmit_skb, src/tcp_output.c:126, icmpv4_reply, src/icmpv4.c:47,
and ip_output, src/ip_output.c:53), and with the batch step
(oracle/_ref/libref_txq.so: those three deferred, ip_output's frame queued,
each flush ONE lvlip_tx_checksum_skb_list over the queue, then the real
dst_neigh_output per skb).  The frames written to the tap must be identical,
frame for frame: SYN with options, the SYN retransmit, 536/536/536/393-B data
segments, ACK, RST, and the echo replies to every ip_rcv case.

Skipped when oracle/_ref was not built (it needs /root/reference at build time)."""
import json
import os
import subprocess
import sys

import pytest

import golden_io
import ref_rx_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXCLOCK = os.path.join(ROOT, "oracle", "_ref", "libref_fixclock.so")
TXQ = os.path.join(ROOT, "oracle", "_ref", "libref_txq.so")

pytestmark = pytest.mark.skipif(not (os.path.exists(FIXCLOCK) and os.path.exists(TXQ)),
                                reason="oracle/_ref/libref_{fixclock,txq}.so not built")


def _requests():
    """Config #1's echo requests (tests/golden/echo.json) and 8 echo requests
    of every ip_rcv case (tests/ref_rx_cases.py: options, bad header
    checksum, bad version / ihl, TTL 0, unknown protocol, bad ICMP checksum)."""
    frs, _ = ref_rx_cases.frames(17, per_kind=8)
    return [c["request_hex"] for c in golden_io.echo()["echo"]] + [bytes(f).hex() for f in frs]


def _run(tmp_path, lib, mode):
    req = tmp_path / "req.json"
    if not req.exists():
        req.write_text(json.dumps(_requests()))
    out = tmp_path / f"{mode}.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_tx_batch_child.py"), str(req), str(out),
                    lib, mode], check=True, stdin=subprocess.DEVNULL, timeout=180)
    return json.loads(out.read_text())


def _check_same(base, got):
    assert len(got["frames"]) == len(base["frames"])
    bad = [i for i, (x, y) in enumerate(zip(base["frames"], got["frames"])) if x != y]
    assert not bad, bad[:5]
    # ARP reply, 8 TCP frames, then one reply per answered request
    assert len(base["frames"]) > 1 + 8 + 4
    assert got["batches"][0] == 8
    # every batched frame deferred two CPU checksum computations (TCP or ICMP,
    # and the IPv4 header)
    assert got["deferred"] == [2 * k for k in got["batches"]]


def test_tx_batch_oracle_fill_matches_unbatched_stack(tmp_path):
    """CPU: the composition with the queue filled by the oracle (the
    harness's own check without a GPU)."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    _check_same(base, _run(tmp_path, TXQ, "oracle"))
    # the fixed clock makes two unbatched runs identical (what the
    # frame-for-frame comparison relies on)
    assert _run(tmp_path, FIXCLOCK, "unbatched")["frames"] == base["frames"]


@pytest.mark.gpu
def test_tx_batch_gpu_fill_matches_unbatched_stack(tmp_path):
    """GPU: each flush is one lvlip_tx_checksum_skb_list over the queued skbs;
    the tap bytes equal the unbatched stack's, frame for frame."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    _check_same(base, _run(tmp_path, TXQ, "gpu"))
