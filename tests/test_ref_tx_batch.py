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


def _run(tmp_path, lib, mode, opts=None, env=None, tag=None):
    req = tmp_path / "req.json"
    if not req.exists():
        req.write_text(json.dumps(_requests()))
    out = tmp_path / f"{tag or mode}.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_tx_batch_child.py"), str(req), str(out),
                    lib, mode, json.dumps(opts or {})], check=True, stdin=subprocess.DEVNULL, timeout=300,
                   env=env)
    got = json.loads(out.read_text())
    got["hold"] = bool((opts or {}).get("hold"))
    return got


def _env(cpu_max=None, **extra):
    """The child's environment: LVLIP_CPU_MAX as given (None: unset, the
    library's default threshold), plus extra variables."""
    env = {k: v for k, v in os.environ.items() if k not in ("LVLIP_CPU_MAX", "LVLIP_FAIL_PIECE")}
    if cpu_max is not None:
        env["LVLIP_CPU_MAX"] = str(cpu_max)
    env.update({k: str(v) for k, v in extra.items()})
    return env


def _check_same(base, got, first_batch=8):
    assert len(got["frames"]) == len(base["frames"])
    bad = [i for i, (x, y) in enumerate(zip(base["frames"], got["frames"])) if x != y]
    assert not bad, bad[:5]
    # ARP reply, the TCP frames, then one reply per answered request
    assert len(base["frames"]) > 1 + 8 + 4
    # holding: the SYN went out early, when tcp_send_next's skb_reset_header
    # was about to rewrite it (the flush before a retransmit)
    early = got["early_frames"]
    assert got["reheld"] == 0 and early == (1 if got.get("hold") else 0)
    assert got["batches"][0] == first_batch - early
    # every batched frame deferred two CPU checksum computations (TCP or ICMP,
    # and the IPv4 header)
    assert sum(got["deferred"]) == 2 * (sum(got["batches"]) + early) or any(r["dropped"] for r in got["reports"])


def test_tx_batch_oracle_fill_matches_unbatched_stack(tmp_path):
    """CPU: the composition with the queue filled by the oracle (the
    harness's own check without a GPU)."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    _check_same(base, _run(tmp_path, TXQ, "oracle"))
    # the fixed clock makes two unbatched runs identical (what the
    # frame-for-frame comparison relies on)
    assert _run(tmp_path, FIXCLOCK, "unbatched", tag="unbatched2")["frames"] == base["frames"]


@pytest.mark.gpu
def test_tx_batch_gpu_fill_matches_unbatched_stack(tmp_path):
    """Each flush is one lvlip_txq_fill (lvlip_tx_checksum_skb_list through a
    context) over the queued skbs; the tap bytes equal the unbatched stack's,
    frame for frame, with the library's default threshold (both flushes, 8
    and 28 frames, are summed on the calling thread) and with threshold 0
    (both on the GPU)."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    dflt = _run(tmp_path, TXQ, "gpu", env=_env(None), tag="default")
    _check_same(base, dflt)
    assert [(r["cpu_calls"], r["gpu_calls"]) for r in dflt["reports"]] == [(1, 0), (1, 0)]
    gpu = _run(tmp_path, TXQ, "gpu", env=_env(0), tag="gpu0")
    _check_same(base, gpu)
    assert [(r["cpu_calls"], r["gpu_calls"]) for r in gpu["reports"]] == [(0, 1), (0, 1)]
    assert not any(r["cpu"] or r["dropped"] for r in dflt["reports"] + gpu["reports"])


def test_tx_batch_no_context_fills_on_cpu(tmp_path):
    """VERDICT r05 Next #2: when the context cannot be made (an invalid device
    index, or no GPU at all: lvlip_csum_ctx_create says LVLIP_ENODEV) the
    flush fills the queue with the library's CPU code, so no frame leaves with
    a deferred, still-zero field: the tap bytes equal the unbatched stack's.
    Runs here and on the GPU box alike."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    got = _run(tmp_path, TXQ, "gpu", {"device": 99}, env=_env(0), tag="nodev")
    assert got["context_error"] == -2  # LVLIP_ENODEV
    _check_same(base, got)
    assert [(r["rc"], r["cpu"], r["dropped"]) for r in got["reports"]] == [(-2, 1, 0)] * 2


@pytest.mark.gpu
def test_tx_batch_gpu_error_fills_on_cpu(tmp_path):
    """The GPU call fails (LVLIP_FAIL_PIECE=1: the first piece of every GPU
    call returns LVLIP_EHIP, after which the call has restored any field it
    stored): the flush fills the queue on the CPU and the tap bytes equal the
    unbatched stack's."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    got = _run(tmp_path, TXQ, "gpu", env=_env(0, LVLIP_FAIL_PIECE=1), tag="hiperr")
    _check_same(base, got)
    assert [(r["rc"], r["cpu"], r["dropped"], r["gpu_calls"]) for r in got["reports"]] == [(-3, 1, 0, 1)] * 2


@pytest.mark.gpu
@pytest.mark.parametrize("cpu_max", [None, 0])
def test_tx_batch_malformed_frame_untouched_and_dropped(tmp_path, cpu_max):
    """A malformed frame (IPv4 version 6) in the queue: the batch call refuses
    it with LVLIP_EINVAL and leaves every queued byte as it was; the flush then
    drops that frame (reported) and fills the rest on the CPU; the tap bytes
    equal the unbatched stack's, which never had the frame."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    got = _run(tmp_path, TXQ, "gpu", {"inject": True}, env=_env(cpu_max), tag=f"inject{cpu_max}")
    assert got["untouched"] == {"rc": -1, "same": True}
    _check_same(base, got, first_batch=8)
    assert got["reports"][0]["dropped"] == 1 and got["reports"][0]["cpu"] == 1
    assert got["reports"][1]["dropped"] == 0


SCALE = {"write_bytes": 12 << 20, "send_next": 0, "hashes": True}


@pytest.mark.gpu
def test_tx_batch_at_scale(tmp_path):
    """VERDICT r05 Next #3: a 12 MiB tcp_send (23 476 segments at level-ip's
    smss of 536, src/tcp.c:115) sent by one tcp_send_next, plus the echo
    replies: ~14 MB of frames in the first flush, more than the 4 MiB first
    piece, so the GPU call runs several pieces through the reference's own TX
    objects.  The tap bytes (23 000+ frames, compared by digest) equal the
    unbatched stack's with the default threshold (the flush goes to the GPU:
    it is above cpu_max) and with threshold 0; with a malformed frame injected
    the batch call leaves the whole queue untouched, and the flush drops that
    frame and fills the rest."""
    base = _run(tmp_path, FIXCLOCK, "unbatched", SCALE)
    n_tcp = 1 + 2 + (SCALE["write_bytes"] + 535) // 536 + 2  # ARP reply, SYN x2, data, ACK, RST
    assert len(base["frames"]) > n_tcp
    for cpu_max in (None, 0):
        got = _run(tmp_path, TXQ, "gpu", SCALE, env=_env(cpu_max), tag=f"scale{cpu_max}")
        _check_same(base, got, first_batch=n_tcp - 1)
        r = got["reports"][0]
        assert (r["gpu_calls"], r["cpu_calls"], r["cpu"]) == (1, 0, 0) and r["pieces"] >= 2, r
    got = _run(tmp_path, TXQ, "gpu", dict(SCALE, inject=True), env=_env(None), tag="scale_inject")
    assert got["untouched"] == {"rc": -1, "same": True}
    assert got["frames"] == base["frames"]
    assert got["reports"][0]["dropped"] == 1


# --- holding the skbs by reference instead of copying them (oracle/ref_txq.c) ---

HOLD = {"hold": True}


def test_tx_batch_hold_oracle_fill_matches_unbatched_stack(tmp_path):
    """CPU: the queue holds each skb itself (its refcnt raised, so the
    caller's free_skb is a no-op; no copy), the oracle fills the held frames,
    the flush sends and releases them, and the SYN the stack retransmits is
    sent before skb_reset_header rewrites it.  The tap bytes equal the
    unbatched stack's."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    _check_same(base, _run(tmp_path, TXQ, "oracle", HOLD, tag="hold_oracle"))


def test_tx_batch_hold_no_context_fills_on_cpu(tmp_path):
    """CPU: held frames, no context: every flush (the early one before the SYN
    retransmit included) fills on the CPU, same tap bytes."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    got = _run(tmp_path, TXQ, "gpu", dict(HOLD, device=99), env=_env(0), tag="hold_nodev")
    _check_same(base, got)
    assert [(r["rc"], r["cpu"], r["dropped"]) for r in got["reports"]] == [(-2, 1, 0)] * 2


@pytest.mark.gpu
@pytest.mark.parametrize("cpu_max", [None, 0])
def test_tx_batch_hold_gpu_fill_matches_unbatched_stack(tmp_path, cpu_max):
    """Held frames filled by ONE lvlip_tx_checksum per flush (the frame-array
    call over {data - 14, len + 14}): on the calling thread with the default
    threshold, on the GPU with 0; tap bytes identical.  With a malformed frame
    injected the call refuses the array untouched and the flush drops it."""
    base = _run(tmp_path, FIXCLOCK, "unbatched")
    got = _run(tmp_path, TXQ, "gpu", HOLD, env=_env(cpu_max), tag=f"hold{cpu_max}")
    _check_same(base, got)
    want = (0, 1) if cpu_max == 0 else (1, 0)
    assert [(r["cpu_calls"], r["gpu_calls"]) for r in got["reports"]] == [want] * 2
    assert not any(r["cpu"] or r["dropped"] for r in got["reports"])
    got = _run(tmp_path, TXQ, "gpu", dict(HOLD, inject=True), env=_env(cpu_max), tag=f"hold_inject{cpu_max}")
    assert got["untouched"] == {"rc": -1, "same": True}
    _check_same(base, got)
    assert got["reports"][0]["dropped"] == 1 and got["reports"][1]["dropped"] == 0


@pytest.mark.gpu
def test_tx_batch_hold_at_scale(tmp_path):
    """The 12 MiB tcp_send with the skbs held: the flush's 23 000+ frames are
    the write queue's own skbs (no copy), filled by one multi-piece GPU call
    (threshold 0 and the default) or, when the call fails (LVLIP_FAIL_PIECE),
    on the CPU; tap bytes identical, and the write queue keeps its skbs
    (nothing freed twice: the run ends cleanly)."""
    base = _run(tmp_path, FIXCLOCK, "unbatched", SCALE)
    n_tcp = 1 + 2 + (SCALE["write_bytes"] + 535) // 536 + 2
    for cpu_max, extra in ((None, {}), (0, {}), (0, {"LVLIP_FAIL_PIECE": 1})):
        got = _run(tmp_path, TXQ, "gpu", dict(SCALE, hold=True), env=_env(cpu_max, **extra),
                   tag=f"hold_scale{cpu_max}{len(extra)}")
        _check_same(base, got, first_batch=n_tcp - 1)
        r = got["reports"][0]
        # the injected failure stops the call at its first piece
        assert r["gpu_calls"] == 1 and r["pieces"] >= (1 if extra else 2) and r["cpu"] == (1 if extra else 0), r


TXQ_SLAB = os.path.join(ROOT, "oracle", "_ref", "libref_txq_slab.so")
FIXCLOCK_SLAB = os.path.join(ROOT, "oracle", "_ref", "libref_fixclock_slab.so")
SLAB = {"slab": 1 << 28}


@pytest.mark.skipif(not (os.path.exists(TXQ_SLAB) and os.path.exists(FIXCLOCK_SLAB)),
                    reason="oracle/_ref/libref_{txq,fixclock}_slab.so not built")
def test_tx_batch_slab_hold_oracle(tmp_path):
    """CPU: every skb buffer from one slab (oracle/ref_slab.c) on both sides,
    the TX frames held and filled by the oracle: the tap bytes equal the
    unbatched stack's (with the same slab, and without it)."""
    base = _run(tmp_path, FIXCLOCK_SLAB, "unbatched", SLAB, tag="unbatched_slab")
    assert base["frames"] == _run(tmp_path, FIXCLOCK, "unbatched", tag="unbatched_plain")["frames"]
    _check_same(base, _run(tmp_path, TXQ_SLAB, "oracle", dict(SLAB, hold=True), tag="slab_hold_oracle"))


@pytest.mark.gpu
@pytest.mark.skipif(not (os.path.exists(TXQ_SLAB) and os.path.exists(FIXCLOCK_SLAB)),
                    reason="oracle/_ref/libref_{txq,fixclock}_slab.so not built")
def test_tx_batch_slab_hold_at_scale(tmp_path):
    """The 12 MiB tcp_send with every skb buffer in one registered slab and
    the frames held: one GPU call moves the write queue's segments as spans
    (their 768-B granules are dense, in order), tap bytes identical."""
    base = _run(tmp_path, FIXCLOCK_SLAB, "unbatched", dict(SCALE, **SLAB), tag="unb_slab_scale")
    n_tcp = 1 + 2 + (SCALE["write_bytes"] + 535) // 536 + 2
    got = _run(tmp_path, TXQ_SLAB, "gpu", dict(SCALE, hold=True, **SLAB), env=_env(0), tag="slab_hold_scale")
    _check_same(base, got, first_batch=n_tcp - 1)
    r = got["reports"][0]
    assert r["gpu_calls"] == 1 and r["cpu"] == 0, r
    # spans: about the segments' granules, not a gather of each frame (~604 B)
    assert 700 * r["frames"] < r["h2d_bytes"] < 1600 * r["frames"], r
