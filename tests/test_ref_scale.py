"""Both batch-and-dispatch steps at scale on level-ip's own stack (VERDICT r05
Next #3): an RX burst of tens of thousands of echo requests of every ip_rcv
kind, through level-ip as it is (oracle/_ref/libref_rxq.so, one skb at a time,
every checksum on the CPU) and through the batched stack
(oracle/_ref/libref_rxtxq.so: one lvlip_rx_verify_skb_list over the queue, the
dispatch, ip_rcv's header sum answered by the verdict, the replies' checksums
deferred and filled by one flush).  The frames on the tap must be identical,
reply for reply (tests/ref_scale_child.py).  Skipped when oracle/_ref was not
built (it needs /root/reference at build time)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
RXQ = os.path.join(REF, "libref_rxq.so")
RXTXQ = os.path.join(REF, "libref_rxtxq.so")
RXTXQ_SLAB = os.path.join(REF, "libref_rxtxq_slab.so")
CHILD = os.path.join(ROOT, "tests", "ref_scale_child.py")

pytestmark = pytest.mark.skipif(not (os.path.exists(RXQ) and os.path.exists(RXTXQ)),
                                reason="oracle/_ref/libref_{rxq,rxtxq}.so not built")


def run(tmp_path, lib, mode, opts, cpu_max=None, tag=None, **extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("LVLIP_CPU_MAX", "LVLIP_FAIL_PIECE")}
    if cpu_max is not None:
        env["LVLIP_CPU_MAX"] = str(cpu_max)
    env.update({k: str(v) for k, v in extra_env.items()})
    out = tmp_path / f"{tag or mode}.json"
    r = subprocess.run([sys.executable, CHILD, str(out), lib, mode, json.dumps(opts)], stdin=subprocess.DEVNULL,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(out.read_text())


def _check(base, got, n):
    assert got["frames"] == base["frames"]
    # the ARP reply and one echo reply per answered request
    assert len(base["frames"]) > n // 4
    # unbatched: ip_rcv sums every header that reaches :38; batched: none
    assert base["cpu_header_sums"] > 0 and base["batch_header_sums"] == 0
    assert got["cpu_header_sums"] == 0 and got["batch_header_sums"] == got["verdicts"].get("1", 0)


def _calls(r, n, cpu_max):
    """(GPU calls, CPU calls) the burst's two library calls should make: the
    RX verify over n + 1 frames (the ARP request too), then the TX flush over
    r["queued"] replies, each on the GPU above the threshold (r holds the
    context's counters over the whole burst)."""
    import lvlip

    t = lvlip.CPU_MAX_DEFAULT if cpu_max is None else cpu_max
    gpu = int(n + 1 > t) + int(r["queued"] > t)
    return gpu, 2 - gpu


def test_rx_tx_burst_oracle_composition(tmp_path):
    """CPU: 2 000 frames with the oracle's verdicts and TX fill in place of the
    library (the harness's own check on a machine without a GPU)."""
    opts = {"n": 2000, "seed": 5, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    _check(base, run(tmp_path, RXTXQ, "oracle", opts), 2000)


@pytest.mark.gpu
@pytest.mark.parametrize("cpu_max", [None, 0])
def test_rx_tx_burst_at_scale(tmp_path, cpu_max):
    """30 000 frames of every kind, one RX call and one TX flush: with the
    default threshold the RX call (30 001 frames) goes to the GPU and the
    flush of ~11 000 replies stays on the calling thread; with threshold 0
    both run on the GPU.  The tap bytes equal the unbatched stack's, frame for
    frame, and no header is summed on the CPU."""
    opts = {"n": 30000, "seed": 6, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ, "batched", opts, cpu_max=cpu_max, tag=f"b{cpu_max}")
    _check(base, got, 30000)
    r = got["reports"][0]
    assert r["cpu"] == 0 and r["frames"] == r["queued"] > 5000
    assert (r["gpu_calls"], r["cpu_calls"]) == _calls(r, 30000, cpu_max), r


@pytest.mark.gpu
def test_rx_tx_small_burst_default_threshold_on_cpu(tmp_path):
    """A burst of 40 frames (level-ip's usual flush size) with the default
    threshold: the RX call and the flush both run on the calling thread, and
    the tap bytes are the unbatched stack's."""
    opts = {"n": 40, "seed": 7, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ, "batched", opts)
    _check(base, got, 40)
    r = got["reports"][0]
    assert (r["gpu_calls"], r["cpu_calls"]) == (0, 2)


@pytest.mark.skipif(not os.path.exists(RXTXQ_SLAB), reason="oracle/_ref/libref_rxtxq_slab.so not built")
def test_rx_tx_burst_slab_allocator_oracle(tmp_path):
    """CPU: the stack with every skb buffer from one slab (oracle/ref_slab.c,
    alloc_skb / free_skb weakened in a copy of skbuff.o) and the oracle in
    place of the library: the tap bytes are the unbatched stack's."""
    opts = {"n": 2000, "seed": 8, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    _check(base, run(tmp_path, RXTXQ_SLAB, "oracle", dict(opts, slab=1 << 28), tag="slab_oracle"), 2000)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(RXTXQ_SLAB), reason="oracle/_ref/libref_rxtxq_slab.so not built")
def test_rx_tx_burst_from_registered_slab(tmp_path):
    """30 000 frames whose skb buffers lie in one slab the context registers
    (LVLIP_REG_DMA): the RX call and the flush move them with the copy engine
    (dense and in order: the flush's bytes moved are its frames' span); the
    tap bytes equal the unbatched stack's."""
    opts = {"n": 30000, "seed": 9, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ_SLAB, "batched", dict(opts, slab=1 << 28), cpu_max=0, tag="slab_gpu")
    _check(base, got, 30000)
    r = got["reports"][0]
    assert r["gpu_calls"] == 2 and r["cpu"] == 0 and r["frames"] == r["queued"] > 5000
    # the burst's skbs (1 600-B buffers in 256-B granules) and the queued
    # replies moved as their own spans, not the whole 256 MiB slab
    assert r["h2d_bytes"] < 2 * 1792 * (30001 + r["queued"]), r


@pytest.mark.gpu
def test_rx_tx_burst_gpu_failure_falls_back(tmp_path):
    """Every GPU call of the burst fails (LVLIP_FAIL_PIECE=1): the RX verify
    (lvlip_rxq_verify, oracle/ref_rxq.c) and the TX flush (lvlip_txq_fill)
    both fall back to the library's CPU code, and the tap bytes are still the
    unbatched stack's: a GPU failure neither drops, admits nor sends a frame
    differently (failure detection)."""
    opts = {"n": 3000, "seed": 10, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ, "batched", opts, cpu_max=0, tag="fail", LVLIP_FAIL_PIECE=1)
    _check(base, got, 3000)
    r = got["reports"][0]
    assert r["rx_cpu_fallback"] == 1 and r["cpu"] == 1 and r["rc"] == -3 and r["frames"] == r["queued"], r


def test_rx_tx_burst_hold_oracle(tmp_path):
    """CPU: the replies held by reference (no copy; oracle/ref_txq.c's hold
    mode) and filled by the oracle: the tap bytes are the unbatched stack's,
    and every reply's skb is freed by the flush (the run ends cleanly)."""
    opts = {"n": 2000, "seed": 11, "kinds": "all"}
    base = run(tmp_path, RXQ, "unbatched", opts)
    _check(base, run(tmp_path, RXTXQ, "oracle", dict(opts, hold=1), tag="hold_oracle"), 2000)


@pytest.mark.gpu
@pytest.mark.parametrize("cpu_max", [None, 0])
def test_rx_tx_burst_hold_at_scale(tmp_path, cpu_max):
    """30 000 frames, the replies held by reference: one RX call, the
    dispatch, one lvlip_tx_checksum over the held replies; tap bytes equal
    the unbatched stack's with either threshold."""
    opts = {"n": 30000, "seed": 12, "kinds": "all", "hold": 1}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ, "batched", opts, cpu_max=cpu_max, tag=f"hold{cpu_max}")
    _check(base, got, 30000)
    r = got["reports"][0]
    assert r["cpu"] == 0 and r["frames"] == r["queued"] > 5000
    assert (r["gpu_calls"], r["cpu_calls"]) == _calls(r, 30000, cpu_max), r


@pytest.mark.parametrize("hold", [0, 1])
def test_rx_tx_burst_no_context_runs_on_cpu(tmp_path, hold):
    """CPU: the batched stack as one C call per burst (lvlip_rxtxq_burst,
    oracle/ref_rxtxq.c) with no context (an invalid device: LVLIP_ENODEV):
    the RX verify and the TX fill both fall back to the library's CPU code,
    and the tap bytes are the unbatched stack's, replies copied or held."""
    opts = {"n": 2000, "seed": 13, "kinds": "all", "device": 99, "hold": hold}
    base = run(tmp_path, RXQ, "unbatched", opts)
    got = run(tmp_path, RXTXQ, "batched", opts, tag=f"nodev{hold}")
    assert got["context_error"] == -2
    _check(base, got, 2000)
    r = got["reports"][0]
    assert r["rx_cpu_fallback"] == 1 and r["cpu"] == 1 and r["rc"] == -2 and r["frames"] == r["queued"], r
