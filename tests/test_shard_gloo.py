"""The multi-GPU path's host logic on CPU: byte-balanced contiguous partition,
per-rank rebasing, and the result all-gather, with a world_size-2 gloo group
(the GPU run uses the same code with RCCL).  Each rank checksums its shard with
the oracle (no GPU here) and the gathered results must equal the single-batch
oracle bit for bit."""
import os
import socket

import numpy as np
import pytest

import shard
import workloads


def test_partition_balanced_and_contiguous():
    rng = np.random.default_rng(1)
    lens = rng.integers(-5, 9000, 10001)
    for world in (1, 2, 3, 8):
        parts = shard.partition(lens, world)
        assert parts[0][0] == 0 and parts[-1][1] == lens.size
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        b = [int(np.maximum(lens[lo:hi], 0).sum()) for lo, hi in parts]
        assert max(b) - min(b) <= 2 * 9000  # within a couple of packets of perfect
    assert shard.partition(np.zeros(5), 2) == [(0, 2), (2, 5)]
    assert shard.partition(np.array([], dtype=np.int64), 4) == [(0, 0)] * 4


def test_local_batch_rebases():
    b = workloads.make("mixed", n=1000)
    d, start, span = shard.local_batch(b.descs, 10, 500)
    assert start % 16 == 0 and span % 16 == 0
    assert int(d["offset"].min()) < 16
    assert np.array_equal(d["len"], b.descs["len"][10:500])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, "..", "level-ip_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import pyoracle
    import shard as sh
    import workloads as wl

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        b = wl.make("mixed", n=3000)
        host = b.host_bytes()
        parts = sh.partition(b.descs["len"], world)
        lo, hi = parts[rank]
        d, start, span = sh.local_batch(b.descs, lo, hi)
        local = pyoracle.batch(host[start:start + span], d) if d.size else np.zeros(0, np.uint16)
        out = sh.gather_results(torch.from_numpy(local.view(np.int16).copy()),
                                [h - l for l, h in parts])
        if rank == 0:
            full = pyoracle.batch(host, b.descs)
            q.put(bool(np.array_equal(out.numpy().view(np.uint16), full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_shards_match_single_batch():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(170)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def _scatter_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, "..", "level-ip_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import pyoracle
    import shard as sh
    import workloads as wl

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        buf, descs = None, None
        if rank == 0:  # the batch originates on one rank only
            b = wl.make("mixed", n=2500)
            buf, descs = torch.from_numpy(b.host_bytes()), b.descs
        local, d, (lo, hi) = sh.scatter_from_root(buf, descs, torch.device("cpu"))
        out = pyoracle.batch(local.numpy(), d) if d.size else np.zeros(0, np.uint16)
        counts = [0] * world
        cnt = torch.tensor([hi - lo], dtype=torch.int64)
        allc = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, cnt)
        counts = [int(c) for c in allc]
        res = sh.gather_results(torch.from_numpy(out.view(np.int16).copy()), counts)
        if rank == 0:
            full = pyoracle.batch(buf.numpy(), descs)
            q.put(bool(np.array_equal(res.numpy().view(np.uint16), full)) and sum(counts) == descs.size)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_scatter_from_root_then_gather(world):
    """Batch held by rank 0 only: scatter byte-balanced shards point to point,
    checksum each shard, all-gather: equals the single batch bit for bit."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(170)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
