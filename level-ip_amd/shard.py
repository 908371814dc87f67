"""Multi-GPU sharding of a checksum batch (one process per GPU).

Packets are independent, so a batch shards by contiguous
descriptor ranges with no exchange on the data path:

  partition(lens, world)   contiguous ranges balanced by bytes (prefix sums), so
                           a ragged batch gives every rank about the same HBM
                           traffic, which is what bounds the kernel
  local_batch(...)         a rank's descriptors rebased to its own byte span
  scatter_from_root(...)   when the batch originates on one GPU: each rank's
                           bytes and descriptors sent point to point from the
                           root (RCCL over xGMI), timed separately from the
                           kernel
  gather_results(...)      results back in batch order (torch.distributed
                           all_gather: RCCL on GPUs, gloo on CPU tests), 2 bytes
                           per packet on the wire

The C-ABI has the same partition (lvlip_partition_bytes, include/lvlip_csum.h
Group 4) for a level-ip daemon that shards over the node's GPUs from threads.

bench.py's weak-scaling run does not move packets at all: each rank
generates its own shard of the stream (workloads.make(first=rank*n)).
"""
from __future__ import annotations

import numpy as np

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])


def partition(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """[lo, hi) descriptor ranges, contiguous, covering all n, balanced by bytes.

    Rank r gets the descriptors whose byte prefix falls in
    [r*T/world, (r+1)*T/world), T = total bytes; empty (len <= 0) descriptors
    cost nothing and go with their neighbours."""
    lens = np.maximum(np.asarray(lens, dtype=np.int64), 0)
    n = lens.size
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    pre = np.concatenate([[0], np.cumsum(lens)])
    total = int(pre[-1])
    if total == 0:  # all empty: split by count
        cuts = [n * r // world for r in range(world + 1)]
    else:
        targets = [total * r // world for r in range(world + 1)]
        cuts = [int(np.searchsorted(pre, t, side="left")) for t in targets]
        cuts[0], cuts[-1] = 0, n
        for r in range(1, world + 1):  # monotone
            cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def local_batch(descs: np.ndarray, lo: int, hi: int) -> tuple[np.ndarray, int, int]:
    """Descriptors [lo, hi) rebased to their own 16-B aligned byte span.

    Returns (local_descs, span_start, span_bytes): the rank needs bytes
    [span_start, span_start + span_bytes) of the global buffer."""
    d = np.ascontiguousarray(descs[lo:hi]).copy()
    if d.size == 0:
        return d, 0, 0
    end = d["offset"] + np.maximum(d["len"], 0).astype(np.uint64)
    start = int(d["offset"].min()) & ~15
    stop = (int(end.max()) + 15) & ~15
    d["offset"] -= np.uint64(start)
    return d, start, stop - start


def gather_results(local_out, counts: list[int], group=None):
    """All-gather per-rank uint16 result tensors (sizes `counts`) into batch order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    m = max(counts) if counts else 0
    # carried as their 2 bytes each (uint8: RCCL and gloo both gather bytes;
    # gloo has no 16-bit integer collective), bit pattern kept
    buf = torch.zeros(2 * m, dtype=torch.uint8, device=local_out.device)
    buf[: 2 * local_out.numel()] = local_out.contiguous().view(torch.int16).view(torch.uint8)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[: 2 * c] for p, c in zip(parts, counts)]).view(torch.int16)


def scatter_from_root(buf, descs, device, group=None, root: int = 0):
    """Distribute a batch held by `root` (buf: uint8 tensor, descs: DESC_DTYPE
    array; both ignored on other ranks).  Returns this rank's
    (local_buf uint8 tensor on `device`, local_descs array, (lo, hi)).

    The partition is byte-balanced and contiguous (partition()); each rank's
    byte span travels as one send from the root, so the only traffic is the
    data itself plus 16 B per descriptor."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    meta = torch.zeros((world, 4), dtype=torch.int64, device=device)  # lo, hi, start, span
    plan = []
    if rank == root:
        for lo, hi in partition(descs["len"], world):
            d, start, span = local_batch(descs, lo, hi)
            plan.append((d, start, span))
            meta[len(plan) - 1] = torch.tensor([lo, hi, start, span], dtype=torch.int64)
    dist.broadcast(meta, src=root, group=group)
    m = meta.cpu().tolist()
    if rank == root:
        reqs = []
        for r in range(world):
            if r == root:
                continue
            d, start, span = plan[r]
            if m[r][1] > m[r][0]:
                dt = torch.from_numpy(d.view(np.uint8).copy()).to(device)
                reqs.append(dist.isend(dt, dst=r, group=group))
            if span:
                reqs.append(dist.isend(buf[start:start + span].contiguous(), dst=r, group=group))
        for q in reqs:
            q.wait()
        d, start, span = plan[root]
        return buf[start:start + span].clone(), d, (m[root][0], m[root][1])
    lo, hi, start, span = m[rank]
    d = np.zeros(hi - lo, dtype=DESC_DTYPE)
    if hi > lo:
        dt = torch.empty((hi - lo) * DESC_DTYPE.itemsize, dtype=torch.uint8, device=device)
        dist.recv(dt, src=root, group=group)
        d = dt.cpu().numpy().view(DESC_DTYPE).copy()
    local = torch.empty(span, dtype=torch.uint8, device=device)
    if span:
        dist.recv(local, src=root, group=group)
    return local, d, (lo, hi)
