"""Group 4 of include/lvlip_csum.h on the CPU: lvlip_partition_bytes gives the
same byte-balanced contiguous cuts as level-ip_amd/shard.py partition() (the
Python side of the multi-GPU bench) on ragged, empty and adversarial batches,
and the multi-context entry refuses bad arguments before any GPU call."""
import ctypes

import numpy as np
import pytest

import lvlip
import shard
import workloads


def _descs(lens):
    d = np.zeros(len(lens), dtype=lvlip.DESC_DTYPE)
    d["len"] = lens
    d["offset"] = np.concatenate([[0], np.cumsum(np.maximum(lens, 0))[:-1]]) if len(lens) else []
    return d


def _py_cuts(lens, parts):
    rng = shard.partition(np.asarray(lens), parts)
    return [rng[0][0]] + [hi for _, hi in rng]


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 7, 8, 16])
def test_cuts_equal_shard_partition_on_ragged(parts):
    rng = np.random.default_rng(parts)
    for trial in range(20):
        n = int(rng.integers(0, 3000))
        lens = rng.integers(-40, 9001, n)  # empty / negative lengths included
        lens[rng.random(n) < 0.05] = 0
        assert lvlip.partition_bytes(_descs(lens), parts) == _py_cuts(lens, parts), (trial, n)


def test_cuts_on_the_configs():
    for name, n in (("mixed", 1 << 15), ("tcp1500", 1 << 12)):
        b = workloads.make(name, n=n)
        for parts in (2, 4, 8):
            cuts = lvlip.partition_bytes(b.descs, parts)
            assert cuts == _py_cuts(b.descs["len"], parts)
            bytes_ = [int(np.maximum(b.descs["len"][lo:hi], 0).sum()) for lo, hi in zip(cuts, cuts[1:])]
            assert max(bytes_) - min(bytes_) <= 2 * int(b.descs["len"].max())  # balanced to a packet per cut


def test_edge_cases():
    # all empty: by count; n < parts; one huge packet; INT_MAX lengths (128-bit products)
    assert lvlip.partition_bytes(_descs([0] * 5), 2) == _py_cuts([0] * 5, 2) == [0, 2, 5]
    assert lvlip.partition_bytes(_descs([]), 4) == [0, 0, 0, 0, 0]
    assert lvlip.partition_bytes(_descs([10, 20]), 5) == _py_cuts([10, 20], 5)
    big = [2**31 - 1] * 1000
    assert lvlip.partition_bytes(_descs(big), 7) == _py_cuts(big, 7)
    assert lvlip.partition_bytes(_descs([5, 1 << 30, 5, 5]), 3) == _py_cuts([5, 1 << 30, 5, 5], 3)
    cuts = lvlip.partition_bytes(_descs(list(range(100))), 8)
    assert cuts[0] == 0 and cuts[-1] == 100 and cuts == sorted(cuts)


def test_bad_arguments():
    L = lvlip.lib()
    cuts = np.zeros(3, dtype=np.uint32)
    d = _descs([1, 2, 3])
    assert L.lvlip_partition_bytes(d.ctypes.data, 3, 0, cuts.ctypes.data) == lvlip.EINVAL
    assert L.lvlip_partition_bytes(None, 3, 2, cuts.ctypes.data) == lvlip.EINVAL
    assert L.lvlip_partition_bytes(d.ctypes.data, 3, 2, None) == lvlip.EINVAL
    assert L.lvlip_partition_bytes(None, 0, 2, cuts.ctypes.data) == lvlip.OK
    out = np.zeros(3, dtype=np.uint16)
    base = np.zeros(64, dtype=np.uint8)
    arr = (ctypes.c_void_p * 2)(None, None)
    assert L.lvlip_csum_batch_host_flat_multi(None, 2, base.ctypes.data, 64, d.ctypes.data, 3,
                                              out.ctypes.data) == lvlip.EINVAL
    assert L.lvlip_csum_batch_host_flat_multi(arr, 0, base.ctypes.data, 64, d.ctypes.data, 3,
                                              out.ctypes.data) == lvlip.EINVAL
    assert L.lvlip_csum_batch_host_flat_multi(arr, 2, base.ctypes.data, 64, d.ctypes.data, 3,
                                              out.ctypes.data) == lvlip.EINVAL  # NULL contexts
    assert L.lvlip_icmp_echo_reply_dev_ex(None, None, 0, 2, None, None) == lvlip.EINVAL  # unknown flag
    same = (ctypes.c_void_p * 2)(0x1000, 0x1000)  # one context twice: refused before it is touched
    assert L.lvlip_csum_batch_host_flat_multi(same, 2, base.ctypes.data, 64, d.ctypes.data, 3,
                                              out.ctypes.data) == lvlip.EINVAL
