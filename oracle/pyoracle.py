"""ctypes access to the CPU oracle and to the compiled reference (oracle/_ref).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / reported CPU baseline.  The
product never imports this module.

  liblib()   oracle/build/liboracle.so     csum_oracle.c at -O2 (checker)
  liblib(0)  oracle/build/liboracle_O0.so  csum_oracle.c at -O0 (reference flags)
  reflib()   oracle/_ref/libref.so         level-ip's own src/*.c (minus main.c),
                                           compiled by oracle/Makefile; None if absent
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "liboracle.so")
ORACLE_O0_SO = os.path.join(HERE, "build", "liboracle_O0.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

CSUM_FN = ctypes.CFUNCTYPE(ctypes.c_uint16, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)

_cache: dict = {}


def _setup_oracle(lib: ctypes.CDLL) -> ctypes.CDLL:
    lib.oracle_sum_every_16bits.restype = ctypes.c_uint32
    lib.oracle_sum_every_16bits.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.oracle_checksum.restype = ctypes.c_uint16
    lib.oracle_checksum.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.oracle_pseudo_sum.restype = ctypes.c_uint32
    lib.oracle_pseudo_sum.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                      ctypes.c_uint16]
    lib.oracle_tcp_udp_checksum.restype = ctypes.c_int
    lib.oracle_tcp_udp_checksum.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                            ctypes.c_void_p, ctypes.c_uint16]
    lib.oracle_ip_send_check.restype = None
    lib.oracle_ip_send_check.argtypes = [ctypes.c_void_p]
    lib.oracle_batch.restype = None
    lib.oracle_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_void_p]
    lib.oracle_batch_mt.restype = ctypes.c_int
    lib.oracle_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    lib.oracle_fill.restype = None
    lib.oracle_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_uint64]
    return lib


def ensure_built() -> None:
    if not (os.path.exists(ORACLE_SO) and os.path.exists(ORACLE_O0_SO)):
        import subprocess
        subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def liblib(opt: int = 2) -> ctypes.CDLL:
    key = ("oracle", opt)
    if key not in _cache:
        ensure_built()
        _cache[key] = _setup_oracle(ctypes.CDLL(ORACLE_SO if opt else ORACLE_O0_SO))
    return _cache[key]


def reflib() -> Optional[ctypes.CDLL]:
    """The reference's own compiled objects, or None when oracle/_ref was not built."""
    if "ref" not in _cache:
        if not os.path.exists(REF_SO):
            _cache["ref"] = None
        else:
            lib = ctypes.CDLL(REF_SO)
            lib.checksum.restype = ctypes.c_uint16
            lib.checksum.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            lib.sum_every_16bits.restype = ctypes.c_uint32
            lib.sum_every_16bits.argtypes = [ctypes.c_void_p, ctypes.c_int]
            lib.tcp_udp_checksum.restype = ctypes.c_int
            lib.tcp_udp_checksum.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                             ctypes.c_void_p, ctypes.c_uint16]
            lib.ip_send_check.restype = None
            lib.ip_send_check.argtypes = [ctypes.c_void_p]
            _cache["ref"] = lib
    return _cache["ref"]


def _u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def _i32(x: int) -> int:
    return ctypes.c_int(ctypes.c_uint32(x & 0xFFFFFFFF).value).value


def checksum(buf, count: Optional[int] = None, start_sum: int = 0) -> int:
    a = _u8(buf)
    count = a.size if count is None else count
    if count > a.size:  # the C oracle would read past the buffer (count <= 0 reads nothing)
        raise ValueError(f"count {count} outside a {a.size}-byte buffer")
    return int(liblib().oracle_checksum(a.ctypes.data if a.size else None, count, _i32(start_sum)))


def sum_every_16bits(buf, count: Optional[int] = None) -> int:
    a = _u8(buf)
    count = a.size if count is None else count
    if count > a.size:
        raise ValueError(f"count {count} outside a {a.size}-byte buffer")
    return int(liblib().oracle_sum_every_16bits(a.ctypes.data if a.size else None, count))


def pseudo_sum(saddr: int, daddr: int, proto: int, length: int) -> int:
    return int(liblib().oracle_pseudo_sum(saddr & 0xFFFFFFFF, daddr & 0xFFFFFFFF, proto & 0xFF,
                                          length & 0xFFFF))


def batch(base: np.ndarray, descs: np.ndarray, threads: int = 1, opt: int = 2,
          use_reference: bool = False, csum_fn=None) -> np.ndarray:
    """out[i] = checksum(base + off_i, len_i, start_i) on the CPU.

    use_reference=True calls the reference's own checksum() from oracle/_ref per
    packet (pthreads over contiguous packet ranges); csum_fn (a ctypes function
    with checksum()'s signature) times another per-call implementation with the
    same harness (bench.py's diag of the product's CPU drop-in)."""
    base = _u8(base)
    descs = np.ascontiguousarray(descs)
    assert descs.dtype.itemsize == 16
    n = descs.size
    out = np.empty(n, dtype=np.uint16)
    lib = liblib(opt)
    fn = ctypes.cast(csum_fn, ctypes.c_void_p) if csum_fn is not None else None
    if use_reference:
        ref = reflib()
        if ref is None:
            raise FileNotFoundError(REF_SO)
        fn = ctypes.cast(ref.checksum, ctypes.c_void_p)
    if threads <= 1 and fn is None:
        lib.oracle_batch(base.ctypes.data, descs.ctypes.data, n, out.ctypes.data)
    else:
        rc = lib.oracle_batch_mt(fn, base.ctypes.data, descs.ctypes.data, n, out.ctypes.data,
                                 max(1, threads))
        if rc != 0:
            raise MemoryError("oracle_batch_mt")
    return out
