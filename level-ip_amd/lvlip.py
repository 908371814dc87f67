"""lvlip — ctypes binding of liblvlip_csum.so (include/lvlip_csum.h).

Host-side mirror of level-ip's checksum interface for tests/ and bench.py.
The names follow the reference:

  checksum(buf, count, start_sum)      src/utils.c:40-55  (include/utils.h:14)
  sum_every_16bits(buf, count)         src/utils.c:22-38  (include/utils.h:13)
  tcp_udp_checksum(saddr, daddr, proto, data, len)   src/tcp.c:87-98
  ip_send_check(iphdr_bytearray)       src/ip_output.c:8-12

plus the batched GPU entry points (batch_dev, Context.batch_host[_flat]).

The library is loaded eagerly and a missing or broken build raises
LvlipUnavailable: there is no Python or CPU fallback for the batched path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblvlip_csum.so")
TESTKIT_PATH = os.path.join(HERE, "liblvlip_testkit.so")
LAB_PATH = os.path.join(HERE, "liblvlip_lab.so")

# error codes (include/lvlip_csum.h)
OK, EINVAL, ENODEV, EHIP, ENOMEM, ERANGE = 0, -1, -2, -3, -4, -5
# the product's kernels (include/lvlip_csum.h)
KERNEL_AUTO, KERNEL_FLAT, KERNEL_WINDOW, KERNEL_LANE = 0, 3, 8, 10
# the A/B variants measured against them, in liblvlip_lab.so (lab_kernels.hip);
# batch_dev sends these ids (and FLAT's A/B shapes) there, the product
# returns EINVAL for them.
KERNEL_WAVE, KERNEL_WFLAT, KERNEL_FLAT_OCC = 1, 9, 13
LAB_KERNELS = (KERNEL_WAVE, KERNEL_WFLAT, KERNEL_FLAT_OCC)
# retired ids (EINVAL in both libraries): 6 and 7 (round 1's balanced stream
# kernels), and the lab kernels pruned in round 4 after losing their A/Bs by
# >= 3 % (k_wave_lds 2, k_wave_simple 4, k_flat v1 5, k_rflat 11, k_wsflat 12,
# k_flat2_perm 14, k_window_dyn 15; DESIGN.md §4, last in commit 4e633d9)
RETIRED_KERNELS = (2, 4, 5, 6, 7, 11, 12, 14, 15)
REG_DMA, REG_ZEROCOPY = 0, 1
KERNEL_NAMES = {"auto": KERNEL_AUTO, "wave": KERNEL_WAVE, "flat": KERNEL_FLAT, "window": KERNEL_WINDOW,
                "wflat": KERNEL_WFLAT, "lane": KERNEL_LANE, "flat_occ": KERNEL_FLAT_OCC}
KERNEL_LABELS = {v: k for k, v in KERNEL_NAMES.items()}

# struct lvlip_csum_desc {u64 offset; i32 len; u32 start_sum;}  (16 B)
DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])
assert DESC_DTYPE.itemsize == 16


class LvlipUnavailable(RuntimeError):
    """liblvlip_csum.so is missing or cannot be loaded."""


class LvlipError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        detail = ""
        try:
            detail = _lib.lvlip_last_hip_error().decode()
        except Exception:  # pragma: no cover
            pass
        msg = f"{what}: {_lib.lvlip_strerror(rc).decode()} ({rc})"
        if detail:
            msg += f" [{detail}]"
        super().__init__(msg)


class LaunchCfg(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int32), ("unroll", ctypes.c_int32),
                ("waves_per_cu", ctypes.c_int32), ("len_hint", ctypes.c_int32)]


class Iov(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("len", ctypes.c_int32), ("start_sum", ctypes.c_uint32)]


class Frame(ctypes.Structure):  # include/lvlip_skb.h: lvlip_frame
    _fields_ = [("head", ctypes.c_void_p), ("len", ctypes.c_uint32)]


class CtxStats(ctypes.Structure):  # include/lvlip_csum.h: lvlip_ctx_stats
    _fields_ = [("gpu_calls", ctypes.c_uint64), ("cpu_calls", ctypes.c_uint64),
                ("pieces", ctypes.c_uint64), ("h2d_bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# include/lvlip_csum.h: host calls of at most this many packets / frames run on
# the calling thread unless the context says otherwise (LVLIP_CPU_MAX)
CPU_MAX_DEFAULT = 16384


# RX verdicts and flags (include/lvlip_skb.h)
RX_OK, RX_NOT_IP, RX_SHORT, RX_BAD_VERSION, RX_BAD_IHL, RX_TTL0, RX_BAD_CSUM, RX_BAD_L4, \
    RX_UNKNOWN_PROTO = range(1, 10)
RX_VERIFY_L4 = 0x1
ECHO_FULL = 0x1  # lvlip_icmp_echo_reply_dev_ex (include/lvlip_skb.h)
PLAN_MALFORMED = 0xFFFFFFFF


def _share_torch_hip_runtime() -> None:
    """Make this process use ONE HIP runtime.

    PyTorch-ROCm ships its own libamdhip64.so (SONAME libamdhip64.so.7) and its
    libtorch_hip.so asks for it by the name "libamdhip64.so".  If our library were
    loaded first, the dynamic linker would resolve its libamdhip64.so.7 from
    /opt/rocm and torch would later map a second runtime next to it.  Preloading
    torch's copy (RTLD_GLOBAL) makes both resolve to the same file."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)


def _load(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise LvlipUnavailable(
            f"{path} not built: run `make -C level-ip_amd` (or __graft_entry__.build())")
    try:
        return ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover
        raise LvlipUnavailable(f"cannot load {path}: {e}") from e


BUILD_SOURCES = os.path.join(HERE, "BUILD_SOURCES")


def source_build_id(list_file: str = BUILD_SOURCES) -> str:
    """SHA-256 (first 16 hex digits) of the sources a list file names, in its
    order: BUILD_SOURCES (the product, lvlip_build_id()), LAB_SOURCES or
    TESTKIT_SOURCES (the helper libraries' stamps) -- what
    level-ip_amd/Makefile compiles into each library."""
    import hashlib

    root = os.path.dirname(HERE)
    h = hashlib.sha256()
    with open(list_file) as f:
        for rel in f.read().split():
            with open(os.path.join(root, rel), "rb") as g:
                h.update(g.read())
    return h.hexdigest()[:16]


def _stamp(lib: ctypes.CDLL, path: str, symbol: str, list_file: str) -> str:
    """The library's build stamp, checked against the tree's sources; a
    library without the symbol (built before stamps existed) or with another
    stamp is stale and refused."""
    try:
        fn = getattr(lib, symbol)
    except AttributeError:
        raise LvlipUnavailable(f"{path} has no {symbol} (built before build stamps): rebuild with "
                               "`make -C level-ip_amd`") from None
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    got, want = fn().decode(), source_build_id(list_file)
    if got != want:
        raise LvlipUnavailable(f"{path} was built from other sources (stamp {got}, tree {want}): "
                               "rebuild with `make -C level-ip_amd`")
    return got


_share_torch_hip_runtime()
_lib = _load(LIB_PATH)
BUILD_ID = _stamp(_lib, LIB_PATH, "lvlip_build_id", BUILD_SOURCES)

# every entry point declared in include/lvlip_csum.h, with its ctypes signature
SIGNATURES = {
    "sum_every_16bits": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int]),
    "checksum": (ctypes.c_uint16, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "lvlip_pseudo_sum": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                            ctypes.c_uint16]),
    "tcp_udp_checksum": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                        ctypes.c_void_p, ctypes.c_uint16]),
    "tcp_v4_checksum": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]),
    "ip_send_check": (None, [ctypes.c_void_p]),
    "lvlip_csum_batch_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "lvlip_csum_batch_dev_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.POINTER(LaunchCfg)]),
    "lvlip_csum_ctx_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                             ctypes.c_size_t]),
    "lvlip_csum_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "lvlip_csum_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Iov), ctypes.c_uint32,
                                             ctypes.c_void_p]),
    "lvlip_csum_batch_host_flat": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_void_p]),
    "lvlip_csum_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_uint32]),
    "lvlip_csum_unregister": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lvlip_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    # include/lvlip_skb.h (f1/f2 frame batches)
    "lvlip_rx_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Frame), ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_void_p]),
    "lvlip_rx_plan": (ctypes.c_uint32, [ctypes.POINTER(Frame), ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.POINTER(Iov), ctypes.c_void_p]),
    "lvlip_rx_apply": (None, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                              ctypes.c_void_p]),
    "lvlip_tx_checksum": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Frame), ctypes.c_uint32]),
    "lvlip_tx_plan": (ctypes.c_uint32, [ctypes.POINTER(Frame), ctypes.c_uint32, ctypes.POINTER(Iov),
                                        ctypes.c_void_p]),
    "lvlip_tx_apply": (None, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "lvlip_icmp_echo_reply_csum": (ctypes.c_uint32, [ctypes.c_uint16]),
    "lvlip_icmp_echo_reply_fill": (ctypes.c_uint32, [ctypes.POINTER(Frame), ctypes.c_uint32]),
    "lvlip_frames_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32]),
    "lvlip_rx_verify_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "lvlip_tx_checksum_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lvlip_pseudo_sum_rfc": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                               ctypes.c_uint16]),
    "lvlip_icmp_echo_reply_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    "lvlip_icmp_echo_reply_dev_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    # Group 4: one batch over several GPUs
    "lvlip_partition_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_void_p]),
    "lvlip_csum_batch_host_flat_multi": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                        ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32,
                                                        ctypes.c_void_p]),
    "lvlip_rx_verify_skb_list": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_void_p, ctypes.c_uint32]),
    "lvlip_tx_checksum_skb_list": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    # round 6: size-based dispatch, counters, context-free CPU frame calls
    "lvlip_csum_ctx_set_cpu_max": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "lvlip_csum_ctx_cpu_max": (ctypes.c_uint32, [ctypes.c_void_p]),
    "lvlip_csum_ctx_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CtxStats)]),
    "lvlip_rx_verify_cpu": (ctypes.c_int, [ctypes.POINTER(Frame), ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_void_p]),
    "lvlip_tx_checksum_cpu": (ctypes.c_int, [ctypes.POINTER(Frame), ctypes.c_uint32]),
    "lvlip_rx_verify_skb_list_cpu": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                    ctypes.c_uint32]),
    "lvlip_tx_checksum_skb_list_cpu": (ctypes.c_int, [ctypes.c_void_p]),
    "lvlip_auto_kernel": (ctypes.c_int, [ctypes.c_int32, ctypes.c_uint32, ctypes.POINTER(LaunchCfg)]),
    "lvlip_batch_launches": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.POINTER(LaunchCfg)]),
    "lvlip_build_id": (ctypes.c_char_p, []),
    "lvlip_abi_version": (ctypes.c_int, []),
    "lvlip_device_count": (ctypes.c_int, []),
    "lvlip_last_hip_error": (ctypes.c_char_p, []),
}
for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(_lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


def lib() -> ctypes.CDLL:
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise LvlipError(rc, what)


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


# --------------------------------------------------------------- per call --

def sum_every_16bits(buf, count: Optional[int] = None) -> int:
    a = _as_u8(buf)
    if count is None:
        count = a.size
    if count > a.size:
        raise ValueError("count exceeds buffer")
    return int(_lib.sum_every_16bits(a.ctypes.data if a.size else None, int(count)))


def checksum(buf, count: Optional[int] = None, start_sum: int = 0) -> int:
    """src/utils.c:40-55; start_sum is the reference's `int` (any u32 bit pattern)."""
    a = _as_u8(buf)
    if count is None:
        count = a.size
    if count > a.size:
        raise ValueError("count exceeds buffer")
    s = ctypes.c_int(ctypes.c_uint32(start_sum & 0xFFFFFFFF).value).value
    return int(_lib.checksum(a.ctypes.data if a.size else None, int(count), s))


def pseudo_sum(saddr: int, daddr: int, proto: int, length: int) -> int:
    """Seed of tcp_udp_checksum (src/tcp.c:87-96), u32 wrap-around."""
    return int(_lib.lvlip_pseudo_sum(saddr & 0xFFFFFFFF, daddr & 0xFFFFFFFF, proto & 0xFF,
                                     length & 0xFFFF))


def tcp_udp_checksum(saddr: int, daddr: int, proto: int, data, length: int) -> int:
    """src/tcp.c:87-98 (len is a uint16_t there, so it is truncated the same way)."""
    length &= 0xFFFF
    a = _as_u8(data)
    if length > a.size:
        raise ValueError("length exceeds buffer")
    return int(_lib.tcp_udp_checksum(saddr & 0xFFFFFFFF, daddr & 0xFFFFFFFF, proto & 0xFF,
                                     a.ctypes.data if a.size else None, length))


def ip_send_check(hdr: bytearray) -> None:
    """src/ip_output.c:8-12: checksum over ihl*4 bytes, stored raw at offset 10."""
    if len(hdr) < max(20, (hdr[0] & 0x0F) * 4):
        raise ValueError("header shorter than ihl*4")
    c = (ctypes.c_char * len(hdr)).from_buffer(hdr)
    _lib.ip_send_check(ctypes.addressof(c))
    del c


# ---------------------------------------------------------- device batches --

def is_lab_kernel(kernel: int, unroll: int = 0) -> bool:
    """The A/B variants that live in liblvlip_lab.so: the lab kernel ids, and
    FLAT's shapes other than the product's (2, 4 or 8 loads per round, block
    order)."""
    if kernel in LAB_KERNELS:
        return True
    return kernel == KERNEL_FLAT and unroll not in (0, 2, 4, 8)


def batch_dev(base_ptr: int, desc_ptr: int, n: int, out_ptr: int, stream: int = 0,
              kernel: int = KERNEL_AUTO, unroll: int = 0, waves_per_cu: int = 0,
              len_hint: int = 0) -> None:
    """lvlip_csum_batch_dev_ex on raw device pointers (async on `stream`); an
    A/B variant id goes to lvlip_lab_batch_dev_ex (liblvlip_lab.so) instead."""
    cfg = LaunchCfg(kernel, unroll, waves_per_cu, min(max(int(len_hint), 0), 0x7FFFFFFF))
    if is_lab_kernel(kernel, unroll):
        _check(lab().lvlip_lab_batch_dev_ex(base_ptr, desc_ptr, n, out_ptr, stream or None,
                                            ctypes.byref(cfg)), "lvlip_lab_batch_dev_ex")
        return
    _check(_lib.lvlip_csum_batch_dev_ex(base_ptr, desc_ptr, n, out_ptr, stream or None,
                                        ctypes.byref(cfg)), "lvlip_csum_batch_dev_ex")


def auto_kernel(len_hint: int, n: int) -> LaunchCfg:
    """The kernel and shape LVLIP_KERNEL_AUTO runs (lvlip_auto_kernel)."""
    cfg = LaunchCfg()
    _lib.lvlip_auto_kernel(min(max(int(len_hint), 0), 0x7FFFFFFF), n, ctypes.byref(cfg))
    return cfg


def batch_launches(n: int, kernel: int = KERNEL_AUTO, unroll: int = 0, waves_per_cu: int = 0,
                   len_hint: int = 0) -> int:
    """Kernel launches one batch_dev call of n descriptors issues with this
    launch config (lvlip_batch_launches; AUTO resolved as the call does)."""
    if is_lab_kernel(kernel, unroll):  # the lab launches 2^30 descriptors at most
        return (n + (1 << 30) - 1) >> 30
    cfg = LaunchCfg(kernel, unroll, waves_per_cu, min(max(int(len_hint), 0), 0x7FFFFFFF))
    return int(_lib.lvlip_batch_launches(n, ctypes.byref(cfg)))


def auto_kernel_name(len_hint: int, n: int) -> str:
    return KERNEL_LABELS[auto_kernel(len_hint, n).kernel]


def batch_torch(base, descs, out=None, kernel: int = KERNEL_AUTO, unroll: int = 0,
                waves_per_cu: int = 0, stream=None, len_hint: int = 0):
    """Checksums a device batch held in torch tensors on the current stream.

    base:  uint8 CUDA tensor (16-B aligned, padded to a 16-B multiple past the last packet)
    descs: CUDA tensor of n*16 bytes (uint8 or int64 view of lvlip_csum_desc[n])
    out:   int16/uint16 CUDA tensor of n elements (allocated when None)
    """
    import torch

    if not (base.is_cuda and descs.is_cuda):
        raise ValueError("batch_torch needs CUDA tensors")
    if descs.device != base.device:
        raise ValueError("base and descs must be on the same device")
    if not (base.is_contiguous() and descs.is_contiguous()):
        raise ValueError("base and descs must be contiguous")
    nbytes = descs.numel() * descs.element_size()
    if nbytes % 16:
        raise ValueError(f"descs holds {nbytes} B, not a multiple of the 16-B descriptor")
    n = nbytes // 16
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=base.device)
    elif (not out.is_cuda or out.device != base.device or out.element_size() != 2
          or not out.is_contiguous() or out.numel() < n):
        raise ValueError(f"out must be a contiguous 2-byte CUDA tensor of >= {n} elements "
                         "on base's device")
    if stream is None:
        stream = torch.cuda.current_stream(base.device)
    batch_dev(base.data_ptr(), descs.data_ptr(), n, out.data_ptr(), stream.cuda_stream,
              kernel, unroll, waves_per_cu, len_hint)
    return out


def device_count() -> int:
    return int(_lib.lvlip_device_count())


# ------------------------------------------------------------ frame batches --

def frames_array(frames: Sequence[bytearray]):
    """lvlip_frame[n] over writable buffers (bytearray / uint8 ndarray), in place.

    Returns (array, keep); keep holds the buffer views alive while C uses them."""
    n = len(frames)
    arr = (Frame * max(n, 1))()
    keep = []
    for i, f in enumerate(frames):
        if isinstance(f, np.ndarray):
            a = f.view(np.uint8).reshape(-1)
            if not a.flags.c_contiguous:
                raise ValueError("frames must be contiguous")
            ptr, ln = a.ctypes.data, a.size
            keep.append(a)
        else:
            ln = len(f)
            c = (ctypes.c_char * max(ln, 1)).from_buffer(f) if ln else None
            ptr = ctypes.addressof(c) if c is not None else None
            keep.append(c)
        arr[i].head = ptr
        arr[i].len = ln
    return arr, keep


def pseudo_sum_rfc(saddr: int, daddr: int, proto: int, length: int) -> int:
    return int(_lib.lvlip_pseudo_sum_rfc(saddr & 0xFFFFFFFF, daddr & 0xFFFFFFFF, proto & 0xFF,
                                         length & 0xFFFF))


def rx_plan(frames, flags: int = 0):
    """lvlip_rx_plan: (verdict[n] uint8, [(ptr, len, start_sum)] * m, tag[m] uint32)."""
    n = len(frames)
    arr, keep = frames_array(frames)
    verdict = np.zeros(max(n, 1), dtype=np.uint8)
    iov = (Iov * max(2 * n, 1))()
    tag = np.zeros(max(2 * n, 1), dtype=np.uint32)
    m = _lib.lvlip_rx_plan(arr, n, flags, verdict.ctypes.data, iov, tag.ctypes.data)
    del keep
    return verdict[:n], [(iov[k].ptr, iov[k].len, iov[k].start_sum) for k in range(m)], tag[:m]


def rx_apply(verdict: np.ndarray, tag: np.ndarray, csum: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(verdict, dtype=np.uint8).copy()
    t = np.ascontiguousarray(tag, dtype=np.uint32)
    c = np.ascontiguousarray(csum, dtype=np.uint16)
    _lib.lvlip_rx_apply(v.size, v.ctypes.data, t.size, t.ctypes.data, c.ctypes.data)
    return v


def tx_plan(frames):
    """lvlip_tx_plan: ([(ptr, len, start_sum)] * m, field pointers[m]) or None if malformed."""
    n = len(frames)
    arr, keep = frames_array(frames)
    iov = (Iov * max(2 * n, 1))()
    field = np.zeros(max(2 * n, 1), dtype=np.uint64)
    m = _lib.lvlip_tx_plan(arr, n, iov, field.ctypes.data)
    del keep
    if m == PLAN_MALFORMED:
        return None
    return [(iov[k].ptr, iov[k].len, iov[k].start_sum) for k in range(m)], field[:m].copy()


CSUM_RECOMPUTE = 0xFFFFFFFF

# struct lvlip_frame_desc {u64 offset; u32 len; u32 reserved;}  (include/lvlip_skb.h)
FRAME_DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("reserved", "<u4")])


def pack_frames(frames, align_mod: int = 16, seed: int = 0):
    """Lay frames end to end in one uint8 array (each starting at a random
    offset mod `align_mod`), for the device-resident frame API.  Returns
    (buffer, FRAME_DESC_DTYPE descriptors)."""
    rng = np.random.default_rng(seed)
    offs, pos = [], 0
    for f in frames:
        pos += int(rng.integers(0, align_mod)) if align_mod > 1 else 0
        offs.append(pos)
        pos += len(f)
    buf = np.zeros((pos + 64 + 15) & ~15, dtype=np.uint8)
    d = np.zeros(len(frames), dtype=FRAME_DESC_DTYPE)
    for i, (o, f) in enumerate(zip(offs, frames)):
        buf[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        d[i]["offset"], d[i]["len"] = o, len(f)
    return buf, d


def _frames_dev(base, fdescs):
    import torch

    n = fdescs.numel() * fdescs.element_size() // 16 if hasattr(fdescs, "numel") else len(fdescs)
    if not hasattr(fdescs, "numel"):
        fdescs = torch.from_numpy(np.ascontiguousarray(fdescs, dtype=FRAME_DESC_DTYPE)
                                  .view(np.uint8).copy()).to(base.device)
    return n, fdescs


def rx_verify_dev(base, fdescs, flags: int = 0, stream=None):
    """lvlip_rx_verify_dev on frames in a CUDA uint8 tensor; returns the verdicts
    (uint8 CUDA tensor), asynchronously on `stream` (default: current)."""
    import torch

    n, fd = _frames_dev(base, fdescs)
    verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=base.device)
    s = stream or torch.cuda.current_stream(base.device)
    _check(_lib.lvlip_rx_verify_dev(base.data_ptr(), fd.data_ptr(), n, flags, verdict.data_ptr(),
                                    None, s.cuda_stream), "lvlip_rx_verify_dev")
    return verdict[:n]


def tx_checksum_dev(base, fdescs, stream=None):
    """lvlip_tx_checksum_dev in place on frames in a CUDA uint8 tensor; returns
    the per-frame status (1 filled, 0 malformed and untouched)."""
    import torch

    n, fd = _frames_dev(base, fdescs)
    status = torch.empty(max(n, 1), dtype=torch.uint8, device=base.device)
    s = stream or torch.cuda.current_stream(base.device)
    _check(_lib.lvlip_tx_checksum_dev(base.data_ptr(), fd.data_ptr(), n, status.data_ptr(),
                                      None, s.cuda_stream), "lvlip_tx_checksum_dev")
    return status[:n]


def icmp_echo_reply_dev(base, fdescs, stream=None, flags: int = 0):
    """lvlip_icmp_echo_reply_dev[_ex] (f4) in place on frames in a CUDA uint8
    tensor; returns the per-frame status (1 updated, 2 recomputed, 0
    untouched).  flags 0: the RFC 1624 update, exact for requests whose ICMP
    checksum verified (the caller's precondition); ECHO_FULL: icmpv4_reply's
    full recomputation for any request."""
    import torch

    n, fd = _frames_dev(base, fdescs)
    status = torch.empty(max(n, 1), dtype=torch.uint8, device=base.device)
    s = stream or torch.cuda.current_stream(base.device)
    if flags == 0:
        rc = _lib.lvlip_icmp_echo_reply_dev(base.data_ptr(), fd.data_ptr(), n, status.data_ptr(), s.cuda_stream)
    else:
        rc = _lib.lvlip_icmp_echo_reply_dev_ex(base.data_ptr(), fd.data_ptr(), n, flags, status.data_ptr(),
                                               s.cuda_stream)
    _check(rc, "lvlip_icmp_echo_reply_dev")
    return status[:n]


# ----------------------------------------------------- Group 4: several GPUs --

def partition_bytes(descs: np.ndarray, parts: int) -> list:
    """lvlip_partition_bytes: cuts[0..parts] of the byte-balanced contiguous
    partition (part p = descriptors [cuts[p], cuts[p+1]))."""
    d = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    cuts = np.zeros(parts + 1, dtype=np.uint32)
    _check(_lib.lvlip_partition_bytes(d.ctypes.data if d.size else None, d.size, parts, cuts.ctypes.data),
           "lvlip_partition_bytes")
    return [int(c) for c in cuts]


def batch_host_flat_multi(ctxs, base: np.ndarray, descs: np.ndarray) -> np.ndarray:
    """lvlip_csum_batch_host_flat_multi over Contexts (one per device, or
    several on one device), one host thread each."""
    base = _as_u8(base)
    d = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    out = np.empty(d.size, dtype=np.uint16)
    _check(_lib.lvlip_csum_batch_host_flat_multi(arr, len(ctxs), base.ctypes.data, base.size, d.ctypes.data,
                                                 d.size, out.ctypes.data), "lvlip_csum_batch_host_flat_multi")
    return out


def frames_variant_dev(mode: int, variant: int, base, fdescs, stream=None):
    """The frame calls' A/B variants (lvlip_lab_frames_dev, liblvlip_lab.so):
    mode 0 TX fill, 1 RX header on the flat sweep, 2 RX + L4; variant bits 1
    plain field stores, 2 eight loads per round, 4 block order; modes 4 / 5
    the echo reply (LVLIP_ECHO_FULL / flags 0) with the reply's store form as
    the variant (0 byte stores, 2-6 u16 stores with a cache policy).  Returns
    the per-frame status / verdict tensor."""
    import torch

    n, fd = _frames_dev(base, fdescs)
    out8 = torch.empty(max(n, 1), dtype=torch.uint8, device=base.device)
    s = stream or torch.cuda.current_stream(base.device)
    _check(lab().lvlip_lab_frames_dev(mode, variant, base.data_ptr(), fd.data_ptr(), n, out8.data_ptr(),
                                      s.cuda_stream), "lvlip_lab_frames_dev")
    return out8[:n]


def icmp_echo_reply_csum(req_csum: int) -> int:
    """f4 (RFC 1624): reply checksum field from a verified request's field, or
    CSUM_RECOMPUTE."""
    return int(_lib.lvlip_icmp_echo_reply_csum(req_csum & 0xFFFF))


def icmp_echo_reply_fill(frames) -> int:
    """In place: echo requests -> replies' ICMP part (type 0 + checksum).
    Returns how many needed a full recomputation; raises on a non-request."""
    arr, keep = frames_array(frames)
    r = int(_lib.lvlip_icmp_echo_reply_fill(arr, len(frames)))
    del keep
    if r == PLAN_MALFORMED:
        raise ValueError("not an ICMP echo request frame")
    return r


def rx_verify_cpu(frames, flags: int = 0) -> np.ndarray:
    """lvlip_rx_verify_cpu: the RX verdicts on the calling thread (no context)."""
    n = len(frames)
    arr, keep = frames_array(frames)
    verdict = np.zeros(max(n, 1), dtype=np.uint8)
    _check(_lib.lvlip_rx_verify_cpu(arr, n, flags, verdict.ctypes.data), "lvlip_rx_verify_cpu")
    del keep
    return verdict[:n]


def tx_checksum_cpu(frames) -> None:
    """lvlip_tx_checksum_cpu: the TX fill on the calling thread (no context)."""
    arr, keep = frames_array(frames)
    _check(_lib.lvlip_tx_checksum_cpu(arr, len(frames)), "lvlip_tx_checksum_cpu")
    del keep


def tx_apply(field: np.ndarray, csum: np.ndarray) -> None:
    f = np.ascontiguousarray(field, dtype=np.uint64)
    c = np.ascontiguousarray(csum, dtype=np.uint16)
    _lib.lvlip_tx_apply(f.size, f.ctypes.data, c.ctypes.data)


# ------------------------------------------------------------ host batches --

class Context:
    """lvlip_csum_ctx: pinned arena + device arena + streams, one thread at a time.

    cpu_max: host calls of at most this many packets / frames run on the
    calling thread with the library's CPU code (lvlip_csum_ctx_set_cpu_max);
    None keeps the library's default (LVLIP_CPU_MAX, else CPU_MAX_DEFAULT), 0
    sends every call to the GPU."""

    def __init__(self, device: int = 0, arena_bytes: int = 0, cpu_max: Optional[int] = None):
        self._h = ctypes.c_void_p()
        _check(_lib.lvlip_csum_ctx_create(ctypes.byref(self._h), device, arena_bytes),
               "lvlip_csum_ctx_create")
        if cpu_max is not None:
            self.set_cpu_max(cpu_max)

    def set_cpu_max(self, cpu_max: int) -> None:
        _check(_lib.lvlip_csum_ctx_set_cpu_max(self._h, int(cpu_max)), "lvlip_csum_ctx_set_cpu_max")

    @property
    def cpu_max(self) -> int:
        return int(_lib.lvlip_csum_ctx_cpu_max(self._h))

    def stats(self) -> dict:
        st = CtxStats()
        _check(_lib.lvlip_csum_ctx_stats(self._h, ctypes.byref(st)), "lvlip_csum_ctx_stats")
        return st.as_dict()

    def close(self) -> None:
        if self._h:
            _lib.lvlip_csum_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def batch_host(self, packets: Sequence, start_sums: Sequence[int]) -> np.ndarray:
        """packets: sequence of bytes-like / uint8 arrays (the skb payloads)."""
        n = len(packets)
        keep = [_as_u8(p) for p in packets]
        iov = (Iov * n)()
        for i, (a, s) in enumerate(zip(keep, start_sums)):
            iov[i].ptr = a.ctypes.data if a.size else None
            iov[i].len = a.size
            iov[i].start_sum = s & 0xFFFFFFFF
        out = np.empty(n, dtype=np.uint16)
        _check(_lib.lvlip_csum_batch_host(self._h, iov, n, out.ctypes.data),
               "lvlip_csum_batch_host")
        return out

    def batch_host_flat(self, base: np.ndarray, descs: np.ndarray) -> np.ndarray:
        base = _as_u8(base)
        descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
        n = descs.size
        out = np.empty(n, dtype=np.uint16)
        _check(_lib.lvlip_csum_batch_host_flat(self._h, base.ctypes.data, base.size,
                                               descs.ctypes.data, n, out.ctypes.data),
               "lvlip_csum_batch_host_flat")
        return out

    def register(self, buf: np.ndarray, flags: int = REG_DMA) -> None:
        """f3: pin `buf` (a contiguous uint8 array kept alive by the caller) in
        place; batches inside it skip the pinned-arena gather."""
        a = buf.view(np.uint8).reshape(-1)
        if not a.flags.c_contiguous:
            raise ValueError("register needs a contiguous buffer")
        _check(_lib.lvlip_csum_register(self._h, a.ctypes.data, a.size, flags),
               "lvlip_csum_register")

    def unregister(self, buf: np.ndarray) -> None:
        _check(_lib.lvlip_csum_unregister(self._h, buf.ctypes.data), "lvlip_csum_unregister")

    def rx_verify(self, frames, flags: int = 0) -> np.ndarray:
        """lvlip_rx_verify (f1): one verdict per frame (RX_*), frames untouched."""
        n = len(frames)
        arr, keep = frames_array(frames)
        verdict = np.zeros(max(n, 1), dtype=np.uint8)
        _check(_lib.lvlip_rx_verify(self._h, arr, n, flags, verdict.ctypes.data),
               "lvlip_rx_verify")
        del keep
        return verdict[:n]

    def tx_checksum(self, frames) -> None:
        """lvlip_tx_checksum (f2): fills TCP/ICMP and IPv4 checksums in place."""
        arr, keep = frames_array(frames)
        _check(_lib.lvlip_tx_checksum(self._h, arr, len(frames)), "lvlip_tx_checksum")
        del keep


# ------------------------------------------------------------------ testkit --

_testkit = None


def testkit() -> ctypes.CDLL:
    global _testkit
    if _testkit is None:
        tk = _load(TESTKIT_PATH)
        _stamp(tk, TESTKIT_PATH, "lvlip_testkit_build_id", os.path.join(HERE, "TESTKIT_SOURCES"))
        tk.lvlip_testkit_fill.restype = ctypes.c_int
        tk.lvlip_testkit_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_void_p]
        tk.lvlip_testkit_paint.restype = ctypes.c_int
        tk.lvlip_testkit_paint.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p]
        _testkit = tk
    return _testkit


_lab = None


def lab() -> ctypes.CDLL:
    """liblvlip_lab.so: read-bandwidth probes and the A/B kernels (diagnostics only)."""
    global _lab
    if _lab is None:
        lb = _load(LAB_PATH)
        _stamp(lb, LAB_PATH, "lvlip_lab_build_id", os.path.join(HERE, "LAB_SOURCES"))
        lb.lvlip_lab_probe.restype = ctypes.c_int
        lb.lvlip_lab_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p]
        lb.lvlip_lab_atomics.restype = ctypes.c_int
        lb.lvlip_lab_atomics.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint32, ctypes.c_void_p]
        lb.lvlip_lab_probe_tl.restype = ctypes.c_int
        lb.lvlip_lab_probe_tl.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p]
        lb.lvlip_lab_probe_chunk.restype = ctypes.c_int
        lb.lvlip_lab_probe_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_int, ctypes.c_void_p]
        lb.lvlip_lab_batch_dev_ex.restype = ctypes.c_int
        lb.lvlip_lab_batch_dev_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(LaunchCfg)]
        lb.lvlip_lab_frames_dev.restype = ctypes.c_int
        lb.lvlip_lab_frames_dev.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        lb.lvlip_lab_probe_pkwin.restype = ctypes.c_int
        lb.lvlip_lab_probe_pkwin.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lab = lb
    return _lab
