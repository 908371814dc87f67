"""Synthetic packet batches of BASELINE.json's configurations.

Every byte and descriptor is a pure function of (seed, global index), so a
rank's shard of a multi-GPU batch is exactly the corresponding slice of the
single-GPU batch, and the CPU side regenerates the same bytes as the GPU.

  tcp1500  1 M x 1500 B TCP segments (MTU), 16-B aligned slots (stride 1504)
  tcp9000  1 M x 9000 B TCP segments (jumbo), 16-B aligned slots (stride 9008)
  mixed    2 M frames = 4 M descriptors: a 20-B IPv4 header at frame+14 and an
           ICMP or TCP payload of U[64,1460] B (odd lengths included) at frame+34,
           the skb layout of include/ip.h:47-50 / include/tcp.h:224-227 (2 mod 4)

Per packet: TCP start_sum = saddr + daddr + htons(6) + htons(len) with u32 wrap
(src/tcp.c:92-95) from random saddr/daddr, so ~half the packets lose the
carry exactly as the reference does; IPv4 headers and ICMP use 0.  1 % of the
packets (frames) are all-0x00 and 1 % all-0xff (adversarial fold cases).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED = 0x1E7E1C5
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_FILL_MUL = np.uint64(0xD1B54A32D192ED03)

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<i4"), ("start_sum", "<u4")])


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def subseed(seed: int, k: int) -> int:
    return int(splitmix64(np.array([seed ^ k], dtype=np.uint64))[0])


def fill_bytes(nbytes: int, seed: int = SEED, first_byte: int = 0) -> np.ndarray:
    """Byte stream of oracle_fill / testkit k_fill (first_byte multiple of 8)."""
    assert first_byte % 8 == 0
    nwords = (nbytes + 7) // 8
    j = np.arange(first_byte // 8, first_byte // 8 + nwords, dtype=np.uint64)
    with np.errstate(over="ignore"):
        w = splitmix64(np.uint64(seed) ^ (j * _FILL_MUL))
    return w.view(np.uint8)[:nbytes].copy()


def bswap16(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint32) & np.uint32(0xFFFF)
    return ((x << np.uint32(8)) | (x >> np.uint32(8))) & np.uint32(0xFFFF)


def pseudo_sum(saddr, daddr, proto: int, length) -> np.ndarray:
    """src/tcp.c:92-95 vectorised: u32 wrap-around, carry out of bit 31 lost."""
    s = (np.asarray(saddr, dtype=np.uint64) + np.asarray(daddr, dtype=np.uint64)
         + np.uint64(int(bswap16(np.array([proto]))[0])) + bswap16(length).astype(np.uint64))
    return (s & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def align16(x):
    return (x + 15) & ~15


@dataclass
class Batch:
    name: str
    descs: np.ndarray       # DESC_DTYPE[n], offsets relative to this shard's buffer
    nbytes: int             # buffer bytes (multiple of 16, covers every chunk)
    paint: np.ndarray       # uint8[n]: 0 keep, 1 all-0x00, 2 all-0xff
    first_byte: int         # global stream offset of this shard's buffer (for fill)
    algo_bytes: int         # sum of packet lengths (the roofline's algorithmic read bytes)

    @property
    def n(self) -> int:
        return int(self.descs.size)

    def host_bytes(self, seed: int = SEED) -> np.ndarray:
        """The buffer exactly as testkit fill + paint produce it on the GPU."""
        buf = fill_bytes(self.nbytes, seed, self.first_byte)
        for i in np.nonzero(self.paint)[0]:
            d = self.descs[i]
            if d["len"] > 0:
                buf[int(d["offset"]): int(d["offset"]) + int(d["len"])] = (
                    0x00 if self.paint[i] == 1 else 0xFF)
        return buf


def _paint(idx: np.ndarray, seed: int) -> np.ndarray:
    h = splitmix64(np.uint64(subseed(seed, 3)) ^ idx.astype(np.uint64)) % np.uint64(100)
    p = np.zeros(idx.size, dtype=np.uint8)
    p[h == 0] = 1
    p[h == 1] = 2
    return p


def uniform(n: int, length: int, first: int = 0, seed: int = SEED, stride: int | None = None,
            name: str | None = None) -> Batch:
    """Packets first..first+n-1 of an unbounded uniform TCP-segment stream."""
    stride = align16(length) if stride is None else stride
    idx = np.arange(first, first + n, dtype=np.uint64)
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    d["len"] = length
    sd = splitmix64(np.uint64(subseed(seed, 1)) ^ idx)
    d["start_sum"] = pseudo_sum(sd & np.uint64(0xFFFFFFFF), sd >> np.uint64(32), 6,
                                np.full(n, length, dtype=np.uint32))
    nbytes = align16((n - 1) * stride + length) if n else 16
    first_byte = first * stride
    return Batch(name or f"tcp{length}", d, int(nbytes), _paint(idx, seed), int(first_byte),
                 int(n) * int(length))


def mixed(frames: int, first: int = 0, seed: int = SEED) -> Batch:
    """Config #4: header + payload descriptor pairs in skb layout, frames first..first+frames-1.

    Offsets are relative to this shard's buffer; frames are packed at 16-B aligned
    starts.  Descriptors (lengths, seeds, paint) of a shard equal the matching
    slice of the full batch; the filler bytes of a shard come from its own stream
    origin (first * 2048), so a shard is a self-contained valid batch.
    """
    idx = np.arange(first, first + frames, dtype=np.uint64)
    h = splitmix64(np.uint64(subseed(seed, 2)) ^ idx)
    plen = (np.uint64(64) + h % np.uint64(1397)).astype(np.int64)       # 64..1460
    tcp = ((h >> np.uint64(20)) & np.uint64(1)).astype(bool)
    fsize = align16(34 + plen)
    fstart = np.concatenate([[0], np.cumsum(fsize)[:-1]]).astype(np.uint64)
    d = np.zeros(2 * frames, dtype=DESC_DTYPE)
    d["offset"][0::2] = fstart + np.uint64(14)
    d["len"][0::2] = 20
    d["start_sum"][0::2] = 0
    d["offset"][1::2] = fstart + np.uint64(34)
    d["len"][1::2] = plen
    sd = splitmix64(np.uint64(subseed(seed, 1)) ^ idx)
    ps = pseudo_sum(sd & np.uint64(0xFFFFFFFF), sd >> np.uint64(32), 6, plen.astype(np.uint32))
    d["start_sum"][1::2] = np.where(tcp, ps, np.uint32(0))
    fp = _paint(idx, seed)
    paint = np.repeat(fp, 2)
    nbytes = int(align16(int(fstart[-1]) + int(fsize[-1]))) if frames else 16
    first_byte = int(first) * 2048
    return Batch("mixed", d, nbytes, paint, first_byte, int(20 * frames + plen.sum()))


CONFIGS = {
    "tcp1500": lambda first=0, n=1 << 20: uniform(n, 1500, first, name="tcp1500"),
    "tcp9000": lambda first=0, n=1 << 20: uniform(n, 9000, first, name="tcp9000"),
    "mixed": lambda first=0, n=1 << 21: mixed(n, first),
    # config #5: 64 M x 1500 B = 96 GB, fits one 288 GB MI355X; strong scaling
    "tcp1500x64m": lambda first=0, n=64 << 20: uniform(n, 1500, first, name="tcp1500x64m"),
}
# layout variants of configs[1] for the lab scripts (slot stride: packed,
# 128-B lines, 2 KiB NIC-style buffers); not bench workloads
for _st in (1500, 1536, 2048):
    CONFIGS[f"tcp1500_s{_st}"] = (lambda st: lambda first=0, n=1 << 20: uniform(
        n, 1500, first, stride=st, name=f"tcp1500_s{st}"))(_st)
# uniform small segments (~1.6 GB each) for the flat sweep's lab A/Bs
for _ln in (64, 128, 160, 192, 224, 256, 512):
    CONFIGS[f"tcp{_ln}"] = (lambda ln: lambda first=0, n=None: uniform(
        n or (1600 << 20) // align16(ln), ln, first, name=f"tcp{ln}"))(_ln)


def make(name: str, n: int | None = None, first: int = 0) -> Batch:
    f = CONFIGS[name]
    return f(first) if n is None else f(first, n)


# ------------------------------------------------------------ device side --

def to_device(b: Batch, device="cuda", seed: int = SEED, stream=None):
    """Materialise a Batch in HBM: bytes generated on the GPU by the testkit
    (identical to Batch.host_bytes()), descriptors and paint uploaded.
    Returns (base_u8, descs_u8, out_i16) torch tensors."""
    import torch

    import lvlip

    tk = lvlip.testkit()
    nbytes = (b.nbytes + 15) & ~15
    base = torch.empty(nbytes, dtype=torch.uint8, device=device)
    s = (stream or torch.cuda.current_stream(base.device)).cuda_stream
    rc = tk.lvlip_testkit_fill(base.data_ptr(), nbytes & ~7, seed, b.first_byte, s)
    if rc != 0:
        raise RuntimeError(f"testkit fill failed: {rc}")
    descs = torch.from_numpy(b.descs.view(np.uint8).copy()).to(device)
    if b.paint.any():
        paint = torch.from_numpy(b.paint).to(device)
        rc = tk.lvlip_testkit_paint(base.data_ptr(), descs.data_ptr(), paint.data_ptr(), b.n, s)
        if rc != 0:
            raise RuntimeError(f"testkit paint failed: {rc}")
    out = torch.empty(b.n, dtype=torch.int16, device=device)
    return base, descs, out


# ------------------------------------------------------------------ frames --

def frames(n: int, seed: int = SEED, max_l4: int = 1480, options: bool = True,
           protos=(6, 1)) -> list[bytearray]:
    """n Ethernet/IPv4 frames as level-ip builds them (include/skbuff.h:9-23):
    14-B Ethernet header, IPv4 header (ihl 5, or up to 15 with options), then a
    TCP (>= 20 B) or ICMP (>= 8 B) segment of random, often odd, length.  Every
    checksum field holds garbage; bytes past the IP total length (Ethernet
    padding) are random too.  Used by the f1/f2 tests (include/lvlip_skb.h)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        proto = int(rng.choice(protos))
        ihl = int(rng.integers(6, 16)) if options and rng.random() < 0.2 else 5
        lo = 20 if proto == 6 else 8
        l4 = int(rng.integers(lo, max(lo, max_l4) + 1))
        pad = int(rng.integers(0, 8)) if rng.random() < 0.3 else 0
        iplen = ihl * 4 + l4
        f = bytearray(rng.integers(0, 256, 14 + iplen + pad, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00"
        f[14] = 0x40 | ihl
        f[16:18] = iplen.to_bytes(2, "big")
        f[22] = int(rng.integers(1, 256))  # ttl != 0
        f[23] = proto
        if proto == 1:
            f[14 + ihl * 4] = 8  # echo request
        out.append(f)
    return out
