"""CPU restatement of level-ip's per-frame checksum decisions.

TEST INFRASTRUCTURE ONLY — the checker for include/lvlip_skb.h.  Imported by
tests/ only; the product never imports it.  Every checksum goes through
pyoracle.checksum (csum_oracle.c, pinned against the reference's golden
vectors); what is restated here is only which bytes are summed, with which
seed, and in which order the drop decisions are taken.

  rx_verdict(frame, flags)   netdev_receive (src/netdev.c:67-80) + ip_rcv
                             (src/ip_input.c:17-60); optional L4 verify with
                             the RFC 1071 pseudo-header seed
  tx_fill(frame)             tcp_transmit_skb (src/tcp_output.c:110,126 ->
                             src/tcp.c:87-98), icmpv4_reply (src/icmpv4.c:46-47),
                             ip_output (src/ip_output.c:42,53 -> ip_send_check,
                             src/ip_output.c:8-12); fields zeroed, then summed,
                             stored raw (native LE u16)
"""
from __future__ import annotations

import struct

import pyoracle

ETH = 14
RX_OK, RX_NOT_IP, RX_SHORT, RX_BAD_VERSION, RX_BAD_IHL, RX_TTL0, RX_BAD_CSUM, RX_BAD_L4, \
    RX_UNKNOWN_PROTO = range(1, 10)
RX_VERIFY_L4 = 0x1


def pseudo_sum_rfc(saddr: int, daddr: int, proto: int, length: int) -> int:
    """Pseudo header as 16-bit halves: the same words src/tcp.c:92-95 adds, no lost carry."""
    sw = lambda x: ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)
    return ((saddr & 0xFFFF) + (saddr >> 16) + (daddr & 0xFFFF) + (daddr >> 16) + sw(proto) +
            sw(length & 0xFFFF))


def rx_verdict(frame: bytes, flags: int = 0) -> int:
    f = bytes(frame)
    if len(f) < ETH + 20:
        return RX_SHORT
    if struct.unpack_from(">H", f, 12)[0] != 0x0800:  # src/netdev.c:67-80
        return RX_NOT_IP
    ih = f[ETH:]
    version, ihl = ih[0] >> 4, ih[0] & 0xF
    if version != 4:  # src/ip_input.c:22
        return RX_BAD_VERSION
    if ihl < 5:  # src/ip_input.c:27
        return RX_BAD_IHL
    if ih[8] == 0:  # src/ip_input.c:32
        return RX_TTL0
    if len(ih) < ihl * 4:
        return RX_SHORT
    if pyoracle.checksum(ih[: ihl * 4], ihl * 4, 0) != 0:  # src/ip_input.c:38-43
        return RX_BAD_CSUM
    proto = ih[9]
    if proto not in (1, 6):  # src/ip_input.c:51-60
        return RX_UNKNOWN_PROTO
    if flags & RX_VERIFY_L4:
        iplen = struct.unpack_from(">H", ih, 2)[0]
        if iplen < ihl * 4 or len(ih) < iplen:
            return RX_SHORT
        l4 = ih[ihl * 4: iplen]
        seed = 0
        if proto == 6:
            saddr, daddr = struct.unpack_from("<II", ih, 12)
            seed = pseudo_sum_rfc(saddr, daddr, 6, len(l4))
        if pyoracle.checksum(l4, len(l4), seed) != 0:
            return RX_BAD_L4
    return RX_OK


def tx_fill(frame: bytearray) -> None:
    """Fills the checksums of one built frame the way the reference's TX path does."""
    ih_off = ETH
    ih = frame[ih_off:]
    ihl = ih[0] & 0xF
    iplen = struct.unpack_from(">H", ih, 2)[0]
    proto = ih[9]
    l4_off = ih_off + ihl * 4
    l4len = iplen - ihl * 4
    if proto == 6 and l4len >= 20:
        frame[l4_off + 16: l4_off + 18] = b"\0\0"  # thdr->csum = 0
        saddr, daddr = struct.unpack_from("<II", frame, ih_off + 12)
        c = pyoracle.checksum(bytes(frame[l4_off: l4_off + l4len]), l4len,
                              pyoracle.pseudo_sum(saddr, daddr, 6, l4len))
        frame[l4_off + 16: l4_off + 18] = struct.pack("<H", c)
    elif proto == 1 and l4len >= 4:
        frame[l4_off + 2: l4_off + 4] = b"\0\0"  # icmp->csum = 0
        c = pyoracle.checksum(bytes(frame[l4_off: l4_off + l4len]), l4len, 0)
        frame[l4_off + 2: l4_off + 4] = struct.pack("<H", c)
    frame[ih_off + 10: ih_off + 12] = b"\0\0"  # ihdr->csum = 0
    c = pyoracle.checksum(bytes(frame[ih_off: ih_off + ihl * 4]), ihl * 4, 0)
    frame[ih_off + 10: ih_off + 12] = struct.pack("<H", c)
