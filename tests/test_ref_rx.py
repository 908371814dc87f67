"""The RX oracle pinned to level-ip itself: oracle/skb_oracle.rx_verdict, the CPU
restatement the frame-batch tests check the GPU against, decides every frame the
way the reference's own ip_rcv does (src/ip_input.c:17-60, compiled from
/root/reference into oracle/_ref/libref.so and driven by tests/ref_rx_child.py).

Skipped when oracle/_ref was not built (it needs /root/reference at build time)."""
import os

import pytest

import pyoracle
import ref_rx_cases
import skb_oracle

pytestmark = pytest.mark.skipif(not os.path.exists(ref_rx_cases.REF_SO),
                                reason="oracle/_ref/libref.so not built")

EXPECTED = {"ok": skb_oracle.RX_OK, "ok_options": skb_oracle.RX_OK,
            "ip_csum": skb_oracle.RX_BAD_CSUM, "version": skb_oracle.RX_BAD_VERSION,
            "ihl": skb_oracle.RX_BAD_IHL, "ttl0": skb_oracle.RX_TTL0,
            "proto": skb_oracle.RX_UNKNOWN_PROTO, "icmp_csum": skb_oracle.RX_OK}


def test_rx_oracle_matches_reference_ip_rcv():
    frs, kinds = ref_rx_cases.frames(7)
    replies = ref_rx_cases.reference_replies(frs)
    for f, k, r in zip(frs, kinds, replies):
        v = skb_oracle.rx_verdict(f, 0)
        assert v == EXPECTED[k], k
        # ip_rcv hands the frame on (and the stack answers the echo) exactly when
        # the oracle says RX_OK
        assert (v == skb_oracle.RX_OK) == (r is not None), (k, v)
        if k == "icmp_csum":
            # level-ip answers a corrupted echo request (no ICMP RX verify,
            # src/icmpv4.c:11); the L4 check of the batch API is what catches it
            assert skb_oracle.rx_verdict(f, skb_oracle.RX_VERIFY_L4) == skb_oracle.RX_BAD_L4
        if k in ("ok", "icmp_csum"):
            # the reply the reference wrote verifies: IPv4 header and ICMP message
            ih = r[14:34]
            assert pyoracle.checksum(ih, 20, 0) == 0
            icmp = r[34:14 + int.from_bytes(ih[2:4], "big")]
            assert icmp[0] == 0 and pyoracle.checksum(icmp, len(icmp), 0) == 0
