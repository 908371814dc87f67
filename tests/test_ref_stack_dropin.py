"""The reference stack itself, running on the drop-in checksum (north_star: "keeping
the existing call sites in src/ip_input.c, src/ip_output.c, src/tcp.c and
src/icmpv4.c").

oracle/_ref/libref_dropin.so is level-ip's own objects (every src/*.c but main.c,
compiled from /root/reference by oracle/Makefile) with src/utils.c's checksum()
and sum_every_16bits() made local, linked against level-ip_amd/liblvlip_csum.so.
The call sites are unchanged object code; at load time they bind to the product
library.  These tests drive that stack and require the bytes it writes to equal
the fixtures the unmodified reference wrote (tests/golden/).

Skipped when oracle/_ref was not built (it needs /root/reference at build time)."""
import ctypes
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_io
import pyoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "libref_dropin.so")

pytestmark = pytest.mark.skipif(not os.path.exists(DROPIN),
                                reason="oracle/_ref/libref_dropin.so not built")


def test_call_sites_bind_to_the_product(tmp_path):
    """Config #1 through the reference stack on the drop-in: ARP, then four echo
    requests into ip_rcv (src/ip_input.c:38 verifies the header) -> icmpv4_reply
    (src/icmpv4.c:47) -> ip_output (src/ip_output.c:53) -> tun_write.  Every frame
    the stack writes equals the reference's own, and the dynamic linker reports
    `checksum` bound from libref_dropin.so to liblvlip_csum.so."""
    out = tmp_path / "echo.json"
    env = dict(os.environ, LD_DEBUG="bindings", LD_DEBUG_OUTPUT=str(tmp_path / "ld"))
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "golden", "make_golden.py"),
                    "--echo-child", str(out), DROPIN],
                   check=True, stdin=subprocess.DEVNULL, env=env, timeout=120)
    got = json.loads(out.read_text())
    want = golden_io.echo()
    assert got["arp_reply_hex"] == want["arp_reply_hex"]
    assert len(got["echo"]) == len(want["echo"]) >= 4
    for g, w in zip(got["echo"], want["echo"]):
        assert g["request_hex"] == w["request_hex"]
        assert g["reply_hex"] == w["reply_hex"], g["data_len"]

    bound, back = [], []
    for fn in glob.glob(str(tmp_path / "ld*")):
        with open(fn, errors="replace") as f:
            for ln in f:
                if "binding file" not in ln:
                    continue
                if "libref_dropin.so [0] to" in ln and "`checksum'" in ln:
                    bound.append(ln)
                # the product binds its own internals (-Bsymbolic-functions): the
                # host's tcp_udp_checksum/checksum never interpose inside it
                if "liblvlip_csum.so [0] to" in ln and "libref_dropin.so" in ln.split(" to ")[1]:
                    back.append(ln)
    assert bound, "no binding of checksum from libref_dropin.so was logged"
    assert all("liblvlip_csum.so" in ln for ln in bound), bound[:3]
    assert not back, back[:3]


def test_reference_tcp_transmit_on_the_dropin(tmp_path):
    """level-ip's TCP transmit path on the drop-in (tests/ref_stack_child.py):
    SYN with options, a SYN retransmit, four data segments of 536/536/536/393 B,
    a bare ACK and a RST, each checksummed at src/tcp_output.c:126 and
    src/ip_output.c:53 through the product.  Every frame's TCP checksum equals
    the unmodified reference's tcp_udp_checksum (oracle/_ref/libref.so) over the
    same segment, and its IPv4 header verifies to 0 as ip_rcv requires."""
    out = tmp_path / "tcp.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_stack_child.py"),
                    str(out), DROPIN], check=True, stdin=subprocess.DEVNULL, timeout=120)
    d = json.loads(out.read_text())
    ref = pyoracle.reflib()
    assert ref is not None
    frames = [bytes.fromhex(f) for f in d["frames"]]
    assert len(frames) == 8
    data = b""
    for fr in frames:
        ip = fr[14:34]
        assert ip[9] == 6 and pyoracle.checksum(ip, 20, 0) == 0
        ref_ip = bytearray(ip)
        ref_ip[10:12] = b"\0\0"
        buf = (ctypes.c_char * 20).from_buffer(ref_ip)
        ref.ip_send_check(ctypes.addressof(buf))
        del buf
        assert bytes(ref_ip) == ip
        seg = bytearray(fr[34:14 + int.from_bytes(ip[2:4], "big")])
        want = bytes(seg[16:18])
        seg[16:18] = b"\0\0"
        saddr = int.from_bytes(ip[12:16], "little")  # htonl(sk->saddr) as stored
        daddr = int.from_bytes(ip[16:20], "little")
        got = ref.tcp_udp_checksum(saddr, daddr, 6, bytes(seg), len(seg)) & 0xFFFF
        assert got.to_bytes(2, "little") == want
        data += bytes(seg[(seg[12] >> 4) * 4:])
    assert frames[0][47] & 0x02 and frames[1][47] & 0x02  # SYN, SYN again
    assert frames[-1][47] & 0x04  # RST
    assert data == bytes.fromhex(d["payload_hex"])
    assert [len(f) - 54 for f in frames[2:6]] == [536, 536, 536, 393]


def _dropin():
    lib = ctypes.CDLL(DROPIN)
    lib.tcp_udp_checksum.restype = ctypes.c_int
    lib.tcp_udp_checksum.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                     ctypes.c_void_p, ctypes.c_uint16]
    lib.ip_send_check.restype = None
    lib.ip_send_check.argtypes = [ctypes.c_void_p]
    return lib


def test_reference_tcp_udp_checksum_on_the_dropin():
    """src/tcp.c:87-98 as compiled from the reference (pseudo-header sum with the
    lost carry, then checksum() -> the product) on every golden TCP/UDP case."""
    lib = _dropin()
    t = golden_io.tcp()
    for i in range(t["len"].size):
        off, ln = int(t["offset"][i]), int(t["len"][i])
        seg = np.ascontiguousarray(t["blob"][off:off + max(ln, 1)])
        got = lib.tcp_udp_checksum(int(t["saddr"][i]), int(t["daddr"][i]), int(t["proto"][i]),
                                   seg.ctypes.data, ln) & 0xFFFF
        assert got == int(t["expected"][i]), i


def test_reference_ip_send_check_on_the_dropin():
    """src/ip_output.c:8-12 as compiled from the reference on every golden header
    (ihl 5..15): the field it writes equals the reference's."""
    lib = _dropin()
    h = golden_io.iphdr()
    for hdr, after in zip(h["hdr"], h["after"]):
        b = bytearray(hdr.tobytes())
        c = (ctypes.c_char * len(b)).from_buffer(b)
        lib.ip_send_check(ctypes.addressof(c))
        del c
        assert bytes(b) == after.tobytes()
