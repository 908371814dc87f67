"""ISA guards for the stream kernels (CPU-only: hipcc cross-compiles gfx950).

The stream kernels rely on hand-placed inline asm (the ring of csum_dev.h, run
by k_window in the product, csum_kernels.hip, and by k_stream in the lab
library, lab_kernels.hip):
  * buffer_load_dwordx4 whose resource words come from v_readfirstlane, a VALU
    write of SGPRs: a VMEM read of them needs 5 wait states (s_nop 4), which
    hipcc does not insert around inline asm;
  * an LDS-DMA whose M0 is written just before it (needs a wait state);
  * a ring of R two-load pieces retired by vmcnt(2(R-1)): hipcc must not add
    draining waits.
These checks read the generated assembly and fail if any of that regresses.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "level-ip_amd", "csrc", f) for f in ("csum_kernels.hip", "lab_kernels.hip")]
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def asm():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    text = []
    with tempfile.TemporaryDirectory() as d:
        for i, src in enumerate(SRCS):
            out = os.path.join(d, f"k{i}.s")
            subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17",
                            "-I" + os.path.join(ROOT, "include"), "-S", "--cuda-device-only",
                            src, "-o", out], check=True, capture_output=True)
            text.append(open(out).read())
    return "\n".join(text)


def functions(text):
    """name -> list of instruction lines (comments/labels/directives dropped),
    from the function's label to its .Lfunc_end marker (a kernel with an early
    return has more than one s_endpgm)."""
    funcs, cur, name = {}, None, None
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, cur = m.group(1), []
            funcs[name] = cur
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        cur.append(s)
    return funcs


def stream_kernels(asm):
    """k_stream and k_window instantiations (the ring kernels, one body)."""
    f = functions(asm)
    ks = {n: body for n, body in f.items() if "k_stream" in n or "k_window" in n}
    # k_stream<R, POL>: 2-4 pieces in flight, the five load policies
    st = {tuple(int(x) for x in re.search(r"k_streamILi(\d+)ELi(\d+)E", n).groups())
          for n in ks if "k_stream" in n}
    assert st == {(r, p) for r in (2, 3, 4) for p in range(5)}, sorted(st)
    # k_window<R, G>: every pieces-in-flight x group-size pair the launcher uses
    win = {tuple(int(x) for x in re.search(r"k_windowILi(\d+)ELi(\d+)E", n).groups())
           for n in ks if "k_windowI" in n}
    # the lab's stamped k_window (same ring, 4 / 8 / 12 waves per workgroup)
    assert any("k_window_stamp" in n for n in ks)
    assert win == {(r, g) for r in (2, 3, 4) for g in (1, 2, 3, 4, 8)}, sorted(win)
    return ks


def pieces(name):
    """R (pieces in flight) of a k_stream / k_window instantiation."""
    return int(re.search(r"k_(?:stream|window|window_stamp|window_dyn)ILi(\d+)E", name).group(1))


def test_buffer_loads_padded_against_valu_sgpr_hazard(asm):
    for name, body in stream_kernels(asm).items():
        n = 0
        for i, ins in enumerate(body):
            if ins.startswith("buffer_load_dwordx4") and " offen" in ins:
                n += 1
                assert body[i - 1] == "s_nop 4", (name, i, body[i - 3:i + 1])
        assert n >= 2, name


def test_lds_dma_m0_sequence(asm):
    for name, body in stream_kernels(asm).items():
        n = 0
        for i, ins in enumerate(body):
            if ins.startswith("global_load_lds_dwordx4"):
                n += 1
                assert body[i - 1] == "s_nop 0", (name, body[i - 3:i + 1])
                assert body[i - 2].startswith("s_mov_b32 m0,"), (name, body[i - 3:i + 1])
                assert body[i - 3] == "s_nop 4", (name, body[i - 4:i + 1])
            elif "m0" in re.split(r"[\s,]+", ins):
                assert ins.startswith("s_mov_b32 m0,") and body[i + 2].startswith(
                    "global_load_lds"), (name, ins)
        assert n >= 2, name


def test_ring_waits_are_counted_not_draining(asm):
    for name, body in stream_kernels(asm).items():
        r = pieces(name)
        waits = [ins for ins in body if ins.startswith("s_waitcnt") and "vmcnt" in ins]
        ring = [w for w in waits if f"vmcnt({2 * (r - 1)})" in w]
        assert len(ring) == r, (name, waits)
        # one drain after the first window fill, one before s_endpgm
        drains = [ins for ins in body if ins.startswith("s_waitcnt") and "vmcnt(0)" in ins]
        assert len(drains) <= 2, (name, waits)


def test_pipelined_flat_sweep_registers_not_read_in_flight(asm):
    """The lab's pipelined k_flat2 sweep (FLAT unroll bit 11): no path from a
    ring load to its retiring wait touches the load's destination registers
    (the bank-across-the-back-edge version failed this and the parity tests)."""
    from isa_inflight import inflight_hazards

    f = functions_with_labels(asm)
    ks = {n: b for n, b in f.items() if "k_flat2" in n and "DescSrcELi1ELb1E" in n}
    assert len(ks) == 4, sorted(ks)
    for name, body in ks.items():
        h = inflight_hazards(body, r"global_load_dwordx4 v\[\d+:\d+\], v\[\d+:\d+\], off nt")
        assert not h, (name, h[:3])


def functions_with_labels(text):
    """name -> instruction lines with block labels kept (for the flow check)."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = []
            funcs[m.group(1)] = cur
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.split(";")[0].strip()
        if not s or (s.startswith(".") and not s.endswith(":")):
            continue
        cur.append(s)
    return funcs


def test_no_scratch(asm):
    for m in re.finditer(r"\.name:\s+(_Z\w*k_(?:stream|window)\w*)\n(?:.*\n){0,60}?\s+\.private_segment_fixed_size:\s+(\d+)",
                         asm):
        assert int(m.group(2)) == 0, m.group(1)
