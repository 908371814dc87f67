"""The C-ABI boundary: the library loads, exports exactly what include/*.h
declares, and rejects bad arguments without touching a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import lvlip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lvlip_csum.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "lvlip_skb.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names += re.findall(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("defined",)))


def test_header_declares_the_reference_names():
    names = declared_functions()
    # include/utils.h:13-14 drop-ins
    assert "checksum" in names and "sum_every_16bits" in names
    for n in ("lvlip_csum_batch_dev", "lvlip_csum_batch_dev_ex", "lvlip_csum_batch_host",
              "lvlip_csum_batch_host_flat", "lvlip_csum_ctx_create", "lvlip_csum_ctx_destroy",
              "lvlip_pseudo_sum"):
        assert n in names


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    exported = subprocess.run(["nm", "-D", "--defined-only", lvlip.LIB_PATH], check=True,
                              capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in exported.splitlines() if " T " in l}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # and nothing else leaks (kernel stubs, C++ helpers)
    extra = sorted(exported - set(names))
    assert not extra, extra
    for n in names:
        assert hasattr(lvlip.lib(), n)


def test_header_is_plain_c():
    # compiles as C99 with no HIP/torch headers on the include path
    for h in HEADERS:
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only",
                            "-I", os.path.dirname(h), "-x", "c", "-"],
                           input=f'#include "{h}"\nint main(void){{return 0;}}\n', text=True,
                           capture_output=True)
        assert r.returncode == 0, r.stderr
        body = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        assert not re.search(r"\bhip\w*_t\b|#include\s*<hip", body)
        assert "torch" not in body.lower()


def test_desc_layout():
    assert lvlip.DESC_DTYPE.itemsize == 16
    assert ctypes.sizeof(lvlip.LaunchCfg) == 16
    assert lvlip.lib().lvlip_abi_version() == 2


def test_error_paths_without_gpu():
    L = lvlip.lib()
    out = np.zeros(4, dtype=np.uint16)
    # NULL pointers / misaligned base -> EINVAL before any HIP call
    assert L.lvlip_csum_batch_dev(None, None, 4, out.ctypes.data, None) == lvlip.EINVAL
    assert L.lvlip_csum_batch_dev(1, 16, 4, out.ctypes.data, None) == lvlip.EINVAL
    # n == 0 is a no-op success
    assert L.lvlip_csum_batch_dev(None, None, 0, None, None) == lvlip.OK
    assert L.lvlip_csum_ctx_destroy(None) == lvlip.EINVAL
    assert L.lvlip_csum_register(None, 4096, 4096, 0) == lvlip.EINVAL
    assert L.lvlip_csum_unregister(None, 4096) == lvlip.EINVAL
    assert L.lvlip_strerror(lvlip.ERANGE) == b"batch exceeds context arena"
    cfg = lvlip.LaunchCfg(99, 0, 0, 0)
    assert L.lvlip_csum_batch_dev_ex(16 * 1024, 16, 1, 16, None, ctypes.byref(cfg)) == lvlip.EINVAL


def test_no_device_context_fails_loudly():
    if lvlip.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(lvlip.LvlipError) as e:
        lvlip.Context(0)
    assert "no HIP device" in str(e.value)


def test_gfx950_code_object_present():
    # the kernels are cross-compiled for gfx950 only (no other offload targets)
    blob = open(lvlip.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx\w+)", blob))
    assert targets == {b"gfx950"}, targets


def test_integration_index_names_every_declared_function():
    """INTEGRATION.md §6 maps each entry point to the level-ip interface it
    replaces; a function added to include/*.h without a row there fails here."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    index = doc.split("## 6. Entry-point index", 1)[1]
    missing = [f for f in declared_functions() if f"`{f}`" not in index]
    assert not missing, missing


def test_auto_selection_table():
    """LVLIP_KERNEL_AUTO's choice by length hint (DESIGN.md §4's table), as
    lvlip_auto_kernel reports it; no compute, so it runs without a GPU (the
    window shapes assume 256 CUs there)."""
    flat, window, lane = lvlip.KERNEL_FLAT, lvlip.KERNEL_WINDOW, lvlip.KERNEL_LANE
    n = 1 << 20
    for hint, kernel, unroll in ((0, flat, 8), (1, lane, 4 | (2 << 8) | (2 << 16)),
                                 (32, lane, 4 | (2 << 8) | (2 << 16)), (33, flat, 2), (39, flat, 2),
                                 (40, flat, 4), (175, flat, 4), (176, flat, 8), (391, flat, 8),
                                 (895, flat, 8)):
        cfg = lvlip.auto_kernel(hint, n)
        assert (cfg.kernel, cfg.unroll) == (kernel, unroll), hint
    for hint, wpc, g in ((896, 16, 4), (1500, 12, 4), (1792, 8, 2), (9000, 8, 3)):
        cfg = lvlip.auto_kernel(hint, n)
        assert cfg.kernel == window and cfg.waves_per_cu == wpc, hint
        assert cfg.unroll == 2 | (g << 8), hint
    # a batch launched as pieces: nothing for an empty one, one launch for a
    # flat batch up to 2^30 descriptors
    assert lvlip.batch_launches(0) == 0
    assert lvlip.batch_launches(1 << 20, lvlip.KERNEL_FLAT, len_hint=391) == 1


def test_stale_or_unstamped_helper_library_refused(tmp_path):
    """VERDICT r03 Next #6 / ADVICE r03: the lab and testkit libraries carry
    source stamps like the product; a library without the stamp symbol (built
    before stamps) or with another stamp raises LvlipUnavailable with the
    rebuild hint instead of running stale A/B code."""
    libc = ctypes.CDLL("libc.so.6")
    with pytest.raises(lvlip.LvlipUnavailable, match="no lvlip_lab_build_id"):
        lvlip._stamp(libc, "libc.so.6", "lvlip_lab_build_id", os.path.join(lvlip.HERE, "LAB_SOURCES"))
    other = tmp_path / "SOURCES"
    other.write_text("include/lvlip_csum.h\n")
    lab = ctypes.CDLL(lvlip.LAB_PATH)
    with pytest.raises(lvlip.LvlipUnavailable, match="other sources"):
        lvlip._stamp(lab, lvlip.LAB_PATH, "lvlip_lab_build_id", str(other))
    # the tree's own builds pass
    assert lvlip.lab() is not None and lvlip.testkit() is not None
    for so, lst in (("liblvlip_lab.so", "LAB_SOURCES"), ("liblvlip_testkit.so", "TESTKIT_SOURCES")):
        assert lvlip.source_build_id(os.path.join(lvlip.HERE, lst)).encode() in open(
            os.path.join(lvlip.HERE, so), "rb").read()
