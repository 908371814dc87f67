"""The host-resident GPU batch paths with AddressSanitizer on their host code.

tests/sanitize/build/ctx_asan (tests/sanitize/Makefile, built by
__graft_entry__.build()) is the product's own sources compiled with
`-Xarch_host -fsanitize=address` plus tests/sanitize/ctx_san.cpp: contexts with
a 1 MiB arena (many double-buffered pieces), scattered and flat batches,
DMA and zero-copy registered regions, the f1/f2 frame calls, a context per
thread, all on exact-size host allocations and checked against the oracle.
The device code objects are the plain gfx950 ones (no GPU sanitizer)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "sanitize", "build", "ctx_asan")


def test_host_batches_under_asan():
    if not os.path.exists(EXE):
        pytest.fail("tests/sanitize/build/ctx_asan missing: run __graft_entry__.build()")
    # the HIP runtime keeps allocations for the process lifetime: leaks are not ours to report
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "all checks passed" in r.stdout
    # built from this tree's product sources (the same hash as the library's)
    import lvlip

    assert f"build_id: {lvlip.source_build_id()}" in r.stdout, r.stdout[:200]
