import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "level-ip_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

# A context's host calls of at most cpu_max packets / frames run on the CPU
# (include/lvlip_csum.h, lvlip_csum_ctx_set_cpu_max).  The parity tests are
# about the GPU path, so their contexts send every call to the GPU; the
# dispatch tests (test_dispatch_gpu.py, test_ref_*_batch.py) set the
# threshold, or remove this, explicitly.
os.environ.setdefault("LVLIP_CPU_MAX", "0")

def _may_rebuild() -> bool:
    """Whether a stale library is rebuilt here or stops the run.
    LVLIP_REBUILD=1 / 0 decides explicitly; by default a machine without a GPU
    (no /dev/kfd: the build container) rebuilds, and a GPU box, which runs the
    prebuilt snapshot and must not build inside a GPU run, refuses."""
    e = os.environ.get("LVLIP_REBUILD")
    if e in ("0", "1"):
        return e == "1"
    return not os.path.exists("/dev/kfd")


def _source_build_id(list_name: str = "BUILD_SOURCES") -> str:
    """lvlip.source_build_id() without importing lvlip (which loads the library)."""
    import hashlib

    h = hashlib.sha256()
    with open(os.path.join(PKG, list_name)) as f:
        for rel in f.read().split():
            with open(os.path.join(ROOT, rel), "rb") as g:
                h.update(g.read())
    return h.hexdigest()[:16]


STAMPED = (("liblvlip_csum.so", "BUILD_SOURCES"), ("liblvlip_testkit.so", "TESTKIT_SOURCES"),
           ("liblvlip_lab.so", "LAB_SOURCES"))


def _libraries_current() -> list:
    """The libraries whose stamp (the tree's source hash, read from the file so
    that nothing loads the HIP runtime here) is missing or differs."""
    stale = []
    for so, lst in STAMPED:
        path = os.path.join(PKG, so)
        if not os.path.exists(path):
            stale.append(so)
            continue
        with open(path, "rb") as f:
            if _source_build_id(lst).encode() not in f.read():
                stale.append(so)
    return stale


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # The libraries must be built from this tree's sources: rebuilt here when
    # that is allowed (_may_rebuild), else a stale one stops the run instead
    # of being tested.
    stale = _libraries_current()
    if stale:
        if not _may_rebuild():
            pytest.exit(f"{', '.join(stale)} not built from this tree's sources (build stamp differs): "
                        "run `make -C level-ip_amd` before testing (or set LVLIP_REBUILD=1)", returncode=3)
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
        stale = _libraries_current()
        if stale:
            pytest.exit(f"{', '.join(stale)} still differ from the tree after make", returncode=3)
    subprocess.run(["make", "-s", "-C", ORACLE, "oracle"], check=True)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def has_gpu():
    import lvlip
    return lvlip.device_count() > 0
