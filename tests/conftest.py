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

BUILD_CONTAINER = os.path.isdir("/root/reference")  # the GPU box has no reference tree


def _source_build_id() -> str:
    """lvlip.source_build_id() without importing lvlip (which loads the library)."""
    import hashlib

    h = hashlib.sha256()
    with open(os.path.join(PKG, "BUILD_SOURCES")) as f:
        for rel in f.read().split():
            with open(os.path.join(ROOT, rel), "rb") as g:
                h.update(g.read())
    return h.hexdigest()[:16]


def _library_current() -> bool:
    """The product library carries the tree's source hash (lvlip_build_id(),
    read from the file so that nothing loads the HIP runtime here)."""
    so = os.path.join(PKG, "liblvlip_csum.so")
    if not os.path.exists(so) or not os.path.exists(os.path.join(PKG, "liblvlip_testkit.so")):
        return False
    with open(so, "rb") as f:
        return _source_build_id().encode() in f.read()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # The product library must be built from this tree's sources.  The build
    # container rebuilds it; anywhere else (the GPU box runs the prebuilt
    # snapshot) a stale library stops the run instead of being tested.
    if not _library_current():
        if not BUILD_CONTAINER:
            pytest.exit("liblvlip_csum.so was not built from this tree's sources (lvlip_build_id "
                        "differs): run `make -C level-ip_amd` before testing", returncode=3)
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
        if not _library_current():
            pytest.exit("liblvlip_csum.so still differs from the tree after make", returncode=3)
    subprocess.run(["make", "-s", "-C", ORACLE, "oracle"], check=True)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def has_gpu():
    import lvlip
    return lvlip.device_count() > 0
