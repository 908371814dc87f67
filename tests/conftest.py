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


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # the product library and the oracle must exist before any test imports them
    if not os.path.exists(os.path.join(PKG, "liblvlip_csum.so")) or not os.path.exists(
            os.path.join(PKG, "liblvlip_testkit.so")):
        subprocess.run(["make", "-s", "-C", PKG, "-j4"], check=True)
    subprocess.run(["make", "-s", "-C", ORACLE, "oracle"], check=True)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def has_gpu():
    import lvlip
    return lvlip.device_count() > 0
