import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP device); run with -m gpu")


def _ensure_built():
    lib = os.path.join(ROOT, "multiagent_orb_slam2_amd", "liborbx.so")
    orc = os.path.join(ROOT, "oracle", "liborb_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        import subprocess
        subprocess.run(["make", "-C", ROOT], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu():
    import multiagent_orb_slam2_amd as pkg
    if pkg.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0
