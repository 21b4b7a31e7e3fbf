import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gpu-ray-tracing_amd")
for p in (PKG, os.path.dirname(os.path.abspath(__file__)), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _built():
    libs = [os.path.join(PKG, "lib", "libmrt.so"), os.path.join(PKG, "lib", "libmrt_host.so")]
    return all(os.path.exists(p) for p in libs)


@pytest.fixture(scope="session", autouse=True)
def native_libs():
    """Build the in-tree libraries once if they are missing (CPU-side build)."""
    if not _built():
        import subprocess
        subprocess.run(["make", "-C", PKG, f"-j{min(16, os.cpu_count() or 1)}"], check=True)
    yield
