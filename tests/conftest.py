import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "cuda-bezier-triangle-raytracer_amd"
for p in (str(PKG), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbzr's HIP kernels)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds on CPU")


@pytest.fixture(scope="session")
def built():
    """Make sure libbzr.so and liboracle.so exist (build() does the same)."""
    jobs = str(min(16, os.cpu_count() or 4))
    if not (PKG / "lib" / "libbzr.so").exists():
        subprocess.run(["make", "-C", str(PKG), "-j", jobs], check=True, capture_output=True)
    subprocess.run(["make", "-C", str(REPO / "oracle")], check=True, capture_output=True)
    return True


@pytest.fixture(scope="session")
def bzr(built):
    import bzr_amd

    bzr_amd.lib()
    return bzr_amd


@pytest.fixture(scope="session")
def orc(built):
    from oracle import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def ctx(bzr):
    n = bzr.device_count()
    if n == 0:
        pytest.fail("GPU test on a machine without a HIP device (libbzr has no CPU path)")
    return bzr.Context(0)


@pytest.fixture(params=["fused", "staged"])
def pipe(request, bzr):
    """The culled path's two pipelines (include/bzr.h BZR_PIPELINE_*): parity tests run both."""
    return bzr.PIPELINE_FUSED if request.param == "fused" else bzr.PIPELINE_STAGED
