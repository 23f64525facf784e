import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every GPU build of the suite also checks its whole table's contiguity on the device
# (k_verify_rows; a violation is SHOCKIDX_EINTERNAL): record.go:51-83 writes contiguous rows
os.environ.setdefault("SHOCKIDX_VERIFY", "1")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    import oracle
    return oracle


@pytest.fixture(scope="session")
def shockidx_so():
    so = os.path.join(ROOT, "shock_amd", "libshockidx.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "shock_amd", "csrc")], check=True)
    return so


@pytest.fixture(scope="session")
def gpu_ctx(shockidx_so):
    from shock_amd import Context
    ctx = Context(0)
    yield ctx
    ctx.close()
