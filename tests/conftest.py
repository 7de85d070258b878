import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    lib = os.path.join(ROOT, "another_raytracer_amd", "libart.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "another_raytracer_amd", "csrc"), "-j8"], check=True)
    so = os.path.join(ROOT, "oracle", "_ref", "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "restate"], check=True)


_ensure_built()


def has_gpu():
    try:
        import another_raytracer_amd as art
        return art.lib.rt_device_count() > 0
    except Exception:
        return False


@pytest.fixture
def options():
    """rt_option_set for one test: every library option is back at its default afterwards."""
    import another_raytracer_amd as art
    art.set_option(None, 0)
    yield art.set_option
    art.set_option(None, 0)


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.fail("no HIP device visible: -m gpu tests must run on an MI355X box")
    return 0
