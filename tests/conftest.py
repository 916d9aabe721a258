import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhq on the GPU)")


def _gpu_available() -> bool:
    try:
        import hybridquantization_amd as hq

        import ctypes

        n = ctypes.c_int(0)
        hq.load().hq_device_count(ctypes.byref(n))
        return n.value > 0
    except OSError:
        return False


def pytest_terminal_summary(terminalreporter):
    """Evidence of the native path: the libhq shared objects this process mapped."""
    try:
        with open("/proc/self/maps") as f:
            libs = sorted({ln.split()[-1] for ln in f if "libhq" in ln and ln.rstrip().endswith(".so")})
    except OSError:
        libs = []
    terminalreporter.write_line("mapped libhq: " + (", ".join(libs) if libs else "none"))


@pytest.fixture(scope="session")
def gpu():
    """Skip-free guard: a gpu-marked test run without a device is an error."""
    if not _gpu_available():
        pytest.fail("gpu test requested but no HIP device / libhq.so")
    # the oracles' argmin distance takes the device's v_sqrt_f32, as the
    # reference's distance() does on this GPU (oracle/hw_sqrt.py; built by
    # build() with the oracle).  Without the helper the oracles keep the
    # correctly rounded root, and the tests that need the device's fail.
    import warnings

    import hw_sqrt

    try:
        hw_sqrt.install()
    except OSError as e:
        warnings.warn(f"oracle/libhq_hwsqrt.so not loadable ({e}): the oracles' argmin uses sqrtf")
    return 0
