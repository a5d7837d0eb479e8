import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libsv2n.so")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test but no ROCm GPU is visible")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _bound_checks(request):
    """With the diagnostic build (make CHECK=1, SV2N_LIB=...libsv2n_check.so)
    every GPU test also asserts that no instrumented kernel index left its
    allocation (sv2n_check_hits; SV2N_CHK in csrc/sv2n_common.h)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    if "check" not in os.path.basename(os.environ.get("SV2N_LIB", "")):
        return
    import ctypes
    from spotv2net_amd import _lib
    lib = _lib.load()
    fn = lib.sv2n_check_hits
    fn.restype = ctypes.c_uint
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    site = ctypes.c_uint(0)
    hits = fn(ctypes.byref(site))
    assert hits == 0, f"{hits} out-of-extent indices (first at site {site.value})"
