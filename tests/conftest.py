import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PKG = "kube-scheduler-simulator_amd"


def pkg(mod: str = ""):
    return importlib.import_module(PKG + ("." + mod if mod else ""))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libksched.so)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def built():
    ge = importlib.import_module("__graft_entry__")
    ge.build()
    return True


@pytest.fixture(autouse=True)
def _device_sync_after_test(request):
    """KSG_TEST_DEVICE_SYNC=1 (diagnosis only): after every GPU test, let the
    persistent servers idle out and synchronise the device, so an
    asynchronous fault is reported by the test whose kernels raised it."""
    yield
    if not os.environ.get("KSG_TEST_DEVICE_SYNC") or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    import gc
    import time
    gc.collect()
    time.sleep(0.15)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGetErrorString.restype = ctypes.c_char_p
    rc = hip.hipDeviceSynchronize()
    if rc != 0:
        pytest.fail(f"device fault after {request.node.nodeid}: {hip.hipGetErrorString(rc).decode()}")
