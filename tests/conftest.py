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
