"""The drop-in boundary from C only (tests/c/snapshot_c_test.c): clusters
built from strings through include/ksched_snapshot.h, encoded by
libksched.so, scheduled on the oracle (CPU) and on the MI355X (GPU, whole
queue and the Go shim's per-cycle path), compared with the oracle."""
import os
import subprocess

import pytest

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "snapshot_c_test")


def _run(flag):
    r = subprocess.run([BIN, flag], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


def test_c_boundary_cpu(built):
    _run("--cpu")


@pytest.mark.gpu
def test_c_boundary_gpu(built):
    _run("--gpu")
