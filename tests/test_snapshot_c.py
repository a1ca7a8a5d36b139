"""The drop-in boundary from C only (tests/c/snapshot_c_test.c): clusters
built from strings through include/ksched_snapshot.h, encoded by
libksched.so, scheduled on the oracle (CPU) and on the MI355X (GPU, whole
queue and the Go shim's per-cycle path), compared with the oracle; and the
reference's export sample profile (per-point plugin sets, Store vs selection
weights) through the C ABI only: placements, status words and annotation
bytes against the oracle's."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c", "snapshot_c_test")
# the reference's export sample profile as a cgo caller passes it
# (tests/golden/make_export_profile.py)
EXPORT_PROFILE = os.path.join(HERE, "golden", "export_profile.txt")


def _run(flag, env=None):
    r = subprocess.run([BIN, flag, EXPORT_PROFILE], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


def test_c_boundary_cpu(built):
    _run("--cpu")


@pytest.mark.gpu
def test_c_boundary_gpu(built):
    _run("--gpu")


@pytest.mark.gpu
def test_c_boundary_gpu_cycle_server(built):
    """The same C-only cycles with the persistent per-cycle server."""
    _run("--gpu", {"KSG_CYCLE_SERVER": "1"})
