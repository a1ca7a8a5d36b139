"""Run bench.py's per-cycle sidecar alone (C driver): python scripts/percycle.py [nodes] [warm] [pods]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PKG = "kube-scheduler-simulator_amd"
native = importlib.import_module(PKG + ".native")
G = importlib.import_module(PKG + ".generator")
S = importlib.import_module(PKG + ".snapshot")
a = [int(x) for x in sys.argv[1:]] + [5000, 500, 2000][len(sys.argv) - 1:]
print(json.dumps(bench.per_cycle_sidecar(native, G, S, a[0], a[1], a[2])), flush=True)
