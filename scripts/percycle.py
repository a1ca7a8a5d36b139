"""Run bench.py's per-cycle sidecar alone (C driver):
python scripts/percycle.py [nodes] [warm] [pods] [c2|c3] [server (default)|launch] [hint_ahead]"""
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
a = [int(x) for x in sys.argv[1:4]] + [5000, 500, 2000][len(sys.argv[1:4]):]
kind = sys.argv[4] if len(sys.argv) > 4 else "c2"
make, label = (G.config3, "configs[2]") if kind == "c3" else (G.config2, "configs[1]")
srv = not (len(sys.argv) > 5 and sys.argv[5] == "launch")
ahead = int(sys.argv[6]) if len(sys.argv) > 6 else 0
print(json.dumps(bench.per_cycle_sidecar(native, G, S, a[0], a[1], a[2], make=make, label=label, server=srv,
                                         hint_ahead=ahead)), flush=True)
