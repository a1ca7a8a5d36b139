"""MI355X-native Filter/Score evaluator for the kube-scheduler-simulator's
debuggable scheduler.

Layout:
  model.py        cluster object model (v1.Node / v1.Pod / NodeInfo subset)
  profile.py      scheduler profile: plugin order, weights, args
  encoder.py      snapshot encoder: objects -> SoA columns + pod programs
  native.py       ctypes binding of include/ksched.h (libksched.so, HIP)
  framework.py    debuggable-scheduler mirror: wrapped plugins + result store
  annotations.py  result store mirror and Go-compatible annotation JSON
  generator.py    seeded synthetic configs C1..C5
  replicas.py     what-if replica sweep across GPUs (torch.distributed)
  csrc/           HIP kernels + C ABI implementation
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
__version__ = "0.1.0"
