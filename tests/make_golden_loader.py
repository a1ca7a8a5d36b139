"""Import shim for tests/golden/make_golden.py (the generator of the golden
vectors), so the tests rebuild inputs exactly as the fixtures were made."""
import importlib.util
import os

_p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_golden.py")
_spec = importlib.util.spec_from_file_location("make_golden", _p)
_m = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_m)

make = _m.make
input_digest = _m.input_digest
annotation_digest = _m.annotation_digest
