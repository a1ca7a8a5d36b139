"""Extract the two /v1/export response bodies (ResourcesForSnap documents)
from the reference's simulator/docs/api-samples/v1/export.md:32,63 into
tests/golden/export_md.json.  Run in the build container only (the reference
is not on the GPU box); the fixture is the data, unchanged."""
import json
import os

SRC = "/root/reference/simulator/docs/api-samples/v1/export.md"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "export_md.json")

if __name__ == "__main__":
    with open(SRC) as f:
        bodies = [json.loads(line) for line in f if line.startswith('{"pods"')]
    assert len(bodies) == 2, len(bodies)
    with open(OUT, "w") as f:
        json.dump({"source": "simulator/docs/api-samples/v1/export.md:32,63", "case1": bodies[0],
                   "case2": bodies[1]}, f, separators=(",", ":"))
        f.write("\n")
