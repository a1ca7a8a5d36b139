"""Host logic of bulk.annotate_queue_device (no GPU): the launch / wait
order the library's three rotating pinned buffers require (chunk j + 2 is
launched only after chunk j's values were handed out), every pod's three
values reaching the sink from the right offsets, and placements in queue
order.  The engine is a stand-in that records the calls."""
import threading

import numpy as np

from conftest import pkg

B = pkg("bulk")


class FakeEngine:
    """run_queue_json_async / json_wait with the library's contract: a ticket
    per chunk, values back to back with offsets [3k .. 3k + 3] per pod."""

    def __init__(self):
        self.calls = []
        self.lock = threading.Lock()
        self.live = 0
        self.max_live = 0

    def attach_annotator(self, ann, weights, mask):
        self.calls.append(("attach",))

    def run_queue_json_async(self, first, count):
        with self.lock:
            self.calls.append(("launch", first, count))
            self.live += 1
            self.max_live = max(self.max_live, self.live)
        return np.arange(first, first + count, dtype=np.int32), None, (first, count)

    def json_wait(self, ticket, count):
        first, k = ticket
        assert k == count
        vals, offs = [], [0]
        for i in range(first, first + count):
            for part in ("f", "s", "t"):
                b = f"{part}{i}".encode()
                vals.append(b)
                offs.append(offs[-1] + len(b))
        with self.lock:
            self.calls.append(("wait", first))
        return memoryview(b"".join(vals)), offs

    def done(self, first):
        with self.lock:
            self.live -= 1


class FakeBulk:
    pool = None
    annotators = [None]
    weights = np.zeros(1, np.int64)
    norm_mask = 0


def test_device_loop_order_and_values():
    eng = FakeEngine()
    got = {}

    def sink(i, vals):
        got[i] = tuple(bytes(v) for v in vals)

    orig_wait = eng.json_wait

    def wait(ticket, count):
        out = orig_wait(ticket, count)
        eng.done(ticket[0])
        return out

    eng.json_wait = wait
    pl = B.annotate_queue_device(eng, FakeBulk(), 10, 1000, sink, chunk=96)
    np.testing.assert_array_equal(pl, np.arange(10, 1010, dtype=np.int32))
    assert sorted(got) == list(range(10, 1010))
    for i in range(10, 1010):
        assert got[i] == (f"f{i}".encode(), f"s{i}".encode(), f"t{i}".encode())
    # chunk j + 2 is launched only after chunk j was waited for: at most three
    # chunks hold a buffer (two launched ahead, one being read)
    order = [c for c in eng.calls if c[0] in ("launch", "wait")]
    launched, waited = [], set()
    for c in order:
        if c[0] == "launch":
            j = (c[1] - 10) // 96
            assert j < 2 or (j - 2) in waited, order[:20]
            launched.append(j)
        else:
            waited.add((c[1] - 10) // 96)
    assert launched == list(range(len(launched))) and len(launched) == (1000 + 95) // 96
    assert eng.max_live <= 3
