"""Host enqueue time vs wall time of bench.py's replica loop: is the 4-replica bench host-bound?
Wraps Engine.run (the graph launches) with a timer and runs the default bench (no CPU leg, no start window)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "3d-genome-cycle_amd")]
from gcs import engine as E  # noqa: E402

acc = {"run_s": 0.0, "calls": 0, "sync_s": 0.0}
_run, _sync = E.Engine.run, E.Engine.synchronize


def run(self, *a, **k):
    t = time.perf_counter()
    r = _run(self, *a, **k)
    acc["run_s"] += time.perf_counter() - t
    acc["calls"] += 1
    return r


def sync(self, *a, **k):
    t = time.perf_counter()
    r = _sync(self, *a, **k)
    acc["sync_s"] += time.perf_counter() - t
    return r


E.Engine.run, E.Engine.synchronize = run, sync
import bench  # noqa: E402

t0 = time.perf_counter()
bench.main(["--cpu-budget", "0", "--no-start-window"] + sys.argv[1:])
print(f"total {time.perf_counter() - t0:.2f} s, Engine.run {acc['run_s']:.2f} s over {acc['calls']} calls "
      f"({1e6 * acc['run_s'] / max(acc['calls'], 1):.0f} us each), synchronize {acc['sync_s']:.2f} s")
