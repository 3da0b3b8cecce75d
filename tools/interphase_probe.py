"""Where the interphase stage's wall time goes (C2, 60,662 particles, through InterphaseDriver at the reference's
cadence: contact map every 20 steps, energy + sampled frame every 1,000, contact read every 10,000): host time in
each engine call the driver makes, the run statistics (graph replays / eager steps / captures), and the same stretch
without the contact map.  No store (the frames' HDF5 writes run on a background writer in the stage CLI anyway).

usage: python tools/interphase_probe.py [steps] [relaxation_steps]"""
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
relax = int(sys.argv[2]) if len(sys.argv) > 2 else 1000


def timed(eng, acc):
    """wrap the engine calls the driver makes: host seconds and calls per method"""
    for name in ("run", "contacts_update", "compute_energy", "get_context", "contacts_accumulate", "contacts_clear",
                 "sample_positions", "get_positions", "apply_schedule", "set_schedule", "set_option"):
        f = getattr(eng, name)

        def w(*a, _f=f, _n=name, **k):
            t0 = time.perf_counter()
            r = _f(*a, **k)
            acc[_n][0] += time.perf_counter() - t0
            acc[_n][1] += 1
            return r
        setattr(eng, name, w)


d = synthetic.make_c2(1)
for contacts in (True, False):
    cfg = InterphaseConfig()
    eng, _ = interphase.build_interphase(Engine, d, cfg)
    acc = defaultdict(lambda: [0.0, 0])
    timed(eng, acc)
    drv = interphase.InterphaseDriver(eng, d, cfg, store=None, log=None)
    t0 = time.perf_counter()
    drv.run_relaxation(relax)
    eng.synchronize()
    t1 = time.perf_counter()
    r0 = eng.run_stats()
    drv.run_simulation(steps, contacts=contacts)
    eng.synchronize()
    t2 = time.perf_counter()
    print(f"contacts={contacts}: relaxation {relax} steps {t1 - t0:.2f} s; simulation {steps} steps {t2 - t1:.2f} s "
          f"= {steps / (t2 - t1):.0f} steps/s ({d.n * steps / (t2 - t1):.3e} bead-updates/s)", flush=True)
    r1 = eng.run_stats()
    print("  run stats (simulation):", {k: r1[k] - r0.get(k, 0) for k in r1}, flush=True)
    print("  list:", eng.list_stats(), flush=True)
    for k, (s, n) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:22s} {n:7d} calls {s:8.3f} s  {1e3 * s / max(n, 1):8.3f} ms/call", flush=True)
    eng.close()
