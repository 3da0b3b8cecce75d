"""Where the interphase stage's wall time goes (C2, 60,662 particles, through InterphaseDriver at the reference's
cadence: contact map every 20 steps, energy + sampled frame every 1,000, contact read every 10,000): host time in
each engine call the driver makes, the run statistics (graph replays / eager steps / captures), and the same stretch
without the contact map.  No store (the frames' HDF5 writes run on a background writer in the stage CLI anyway).

usage: python tools/interphase_probe.py [steps] [relaxation_steps] [contact bits,...] [list skin bases,...]"""
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi, interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
relax = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
cbits = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]  # GCS_OPT_CONTACT_BITS (0: default)
bases = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]  # GCS_OPT_LIST_SKIN_BASE (0: the driver's)


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
for contacts, bits, base in [(True, b, bases[0]) for b in cbits] + [(True, cbits[0], b) for b in bases[1:]] + \
        [(False, 0, bases[0])]:
    cfg = InterphaseConfig()
    eng, _ = interphase.build_interphase(Engine, d, cfg)
    eng.set_option(_abi.OPT_CONTACT_BITS, bits)

    eng.set_option(_abi.OPT_DENSE_NEIGHBORS, 0)  # C2 is list-step territory; the probe upsets rocprofv3 (engine.hip)
    acc = defaultdict(lambda: [0.0, 0])
    timed(eng, acc)
    drv = interphase.InterphaseDriver(eng, d, cfg, store=None, log=None)
    if base:  # (after the driver, which sets its own: gcs/interphase.py SINGLE_SKIN_BASE_F64)
        eng.set_option(_abi.OPT_LIST_SKIN_BASE, base)
        print(f"  list skin base {base}", flush=True)
    t0 = time.perf_counter()
    drv.run_relaxation(relax)
    eng.synchronize()
    t1 = time.perf_counter()
    r0 = eng.run_stats()
    drv.run_simulation(steps, contacts=contacts)
    eng.synchronize()
    t2 = time.perf_counter()
    if contacts:
        import hashlib
        import numpy as np
        digest = hashlib.sha1(np.ascontiguousarray(drv.last_contacts).tobytes()).hexdigest()[:16]
        print(f"  contact bits {bits or 'default'}: last window's table {len(drv.last_contacts)} distinct pairs "
              f"(sha1 {digest})", flush=True)
    print(f"contacts={contacts}: relaxation {relax} steps {t1 - t0:.2f} s; simulation {steps} steps {t2 - t1:.2f} s "
          f"= {steps / (t2 - t1):.0f} steps/s ({d.n * steps / (t2 - t1):.3e} bead-updates/s)", flush=True)
    r1 = eng.run_stats()
    print("  run stats (simulation):", {k: r1[k] - r0.get(k, 0) for k in r1}, flush=True)
    print("  list:", eng.list_stats(), flush=True)
    for k, (s, n) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:22s} {n:7d} calls {s:8.3f} s  {1e3 * s / max(n, 1):8.3f} ms/call", flush=True)
    eng.close()

# the step loop alone, from the same start (after a short run): graph stretches of 20 vs 1,000 steps, with and
# without a contact update per 20 steps
cfg = InterphaseConfig()
for chunk, contacts in ((1000, False), (20, False)):
    eng, _ = interphase.build_interphase(Engine, d, cfg)
    eng.set_schedule(**interphase.interphase_schedule(cfg))
    eng.apply_schedule(0)
    eng.set_option(_abi.OPT_GRAPH_STEPS, chunk)
    eng.set_option(_abi.OPT_DENSE_NEIGHBORS, 0)
    bd = dict(temperature=cfg.temperature, timestep=cfg.timestep, seed=5)
    eng.run(2000, first_step=0, **bd)
    eng.synchronize()
    t0, done = time.perf_counter(), 2000
    while done < 22000:
        if contacts:
            eng.contacts_update(0.2)
        eng.run(chunk, first_step=done, **bd)
        done += chunk
    eng.synchronize()
    el = time.perf_counter() - t0
    print(f"loop: run({chunk}) x {20000 // chunk}, contacts={contacts}: {20000 / el:.0f} steps/s "
          f"({el / (20000 // chunk) * 1e6:.0f} us per run call)", flush=True)
    eng.close()
