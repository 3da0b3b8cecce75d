"""Resident step (GCS_OPT_RESIDENT) vs the list step at the small sizes: steps/s of one trajectory.
C1 (1,002 particles, late schedule), C3 anatelophase (586, telophase field) and prometaphase (1,172), both
precisions.  usage: python tools/resident_probe.py [steps]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi as A  # noqa: E402
from gcs import interphase, mitotic, synthetic  # noqa: E402
from gcs.config import InterphaseConfig, MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

LATE = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000


def systems(prec):
    cfg = InterphaseConfig()
    c1 = synthetic.make_c1()
    e, _ = interphase.build_interphase(Engine, c1, cfg, precision=prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.set_context(LATE)
    yield "c1", e, cfg.temperature, cfg.timestep, LATE["step"]
    mc = MitoticPhaseConfig()
    a = mitotic.anatelophase_design(synthetic.make_c2(), mc)
    s, h = mitotic.build_anatelophase(Engine, a, mc, precision=prec)
    drv = mitotic.AnatelophaseDriver(s, h, a, mc, log=None)
    drv.run(anaphase_steps=10, telophase_steps=10)
    yield "anatelophase", s, mc.temperature, mc.timestep, 20
    p = mitotic.prometaphase_design(a, mc, 1)
    s2, _ = mitotic.build_prometaphase(Engine, p, mc, precision=prec)
    rng = np.random.default_rng(3)
    s2.set_positions(rng.normal(scale=0.8, size=(p.n, 3)))
    yield "prometaphase", s2, mc.temperature, mc.timestep, 0


for prec in (64, 32):
    for name, e, T, dt, first in systems(prec):
        x0, c0 = e.get_positions(), e.get_context()
        out = {}
        for res in (0, 1, 2):  # the list step, the resident step, the resident step at the list step's skin
            e.set_positions(x0)
            e.set_context(c0)
            e.set_option(A.OPT_RESIDENT, min(res, 1))
            if res == 2:
                e.set_option(A.OPT_LIST_SKIN, 500)
            e.run(200, first_step=first, temperature=T, timestep=dt, seed=5)
            e.synchronize()
            t0 = time.perf_counter()
            e.run(steps, first_step=first + 200, temperature=T, timestep=dt, seed=5)
            e.synchronize()
            el = time.perf_counter() - t0
            st, rs = e.list_stats(), e.run_stats()
            out[res] = steps / el
            print(f"[{prec}] {name:13s} n={e.n:5d} {['list    ', 'resident', 'res/500 '][res]} {steps / el:10.0f} steps/s "
                  f"({1e6 * el / steps:6.2f} us/step) builds {st['builds']} every {st['rebuild_every']} skin "
                  f"{st['skin']:.4f} fallback {st['fallback_particle_steps']} resident_steps {rs['resident_steps']} "
                  f"finite {bool(np.isfinite(e.get_positions()).all())}", flush=True)
        print(f"[{prec}] {name}: resident / list = {out[1] / out[0]:.2f}, skin 500: {out[2] / out[0]:.2f}", flush=True)
        e.close()
