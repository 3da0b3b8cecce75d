"""The long-horizon C2 ensemble protocol shared by the oracle fixture (tests/golden/gen_c2_ensemble.py) and the GPU
test (tests/test_gpu_ensemble.py): the production regime of simulation_driver_interphase.cpp:57-63 (dt 1e-5, the
device schedule of :67-90), from the committed step-300,000 bench state."""
from __future__ import annotations

from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
STATE = ROOT / "benchdata" / "c2_interphase_step300000.npz"

NSEED = 8
STEPS = 16000
EVERY = 2000
SKIP = 4000
ORACLE_SEED0 = 71000
ENGINE_SEED0 = 72000
NAMES = ["bond", "rg", "energy_per_particle", "wall_x", "wall_y", "wall_z"]


def state():
    z = np.load(STATE, allow_pickle=False)
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    return np.asarray(z["positions"], dtype=np.float64), ctx


def build(cls, **kw):
    from gcs import interphase, synthetic
    from gcs.config import InterphaseConfig
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    s, _ = interphase.build_interphase(cls, design, cfg, **kw)
    s.set_schedule(**interphase.interphase_schedule(cfg))
    x, ctx = state()
    s.set_positions(x)
    s.set_context(ctx)
    s._design, s._cfg, s._first = design, cfg, ctx["step"]
    return s


def observables(s):
    design = s._design
    x = s.get_positions()
    b = np.concatenate([np.linalg.norm(x[a + 1:t] - x[a:t - 1], axis=1) for _, a, t in design.chains])
    rg = float(np.sqrt(((x - x.mean(axis=0)) ** 2).sum(axis=1).mean()))
    en, _ = s.compute_energy()
    return [float(b.mean()), rg, en / design.n] + [float(v) for v in s.get_context()["wall_semiaxes"]]


def trajectory(s, seed):
    """STEPS steps in EVERY-step runs; the observables after every run past SKIP"""
    cfg, done, out = s._cfg, 0, []
    while done < STEPS:
        s.run(EVERY, first_step=s._first + done, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
        done += EVERY
        if done > SKIP:
            out.append(observables(s))
    return out
