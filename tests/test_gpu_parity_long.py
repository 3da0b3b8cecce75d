"""GPU parity beyond the first steps, on every BASELINE interphase size, against the fp64 oracle (through the C ABI).

Stated bounds (fp64 engine, the default / fp32 engine, tests/tolerances.py):
  forces                |dF| <= 1e-10 / 1e-4 max|F| + 1e-10 / 1e-3 per component
  C5 trajectory         |dx| <= 1e-9 / 2e-5 after 1, 2, 5 and 10 steps from the dense synthetic start
  C2 trajectory         |dx| <= 1e-9 / 2e-5 after 50 steps from the bench state (step 300,000)
  statistics            ensemble means of <|r_i,i+1|>, Rg, E/N and the wall semiaxes within 3 standard errors
                        (engine Philox vs oracle Philox fp64, independent seeds)

The fp64 engine differs from the oracle only in the summation order of pair forces, contractions and last-ulp libm
results (~1e-15 per step), so 1e-9 leaves six orders of magnitude for their growth.  For the fp32 engine, why 2e-5
is an absolute bound and not a ratio: one step moves a particle by mu dt F + noise.  An fp32 force error
|dF| <= 1e-4 max|F| + 1e-3 moves it by at most mu dt |dF| (C5: 2.2e-6 x 0.72 = 1.5e-6; C2 at step 300k:
1e-5 x 0.03 = 3e-7) plus the rounding of the position itself (1 ulp of |x| <= 2: 2.4e-7).  Those per-step errors
are then carried by the dynamics: the oracle alone, started from positions perturbed by 1 ulp, diverges by
3.2e-6 after 10 C5 steps and 1.8e-6 after 100 C2 steps (test_perturbation_growth below measures it in the same
run), so a sum of ten such per-step errors stays below 2e-5.  At the 100 kb timestep a 10 kb soft core is
unstable (k mu dt ~ 1.6): the oracle then amplifies a 1-ulp perturbation to 1.4e-4 in 5 steps and 3e-2 in 10 --
the 1.8e-4 of round 1 -- which is why the C5 configuration scales the timestep with the bead size
(gcs.config.resolution_scaled).
"""
import dataclasses
import json
import os

import numpy as np
import pytest

from gcs import interphase, synthetic
from gcs.config import InterphaseConfig, resolution_scaled
from gcs.engine import Engine
from tolerances import E_REL, F_ABS, F_REL, WALL_REL, X, precisions

import oracle

pytestmark = pytest.mark.gpu

TOL_X = X[32]  # the fp32 engine's bound (the perturbation-growth envelope below is about it)
SEED = 99
OUT = os.environ.get("GCS_PARITY_LOG")  # optional: record the measured errors as JSON lines


def _log(**kw):
    if OUT:
        with open(OUT, "a") as f:
            f.write(json.dumps(kw) + "\n")
    print(kw)


def _pair(design, cfg, x=None, ctx=None, prec=64):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg, precision=prec)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        if x is not None:
            s.set_positions(x)
        if ctx is not None:
            s.set_context(ctx)
    return e, o


def _f32(x):
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def assert_forces_close(fe, fo, prec):
    scale = np.abs(fo).max()
    err = np.abs(fe - fo).max()
    assert err <= F_REL[prec] * scale + F_ABS[prec], (err, scale)
    return err, scale


@pytest.fixture(scope="module")
def c5():
    return synthetic.make_c5(), resolution_scaled(InterphaseConfig(), 10.0)


@precisions
def test_c5_forces_step0(c5, prec):
    design, cfg = c5
    e, o = _pair(design, cfg, x=_f32(design.positions), prec=prec)
    err, scale = assert_forces_close(e.compute_forces(), o.compute_forces(), prec)
    _log(test="c5_forces_step0", prec=prec, err=float(err), max_force=float(scale))


@precisions
def test_c5_trajectory_absolute_bound(c5, prec):
    """engine vs oracle after 1, 2, 5, 10 steps (same fp32-representable start, same Philox stream)"""
    design, cfg = c5
    e, o = _pair(design, cfg, x=_f32(design.positions), prec=prec)
    done, errs = 0, {}
    for k in (1, 2, 5, 10):
        for s in (e, o):
            s.run(k - done, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
        done = k
        errs[k] = float(np.abs(e.get_positions() - o.get_positions()).max())
    _log(test="c5_trajectory", prec=prec, errors=errs, timestep=cfg.timestep)
    assert all(v <= X[prec] for v in errs.values()), errs
    ce, co = e.get_context(), o.get_context()
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])


def test_perturbation_growth(c5):
    """The oracle's own sensitivity: two fp64 runs whose starts differ by 1 ulp (fp32) per coordinate.  The engine's
    per-step fp32 errors are of that size, so this envelope is what the absolute bound has to cover."""
    design, cfg = c5
    x = _f32(design.positions)
    rng = np.random.default_rng(0)
    x32 = x.astype(np.float32)
    xp = (x32 + np.spacing(x32) * rng.choice([-1, 1], size=x.shape)).astype(np.float64)
    runs = []
    for start in (x, xp):
        o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
        o.set_schedule(**interphase.interphase_schedule(cfg))
        o.set_positions(start)
        o.run(10, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
        runs.append(o.get_positions())
    d = float(np.abs(runs[0] - runs[1]).max())
    _log(test="c5_perturbation_growth_10", divergence=d)
    assert d <= TOL_X / 2  # a stable integration: ten such per-step errors fit the stated bound


@precisions
def test_c2_trajectory_from_bench_state(prec):
    """C2 (60,662 beads) k-step trajectory parity from benchdata/c2_interphase_step300000.npz, Philox noise"""
    from pathlib import Path
    z = np.load(Path(__file__).resolve().parents[1] / "benchdata" / "c2_interphase_step300000.npz")
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    e, o = _pair(design, cfg, x=_f32(z["positions"]), ctx=ctx, prec=prec)
    first = ctx["step"]
    done, errs = 0, {}
    for k in (1, 10, 50):
        for s in (e, o):
            s.run(k - done, first_step=first + done, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
        done = k
        errs[k] = float(np.abs(e.get_positions() - o.get_positions()).max())
    _log(test="c2_trajectory_step300k", prec=prec, errors=errs)
    assert all(v <= X[prec] for v in errs.values()), errs
    ce, co = e.get_context(), o.get_context()
    assert ce["step"] == co["step"] == first + 50
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])
    assert e.compute_energy()[0] == pytest.approx(o.compute_energy()[0], rel=E_REL[prec])


def _observables(sys_, design):
    x = sys_.get_positions()
    bonds = []
    for _, s, t in design.chains:
        bonds.append(np.linalg.norm(x[s + 1:t] - x[s:t - 1], axis=1))
    b = np.concatenate(bonds)
    rg = float(np.sqrt(((x - x.mean(axis=0)) ** 2).sum(axis=1).mean()))
    en, _ = sys_.compute_energy()
    return np.array([b.mean(), rg, en / design.n] + list(sys_.get_context()["wall_semiaxes"]))


def test_statistics_engine_vs_oracle(c1_design):
    """Philox fp32 engine trajectories and fp64 oracle trajectories (independent seeds) sample the
    same ensemble: <|r_i,i+1|>, Rg, E/N and the wall semiaxes (late schedule, wall in contact), time-averaged over
    samples every 500 steps of an 8,000-step window, agree within 3 standard errors of the difference of the
    seed means."""
    cfg = InterphaseConfig()
    design = c1_design
    ctx = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}
    nseed, steps, every = 6, 8000, 500
    res = {"engine": [], "oracle": []}
    for kind in res:
        for k in range(nseed):
            if kind == "engine":
                s, _ = interphase.build_interphase(Engine, design, cfg)
            else:
                s, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
            s.set_schedule(**interphase.interphase_schedule(cfg))
            s.set_context(ctx)
            seed = (1000 + k) if kind == "engine" else (5000 + k)
            samples, done = [], 0
            while done < steps:
                s.run(every, first_step=200000 + done, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
                done += every
                if done >= 1000:
                    samples.append(_observables(s, design))
            res[kind].append(np.mean(samples, axis=0))
            if kind == "engine":
                s.close()
    me, mo = np.mean(res["engine"], axis=0), np.mean(res["oracle"], axis=0)
    se = np.std(res["engine"], axis=0, ddof=1) / np.sqrt(nseed)
    so = np.std(res["oracle"], axis=0, ddof=1) / np.sqrt(nseed)
    z = np.abs(me - mo) / np.sqrt(se ** 2 + so ** 2 + 1e-30)
    names = ["bond", "rg", "energy_per_bead", "wall_x", "wall_y", "wall_z"]
    _log(test="statistics_c1", engine=dict(zip(names, me.tolist())), oracle=dict(zip(names, mo.tolist())),
         z=dict(zip(names, z.tolist())))
    assert (z <= 3.0).all(), dict(zip(names, z.tolist()))
    # and the runs did move: the seed spread is not zero
    assert (se[:3] > 0).all() and (so[:3] > 0).all()


@precisions
def test_c2_relaxation_spacestep(prec):
    """The relaxation stage's adaptive step (simulation_driver_relaxation.cpp:48-55: spacestep 1e-3) at C2 size from
    the synthetic start, injected reference noise, 5 steps: positions within the bound, the adapted timestep equal"""
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    steps = 5
    xi = oracle.reference_normals(design.seed, steps * design.n * 3).reshape(steps, design.n, 3)
    e, o = _pair(design, cfg, x=_f32(design.positions), prec=prec)
    for s in (e, o):
        s.apply_schedule(0)
        s.set_noise(xi)
        s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, spacestep=cfg.relaxation_spacestep,
              noise=1)
    err = float(np.abs(e.get_positions() - o.get_positions()).max())
    _log(test="c2_relaxation", prec=prec, error=err)
    assert err <= X[prec]
    assert e.get_context()["last_timestep"] == pytest.approx(o.get_context()["last_timestep"],
                                                             rel={64: 1e-10, 32: 1e-4}[prec])
