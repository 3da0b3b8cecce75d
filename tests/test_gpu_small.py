"""GPU: the persistent small-system step (kernels.hip k_pstep, GCS_OPT_SMALL_STEP: the default for <= 1,536
particles, i.e. the mitotic stages of C3 and the C1 chain): one cooperative launch per chunk of steps, every
workgroup holding the whole system in LDS, all pairs through a fp32 prefilter and the exact pair in R, a tagged
hand-off of the new positions per step, the tail computed by every workgroup.  Checked at both precisions against the fp64 oracle (the
precision's bound, tests/tolerances.py), against the list step (the same pair set, the sum in another order: within
the same bound), chunk-invariant bit for bit (also across the kernel's 2,048-step launches), and the C3 stage sizes.
The mitotic drivers' own parity tests (test_gpu_parity.py C3) run through this path too."""
import time

import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, mitotic
from gcs.config import InterphaseConfig
from gcs.engine import Engine
from tolerances import WALL_REL, X, precisions

import oracle

pytestmark = pytest.mark.gpu

LATE = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}


def _pair(design, cfg, prec, ctx=None, **opts):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg, precision=prec)
    for k, v in opts.items():
        e.set_option(getattr(A, "OPT_" + k.upper()), v)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        if ctx is None:
            s.apply_schedule(0)
        else:
            s.set_context(ctx)
    return e, o


@precisions
@pytest.mark.parametrize("ctx", [None, LATE], ids=["start", "late_wall"])
def test_small_step_c1_vs_oracle(c1_design, interphase_cfg, prec, ctx):
    """C1 (1,000 particles) from the schedule's start (cutoff growing) and in the late window with the wall in
    contact (reactions drive the wall ODE): positions, wall semiaxes and the step counter against the oracle"""
    cfg = interphase_cfg
    e, o = _pair(c1_design, cfg, prec, ctx)
    first = 0 if ctx is None else ctx["step"]
    for s in (e, o):
        s.run(60, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep, seed=31)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= X[prec]
    ce, co = e.get_context(), o.get_context()
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])
    assert ce["step"] == first + 60
    assert e.list_stats()["sync_stalls"] == 0  # no cell-scan look-back timeout (a hand-off stall fails the run)


@precisions
def test_small_step_injected_noise(c1_design, interphase_cfg, prec):
    """the reference-order normals (GCS_NOISE_INJECTED) through the small step's noise cursor"""
    cfg = interphase_cfg
    e, o = _pair(c1_design, cfg, prec)
    noise = np.random.default_rng(3).standard_normal((30, e.n, 3))
    for s in (e, o):
        s.set_noise(noise)
        s.run(30, temperature=cfg.temperature, timestep=cfg.timestep, noise=A.NOISE_INJECTED)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= X[prec]


@precisions
def test_small_step_chunks_bitwise(c1_design, interphase_cfg, prec):
    """2,100 steps in one call (two cooperative launches: 2,048 + 52) and in calls of 700 + 1,400 (launches of
    700, 1,400): the same bits and the same context -- nothing depends on how a run is split"""
    cfg = interphase_cfg
    runs = []
    for chunks in ((2100,), (700, 1400)):
        e, _ = interphase.build_interphase(Engine, c1_design, cfg, precision=prec)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.apply_schedule(0)
        st = 0
        for c in chunks:
            e.run(c, first_step=st, temperature=cfg.temperature, timestep=cfg.timestep, seed=77)
            st += c
        runs.append((e.get_positions(), e.get_context()))
    assert np.array_equal(runs[0][0], runs[1][0])
    assert runs[0][1] == runs[1][1]
    assert runs[0][1]["step"] == 2100


@precisions
def test_small_step_against_list_step(c1_design, interphase_cfg, prec):
    """the default (small) step and the list step (GCS_OPT_FUSED_STEP 3) and the small step switched off
    (GCS_OPT_SMALL_STEP 0: the list step again): the same pair set, so they agree within the precision's bound; the
    small step's sums run in another order, so not bit for bit"""
    cfg = interphase_cfg
    xs = []
    for opts in ({}, {"fused_step": 3}, {"small_step": 0}):
        e, _ = _pair(c1_design, cfg, prec, LATE, **opts)
        e.run(40, first_step=LATE["step"], temperature=cfg.temperature, timestep=cfg.timestep, seed=5)
        xs.append(e.get_positions())
    assert np.array_equal(xs[1], xs[2])
    assert np.abs(xs[0] - xs[1]).max() <= X[prec]


@precisions
def test_small_step_anatelophase_both_paths(prec):
    """C3's 586-bead anaphase + telophase through the driver (gcs.mitotic.AnatelophaseDriver: rods init, kinetochore
    fibers, the field swap): the default small step and the list step (GCS_OPT_SMALL_STEP 0) both within the
    precision's bound of the oracle"""
    from gcs.config import MitoticPhaseConfig
    from gcs import synthetic
    cfg = MitoticPhaseConfig()
    a = mitotic.anatelophase_design(synthetic.make_c2(), cfg)
    xs = []
    for cls, small in ((Engine, 1), (Engine, 0), (oracle.OracleSystem, None)):
        s, h = mitotic.build_anatelophase(cls, a, cfg, precision=prec)
        if small is not None:
            s.set_option(A.OPT_SMALL_STEP, small)
        mitotic.AnatelophaseDriver(s, h, a, cfg, log=None).run(anaphase_steps=40, telophase_steps=40)
        xs.append(s.get_positions())
    assert np.abs(xs[0] - xs[2]).max() <= X[prec]
    assert np.abs(xs[1] - xs[2]).max() <= X[prec]


@precisions
def test_small_step_droplet_many_targets(prec):
    """a droplet of 40 targets (> 16: k_pstep strides a particle's targets over its 4 lanes, whose loop
    trip counts then differ by lane) -- the small step within the precision's bound of the oracle and of the list
    step (GCS_OPT_SMALL_STEP 0), the droplet's attraction included (targets packed within its cutoff)"""
    n = 400
    rng = np.random.default_rng(12)
    x = rng.uniform(-0.45, 0.45, (n, 3))
    tg = np.arange(0, n, 10)
    x[tg] = rng.uniform(-0.15, 0.15, (tg.size, 3))
    xs = []
    for cls, small in ((Engine, 1), (Engine, 0), (oracle.OracleSystem, None)):
        s = cls(n, precision=prec)
        s.add_neighbor_softcore(2.5, 0.1, neighbor_distance=0.1, mix=False, scaled=False)
        s.add_neighbor_softwell(energy=3.0, decay_distance=0.2, cutoff=0.4, targets=tg)
        s.set_positions(x)
        if small is not None:
            s.set_option(A.OPT_SMALL_STEP, small)
        s.run(40, seed=4, timestep=1e-5, temperature=1.0)
        xs.append(s.get_positions())
        if small == 1:
            assert s.run_stats()["eager_steps"] >= 40  # (the small step: one cooperative launch, no graphs)
    assert np.abs(xs[0] - xs[2]).max() <= X[prec]
    assert np.abs(xs[1] - xs[2]).max() <= X[prec]
    # the droplet moved the targets more than the noise alone would at this timestep
    assert np.abs(xs[2][tg] - x[tg]).max() > 0


@precisions
def test_small_step_stall_fails_the_run(c1_design, interphase_cfg, prec, monkeypatch):
    """a workgroup that does not publish its hand-off (GCS_DEBUG_PSTEP_SKIP = workgroup 5, step
    3 of the run's first launch) stalls every workgroup; gcs_engine_run fails with GCS_ESTATE within a second, the
    positions and the context are those before the run, and the engine runs on afterwards"""
    cfg = interphase_cfg
    e, _ = _pair(c1_design, cfg, prec)
    x0, c0 = e.get_positions(), e.get_context()
    monkeypatch.setenv("GCS_DEBUG_PSTEP_SKIP", "5:3")
    t0 = time.perf_counter()
    with pytest.raises(A.GcsError) as err:
        e.run(500, temperature=cfg.temperature, timestep=cfg.timestep, seed=8)
    dt = time.perf_counter() - t0
    monkeypatch.delenv("GCS_DEBUG_PSTEP_SKIP")
    assert err.value.code == A.GCS_ESTATE and "stalled" in str(err.value), err.value
    assert dt < 1.0, dt
    assert np.array_equal(e.get_positions(), x0)
    c1 = e.get_context()
    for k in ("step", "time", "core_scale", "bond_scale", "wall_semiaxes", "inward_reaction", "outward_reaction"):
        assert c1[k] == c0[k], (k, c1[k], c0[k])  # (last_timestep: the run's dt, set before its first launch)
    e.run(20, temperature=cfg.temperature, timestep=cfg.timestep, seed=8)
    assert e.get_context()["step"] == c0["step"] + 20
    assert not np.array_equal(e.get_positions(), x0)
