"""GPU parity of the list step (GCS_OPT_FUSED_STEP 3: neighbour lists with a skin, one launch per step, exact
cell search for any particle the skin no longer covers) against the fp64 oracle, through the C ABI.

Bounds are the ones DESIGN.md §6 states for every step shape, per engine precision (tests/tolerances.py): positions
within 1e-9 (fp64 engine) / 2e-5 (fp32 engine) absolute after k steps, forces/energies through the same engine calls.  The list step changes only the order in which a particle's pair
forces are summed, never the pair set (k_lstep: a particle whose list may be incomplete is searched exactly), so
the same bounds hold with the rebuild period forced far beyond what the skin covers, and with lists that overflow.
"""
import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, synthetic
from gcs.config import InterphaseConfig, resolution_scaled
from gcs.engine import Engine
from tolerances import REACT, WALL_REL, X as TOL_X, precisions

import oracle

pytestmark = pytest.mark.gpu

LATE = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}


def _f32(x):
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def _list_engine(design, cfg, prec=64, **opts):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    e.set_option(A.OPT_FUSED_STEP, 3)
    e.set_option(A.OPT_DENSE_NEIGHBORS, 0)  # the list step at any density (test_dense_start_takes_tile_step: the switch)
    for k, v in opts.items():
        e.set_option(getattr(A, "OPT_" + k.upper()), v)
    return e


def _pair(design, cfg, x=None, ctx=None, prec=64, **opts):
    e = _list_engine(design, cfg, prec, **opts)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg, precision=prec)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        if x is not None:
            s.set_positions(x)
        if ctx is not None:
            s.set_context(ctx)
        else:
            s.apply_schedule(0)
    return e, o


def _run_both(e, o, steps, first, cfg, seed, **kw):
    for s in (e, o):
        s.run(steps, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed, **kw)


@precisions
def test_list_trajectory_c1_from_step0(c1_design, prec):
    """production start (core scale 0.5, growing cutoff), 60 steps, Philox noise"""
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, prec=prec)
    _run_both(e, o, 60, 0, cfg, 987654321)
    err = np.abs(e.get_positions() - o.get_positions()).max()
    st = e.list_stats()
    assert st["active"] == 1 and st["builds"] >= 60 // st["rebuild_every"], st
    assert err <= TOL_X[prec], (err, st)


@precisions
def test_list_trajectory_c1_wall_contact(c1_design, prec):
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE, prec=prec)
    _run_both(e, o, 40, LATE["step"], cfg, 5)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]
    ce, co = e.get_context(), o.get_context()
    assert ce["step"] == co["step"] == LATE["step"] + 40
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])
    rt, at = REACT[prec]
    assert np.allclose(ce["inward_reaction"], co["inward_reaction"], rtol=rt, atol=at)


@precisions
def test_list_injected_reference_noise(c1_design, prec):
    cfg = InterphaseConfig()
    steps = 12
    xi = oracle.reference_normals(c1_design.seed, steps * c1_design.n * 3).reshape(steps, c1_design.n, 3)
    e, o = _pair(c1_design, cfg, prec=prec)
    for s in (e, o):
        s.set_noise(xi)
    _run_both(e, o, steps, 0, cfg, 0, noise=A.NOISE_INJECTED)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]


@precisions
@pytest.mark.parametrize("skin,every", [(30, 200), (400, 64)])
def test_list_exact_when_the_skin_is_outrun(c1_design, skin, every, prec):
    """rebuild period far beyond the skin: particles outrun it and take the exact cell search; same bound"""
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE, prec=prec, list_skin=skin, list_every=every)
    _run_both(e, o, 60, LATE["step"], cfg, 17)
    st = e.list_stats()
    assert st["fallback_particle_steps"] > 0, st
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]


@precisions
def test_list_exact_when_lists_overflow(c1_design, prec):
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE, prec=prec, list_cap=32)
    _run_both(e, o, 30, LATE["step"], cfg, 23)
    st = e.list_stats()
    assert st["fallback_particle_steps"] > 0, st
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]


@precisions
@pytest.mark.parametrize("every", [0, 1, 5])
def test_list_graph_eager_and_chunks_bitwise_identical(c1_design, every, prec):
    """graph vs eager launches and one run vs chunks rebuild at the same steps: identical bits"""
    cfg = InterphaseConfig()
    runs = []
    for g, chunks in ((0, [70]), (8, [70]), (32, [70]), (32, [13, 40, 17]), (32, [1, 1, 3, 65])):
        e = _list_engine(c1_design, cfg, prec, list_every=every, graph_steps=g)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_context(LATE)
        first = LATE["step"]
        for c in chunks:
            e.run(c, first_step=first, seed=11)
            first += c
        runs.append((e.get_positions(), e.get_context()))
        e.close()
    for x, c in runs[1:]:
        assert np.array_equal(x, runs[0][0])
        assert c == runs[0][1]


@precisions
@pytest.mark.parametrize("n", [1, 2, 63, 65, 200, 1025, 1500])
def test_list_small_and_ragged_sizes(n, prec):
    """random ab factors and mobilities (several pair classes, mixed), 20 steps at dt 1e-4"""
    rng = np.random.default_rng(n)
    x = rng.uniform(-0.5, 0.5, size=(n, 3))
    ab = rng.choice([0.0, 0.5, 1.0], size=(n, 2))
    mu = rng.uniform(0.5, 1.5, size=n)
    sysd = {}
    for name, cls in (("e", Engine), ("o", oracle.OracleSystem)):
        s = cls(n, mobilities=mu, ab_factors=ab, precision=prec)
        s.add_neighbor_softcore(2.5, 0.3, 2.5, 0.24, 0.3, mix=True, scaled=True)
        if n > 1:
            s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=100.0, b_spring=50.0, mix=True, scaled=True,
                                  ranges=[(0, n)])
        s.set_context({"core_scale": 0.8, "bond_scale": 0.7, "wall_semiaxes": [1, 1, 1]})
        s.set_positions(x)
        if name == "e":
            s.set_option(A.OPT_FUSED_STEP, 3)
            s.set_option(A.OPT_DENSE_NEIGHBORS, 0)
        sysd[name] = s
    for s in sysd.values():
        s.run(20, seed=1, timestep=1e-4)
    assert sysd["e"].list_stats()["active"] == 1
    assert np.abs(sysd["e"].get_positions() - sysd["o"].get_positions()).max() <= TOL_X[prec]


@precisions
def test_list_c2_trajectory_from_bench_state(prec):
    """C2 (60,662 beads) from benchdata (step 300,000): 1, 10, 50 steps vs the oracle"""
    from pathlib import Path
    z = np.load(Path(__file__).resolve().parents[1] / "benchdata" / "c2_interphase_step300000.npz")
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    e, o = _pair(design, cfg, x=_f32(z["positions"]), ctx=ctx, prec=prec)
    first, done, errs = ctx["step"], 0, {}
    for k in (1, 10, 50):
        _run_both(e, o, k - done, first + done, cfg, 99)
        done = k
        errs[k] = float(np.abs(e.get_positions() - o.get_positions()).max())
    print({"list_c2_errors": errs, "stats": e.list_stats()})
    assert all(v <= TOL_X[prec] for v in errs.values()), errs
    ce, co = e.get_context(), o.get_context()
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])


@precisions
def test_list_c5_trajectory(prec):
    """C5 (606,248 beads, 10 kb, resolution-scaled timestep): 10 steps from the dense synthetic start"""
    design, cfg = synthetic.make_c5(), resolution_scaled(InterphaseConfig(), 10.0)
    e, o = _pair(design, cfg, x=_f32(design.positions), prec=prec)
    _run_both(e, o, 10, 0, cfg, 99)
    err = float(np.abs(e.get_positions() - o.get_positions()).max())
    print({"list_c5_err": err, "stats": e.list_stats()})
    assert err <= TOL_X[prec]


def test_dense_start_takes_tile_step():
    """a threshold of 48 (GCS_OPT_DENSE_NEIGHBORS; the default is 96) probes a fresh chain's density: C5's synthetic
    start (64 neighbours within the cutoff at core scale 0.5) runs the unfused tile step, C2's start (41) the list
    step; a continuing chain keeps its verdict; the tile-step trajectory matches the fp64 oracle"""
    cfg5 = resolution_scaled(InterphaseConfig(), 10.0)
    d5 = synthetic.make_c5()
    e, o = _pair(d5, cfg5, x=_f32(d5.positions), prec=32, dense_neighbors=48)
    _run_both(e, o, 4, 0, cfg5, 99)
    st = e.list_stats()
    assert st["active"] == 0 and st["builds"] == 0, st
    err = float(np.abs(e.get_positions() - o.get_positions()).max())
    assert err <= TOL_X[32], err
    cfg2 = InterphaseConfig()
    d2 = synthetic.make_c2()
    e2, _ = interphase.build_interphase(Engine, d2, cfg2, precision=32)
    e2.set_schedule(**interphase.interphase_schedule(cfg2))
    e2.run(8, first_step=0, temperature=cfg2.temperature, timestep=cfg2.timestep, seed=1)
    e2.run(8, first_step=8, temperature=cfg2.temperature, timestep=cfg2.timestep, seed=1)
    st2 = e2.list_stats()
    assert st2["active"] == 1 and st2["builds"] >= 1, st2  # (one build at the start: the period exceeds 16 steps)


def test_dense_chain_keeps_its_verdict_across_chunks():
    """a dense fp32 chain (C5's synthetic start: the tile step) run as two chunks equals one run bit for bit and
    probes its density once: the verdict holds while the chain continues"""
    cfg5 = resolution_scaled(InterphaseConfig(), 10.0)
    d5 = synthetic.make_c5()
    runs = []
    for chunks in ([6], [2, 4]):
        e, _ = interphase.build_interphase(Engine, d5, cfg5, precision=32)
        e.set_schedule(**interphase.interphase_schedule(cfg5))
        e.set_option(A.OPT_DENSE_NEIGHBORS, 48)
        first = 0
        for c in chunks:
            e.run(c, first_step=first, temperature=cfg5.temperature, timestep=cfg5.timestep, seed=99)
            first += c
        runs.append((e.get_positions(), e.run_stats()["density_probes"], e.list_stats()["active"]))
        e.close()
    assert runs[0][2] == 0 and runs[1][2] == 0  # the tile step
    assert runs[0][1] == 1 and runs[1][1] == 1, (runs[0][1], runs[1][1])
    assert np.array_equal(runs[0][0], runs[1][0])


def test_list_and_rebuild_step_agree_on_neighbour_count():
    """the pair set is the same: the mean neighbour count the list step reports equals the tile kernel's"""
    cfg = InterphaseConfig()
    c2_design = synthetic.make_c2()
    vals = []
    for fused in (2, 3):
        e, _ = interphase.build_interphase(Engine, c2_design, cfg, precision=32)
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_context(LATE)
        p = e.profile(1, first_step=LATE["step"], seed=3)
        vals.append(p["mean_neighbors"])
        e.close()
    assert vals[0] > 0 and vals[1] == pytest.approx(vals[0], rel=1e-4), vals


@precisions
def test_list_two_waves_per_tile(c1_design, prec):
    """GCS_OPT_LIST_WAVES 2 (two list segments per particle): the same bound against the oracle"""
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE, prec=prec, list_waves=2)
    _run_both(e, o, 40, LATE["step"], cfg, 7)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]


@pytest.mark.parametrize("waves,deal", [(4, ""), (4, "0120123"), (4, "3"), (2, "001"), (2, "1"),
                                        (4, "012012013"), (4, "0120120123")])
def test_list_deal_patterns(c1_design, waves, deal):
    """GCS_OPT_LIST_DEAL moves candidate chunks between a slot's list segments (even a single wave taking every
    chunk): the pair set is unchanged, so the same bound against the oracle holds and the neighbour count is equal.
    Periods >= 8 set the top bit of the option word (a negative int64 at the ABI): the pattern is still applied
    (the list build's segment counts differ from the default deal's)."""
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE, list_waves=waves, list_deal=A.list_deal(deal))
    _run_both(e, o, 40, LATE["step"], cfg, 7)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[64]
    assert e.list_stats()["deal"] == A.list_deal(deal)  # the pattern the build applied (not the default's)
    nb = []
    for d in (A.list_deal(deal), 0):  # from the same state
        s = _list_engine(c1_design, cfg, list_waves=waves, list_deal=d)
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.set_context(LATE)
        nb.append(s.profile(1, first_step=LATE["step"], seed=3)["mean_neighbors"])
    assert nb[0] == nb[1], nb


def _c2_observables(s, design):
    x = s.get_positions()
    b = np.concatenate([np.linalg.norm(x[a + 1:t] - x[a:t - 1], axis=1) for _, a, t in design.chains])
    rg = float(np.sqrt(((x - x.mean(axis=0)) ** 2).sum(axis=1).mean()))
    en, _ = s.compute_energy()
    return np.array([b.mean(), rg, en / design.n] + list(s.get_context()["wall_semiaxes"]))


def test_c2_long_horizon_list_vs_rebuild_step():
    """Long horizon at C2 from the bench state (step 300,000): 20,000 steps per trajectory, 6 seeds, through the list
    step (lists + skin + exact fallback; ~2,500 rebuilds in all) and through the rebuild step (a fresh cell list every
    step, no lists): the time-averaged <|r_i,i+1|>, Rg, E/N and wall semiaxes (samples every 2,000 steps after 4,000)
    agree within 3.5 standard errors of the difference of the seed means, every state stays finite, and the list
    step's fallbacks stay rare (< 1e-3 of particle-steps). The two paths share no neighbour machinery, so a list
    that missed partners over long runs would show here."""
    from pathlib import Path
    z = np.load(Path(__file__).resolve().parents[1] / "benchdata" / "c2_interphase_step300000.npz")
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    nseed, steps, every, skip = 6, 20000, 2000, 4000
    res = {3: [], 2: []}
    for fused in res:
        for k in range(nseed):
            s, _ = interphase.build_interphase(Engine, design, cfg, precision=32)
            s.set_schedule(**interphase.interphase_schedule(cfg))
            s.set_option(A.OPT_FUSED_STEP, fused)
            s.set_positions(z["positions"])
            s.set_context(ctx)
            samples, done = [], 0
            while done < steps:
                s.run(every, first_step=ctx["step"] + done, temperature=cfg.temperature, timestep=cfg.timestep,
                      seed=7000 + 10 * k + fused)
                done += every
                if done > skip:
                    samples.append(_c2_observables(s, design))
            assert np.isfinite(s.get_positions()).all()
            if fused == 3:
                st = s.list_stats()
                assert st["active"] == 1
                assert st["fallback_particle_steps"] < 1e-3 * design.n * steps, st
                assert st["sync_stalls"] == 0, st
            res[fused].append(np.mean(samples, axis=0))
            s.close()
    m3, m2 = np.mean(res[3], axis=0), np.mean(res[2], axis=0)
    s3 = np.std(res[3], axis=0, ddof=1) / np.sqrt(nseed)
    s2 = np.std(res[2], axis=0, ddof=1) / np.sqrt(nseed)
    zs = np.abs(m3 - m2) / np.sqrt(s3 ** 2 + s2 ** 2 + 1e-30)
    names = ["bond", "rg", "energy_per_bead", "wall_x", "wall_y", "wall_z"]
    print({n: (float(a), float(b), float(c)) for n, a, b, c in zip(names, m3, m2, zs)})
    assert (zs <= 3.5).all(), dict(zip(names, zs.tolist()))
    assert (s3[:3] > 0).all() and (s2[:3] > 0).all()


def test_c2_production_start_list_vs_rebuild_step():
    """The production start (C2 synthetic design, step 0, core scale 0.5 growing to ~0.67 over the window): 20,000
    steps per trajectory, 6 seeds, fp32, through the list step -- whose skin follows the core scale, changing level
    ~4 times (engine.hip skin_level: a re-primed grid and a rebuild at each change) -- and through the rebuild step (no
    lists): the time-averaged <|r_i,i+1|>, Rg, E/N and wall semiaxes agree within 3.5 standard errors of the difference
    of the seed means, every state stays finite, fallbacks stay rare"""
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    nseed, steps, every, skip = 6, 20000, 2000, 4000
    res = {3: [], 2: []}
    skins = []
    for fused in res:
        for k in range(nseed):
            s, _ = interphase.build_interphase(Engine, design, cfg, precision=32)
            s.set_schedule(**interphase.interphase_schedule(cfg))
            s.set_option(A.OPT_FUSED_STEP, fused)
            s.set_option(A.OPT_DENSE_NEIGHBORS, 0)
            s.set_context(interphase.initial_context(cfg))
            samples, done = [], 0
            while done < steps:
                s.run(every, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep,
                      seed=8000 + 10 * k + fused)
                done += every
                if fused == 3 and done == every:
                    skins.append(s.list_stats()["skin"])
                if done > skip:
                    samples.append(_c2_observables(s, design))
            assert np.isfinite(s.get_positions()).all()
            if fused == 3:
                st = s.list_stats()
                assert st["active"] == 1
                assert st["skin"] > skins[-1], (st, skins[-1])  # the skin grew with the core scale
                assert st["fallback_particle_steps"] < 1e-3 * design.n * steps, st
            res[fused].append(np.mean(samples, axis=0))
            s.close()
    m3, m2 = np.mean(res[3], axis=0), np.mean(res[2], axis=0)
    s3 = np.std(res[3], axis=0, ddof=1) / np.sqrt(nseed)
    s2 = np.std(res[2], axis=0, ddof=1) / np.sqrt(nseed)
    zs = np.abs(m3 - m2) / np.sqrt(s3 ** 2 + s2 ** 2 + 1e-30)
    names = ["bond", "rg", "energy_per_bead", "wall_x", "wall_y", "wall_z"]
    print({n: (float(a), float(b), float(c)) for n, a, b, c in zip(names, m3, m2, zs)})
    assert (zs <= 3.5).all(), dict(zip(names, zs.tolist()))


def test_c5_long_horizon_relative_lists_vs_tile_step():
    """C5 (606,248 particles) from its synthetic start: 6,000 steps per trajectory, 4 seeds, fp32, through the list
    step (plane-relative 16-bit entries, the core-scale skin) and through the unfused tile step (no lists): the
    time-averaged <|r_i,i+1|>, Rg, E/N and wall semiaxes (samples every 1,000 steps after 2,000) agree within 3.5
    standard errors of the difference of the seed means; every state finite; no list escapes its plane span beyond
    the exact search's rare share"""
    cfg = resolution_scaled(InterphaseConfig(), 10.0)
    design = synthetic.make_c5()
    nseed, steps, every, skip = 4, 6000, 1000, 2000
    res = {3: [], 0: []}
    for fused in res:
        for k in range(nseed):
            s, _ = interphase.build_interphase(Engine, design, cfg, precision=32)
            s.set_schedule(**interphase.interphase_schedule(cfg))
            s.set_option(A.OPT_FUSED_STEP, fused)
            s.set_option(A.OPT_DENSE_NEIGHBORS, 0)
            s.set_context(interphase.initial_context(cfg))
            samples, done = [], 0
            while done < steps:
                s.run(every, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep,
                      seed=9000 + 10 * k + fused)
                done += every
                if done > skip:
                    samples.append(_c2_observables(s, design))
            assert np.isfinite(s.get_positions()).all()
            if fused == 3:
                st = s.list_stats()
                assert st["active"] == 1
                assert st["fallback_particle_steps"] < 1e-3 * design.n * steps, st
            res[fused].append(np.mean(samples, axis=0))
            s.close()
    m3, m0 = np.mean(res[3], axis=0), np.mean(res[0], axis=0)
    s3 = np.std(res[3], axis=0, ddof=1) / np.sqrt(nseed)
    s0 = np.std(res[0], axis=0, ddof=1) / np.sqrt(nseed)
    zs = np.abs(m3 - m0) / np.sqrt(s3 ** 2 + s0 ** 2 + 1e-30)
    names = ["bond", "rg", "energy_per_bead", "wall_x", "wall_y", "wall_z"]
    print({n: (float(a), float(b), float(c)) for n, a, b, c in zip(names, m3, m0, zs)})
    assert (zs <= 3.5).all(), dict(zip(names, zs.tolist()))


@precisions
def test_second_neighbour_harmonic_nonzero_k(c1_design, prec):
    """setup_loop_forcefield (simulation_driver_forcefield.cpp:100-136) with K != 0: the (i, i+2) harmonic bonds are
    compiled in (the default config's K = 0 drops them); forces and a 40-step list-step trajectory vs the oracle"""
    import dataclasses
    cfg = dataclasses.replace(InterphaseConfig(), a_core_2nd_bond_spring=40.0, b_core_2nd_bond_spring=15.0)
    e, o = _pair(c1_design, cfg, ctx=LATE, prec=prec)
    fe, fo = e.compute_forces(), o.compute_forces()
    from tolerances import assert_forces_close
    assert_forces_close(fe, fo, prec)
    base, _ = _pair(c1_design, InterphaseConfig(), ctx=LATE, prec=prec)
    assert np.abs(base.compute_forces() - fo).max() > 1e-2  # the field changes the forces
    _run_both(e, o, 40, LATE["step"], cfg, 7)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]


def _relax_engine(design, cfg, prec, **opts):
    e = _list_engine(design, cfg, prec, **opts)
    e.set_schedule(update_time=0, update_scales=0, update_wall=0, timestep=cfg.timestep)
    return e


@precisions
def test_list_relaxation_matches_oracle(c1_design, prec):
    """the relaxation stage's step (spacestep 1e-3, simulation_driver_relaxation.cpp:48-55) on the lists:
    k_lstep<..., RLX> stores the forces and adapts the timestep in its final workgroup, k_lupdate moves the
    particles.  From C1's start (core scale 0.5, fast motion: several rebuilds), 60 steps, Philox noise, then 5 more
    from there: positions within the precision's bound, the adapted timestep equal"""
    cfg = InterphaseConfig()
    e = _relax_engine(c1_design, cfg, prec, list_every=5)
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=prec)
    o.set_schedule(update_time=0, update_scales=0, update_wall=0, timestep=cfg.timestep)
    for s in (e, o):
        s.apply_schedule(0)
    for first, k in ((0, 60), (60, 5)):
        for s in (e, o):
            s.run(k, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep,
                  spacestep=cfg.relaxation_spacestep, seed=4242)
        assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]
        assert e.get_context()["last_timestep"] == pytest.approx(o.get_context()["last_timestep"],
                                                                 rel={64: 1e-10, 32: 1e-4}[prec])
    st, rs = e.list_stats(), e.run_stats()
    assert st["active"] == 1 and st["builds"] >= 65 // 5, st
    assert rs["graph_steps"] > 0, rs
    assert e.get_context()["last_timestep"] < cfg.timestep  # the spacestep limit is active at this start


@precisions
def test_list_relaxation_graph_eager_and_chunks_bitwise_identical(c1_design, prec):
    cfg = InterphaseConfig()
    runs = []
    for g, chunks in ((0, [40]), (32, [40]), (8, [7, 20, 13])):
        e = _relax_engine(c1_design, cfg, prec, list_every=6, graph_steps=g)
        e.apply_schedule(0)
        first = 0
        for c in chunks:
            e.run(c, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep,
                  spacestep=cfg.relaxation_spacestep, seed=3)
            first += c
        runs.append((e.get_positions(), e.get_context()))
        e.close()
    for x, c in runs[1:]:
        assert np.array_equal(x, runs[0][0])
        assert c == runs[0][1]


@precisions
def test_list_relaxation_then_fixed_timestep(c1_design, prec):
    """a relaxation run followed by a fixed-timestep run continuing at its last step: the lists carry over, and the
    context reports the fixed timestep again (the relaxation's adapted one does not leak)"""
    cfg = InterphaseConfig()
    e = _relax_engine(c1_design, cfg, prec)
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=prec)
    o.set_schedule(update_time=0, update_scales=0, update_wall=0, timestep=cfg.timestep)
    for s in (e, o):
        s.apply_schedule(0)
        s.run(20, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, spacestep=cfg.relaxation_spacestep,
              seed=8)
        s.run(20, first_step=20, temperature=cfg.temperature, timestep=cfg.timestep, seed=9)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]
    assert e.get_context()["last_timestep"] == o.get_context()["last_timestep"] == cfg.timestep


@pytest.mark.parametrize("prec,pm", [(64, 350), (32, 500)])
def test_default_skin_per_precision(c1_design, prec, pm):
    """GCS_OPT_LIST_SKIN 0 (the default): 350 per mille of the cutoff at fp64 (its 32-B gathers favour shorter lists),
    500 at fp32; an explicit value applies to both"""
    cfg = InterphaseConfig()
    e = _list_engine(c1_design, cfg, prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.set_context(LATE)
    e.run(2, first_step=LATE["step"], seed=1)
    assert e.list_stats()["skin"] == pytest.approx(pm * 1e-3 * cfg.a_core_diameter, rel=1e-6)
    e.set_option(A.OPT_LIST_SKIN, 420)
    e.run(2, first_step=LATE["step"] + 2, seed=1)
    assert e.list_stats()["skin"] == pytest.approx(0.42 * cfg.a_core_diameter, rel=1e-6)


@precisions
@pytest.mark.parametrize("n", [1, 2, 65, 1025])
def test_list_relaxation_small_and_ragged_sizes(n, prec):
    """the relaxation step on the lists (k_lstep<..., RLX> + k_lupdate) at ragged sizes: random particles, several
    pair classes, a chain; spacestep 2e-3 with dt 1e-4 (the limit active), 15 steps vs the oracle"""
    rng = np.random.default_rng(100 + n)
    x = rng.uniform(-0.5, 0.5, size=(n, 3))
    ab = rng.choice([0.0, 0.5, 1.0], size=(n, 2))
    mu = rng.uniform(0.5, 1.5, size=n)
    sysd = {}
    for name, cls in (("e", Engine), ("o", oracle.OracleSystem)):
        s = cls(n, mobilities=mu, ab_factors=ab, precision=prec)
        s.add_neighbor_softcore(2.5, 0.3, 2.5, 0.24, 0.3, mix=True, scaled=True)
        if n > 1:
            s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=100.0, b_spring=50.0, mix=True, scaled=True,
                                  ranges=[(0, n)])
        s.set_context({"core_scale": 0.8, "bond_scale": 0.7, "wall_semiaxes": [1, 1, 1]})
        s.set_positions(x)
        if name == "e":
            s.set_option(A.OPT_FUSED_STEP, 3)
            s.set_option(A.OPT_DENSE_NEIGHBORS, 0)
        sysd[name] = s
    for s in sysd.values():
        s.run(15, seed=2, timestep=1e-4, spacestep=2e-3)
    assert np.abs(sysd["e"].get_positions() - sysd["o"].get_positions()).max() <= TOL_X[prec]
    assert sysd["e"].get_context()["last_timestep"] == pytest.approx(sysd["o"].get_context()["last_timestep"],
                                                                    rel={64: 1e-10, 32: 1e-4}[prec])


@precisions
def test_list_phase_staggers_rebuilds(c1_design, prec):
    """GCS_OPT_LIST_PHASE (staggered replicas): rebuilds at steps s with (s + phase) % period == 0 -- another set of
    rebuild steps, so other list orders and sums (not bitwise), but the same pair set: within the precision's bound of
    the oracle, chunked runs bitwise equal to one run at the same phase"""
    cfg = InterphaseConfig()
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=prec)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.set_context(LATE)
    o.run(48, first_step=LATE["step"], temperature=cfg.temperature, timestep=cfg.timestep, seed=11)
    xs = {}
    for phase, chunks in ((0, (48,)), (3, (48,)), (3, (20, 28))):
        e = _list_engine(c1_design, cfg, prec, list_every=8, list_phase=phase)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_context(LATE)
        st = LATE["step"]
        for c in chunks:
            e.run(c, first_step=st, temperature=cfg.temperature, timestep=cfg.timestep, seed=11)
            st += c
        xs[(phase, chunks)] = (e.get_positions(), e.list_stats())
        assert np.abs(xs[(phase, chunks)][0] - o.get_positions()).max() <= TOL_X[prec]
    assert np.array_equal(xs[(3, (48,))][0], xs[(3, (20, 28))][0])
    assert xs[(3, (48,))][1]["builds"] == xs[(3, (20, 28))][1]["builds"]


def test_list_skin_base(c1_design):
    """GCS_OPT_LIST_SKIN_BASE (the stage drivers' one-trajectory skin, gcs/interphase.py SINGLE_SKIN_BASE_F64): the
    default skin follows s1 sqrt(cs) with s1 = 400 instead of 350 per mille (fp64) -- longer lists, fewer rebuilds,
    the same pair set: within the fp64 bound of the oracle; 0 is the default again"""
    cfg = InterphaseConfig()
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=64)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.set_context(LATE)
    o.run(48, first_step=LATE["step"], temperature=cfg.temperature, timestep=cfg.timestep, seed=11)
    stats = {}
    for base in (0, 400):
        e = _list_engine(c1_design, cfg, 64, list_skin_base=base)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_context(LATE)
        e.run(48, first_step=LATE["step"], temperature=cfg.temperature, timestep=cfg.timestep, seed=11)
        assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[64]
        stats[base] = e.list_stats()
        e.close()
    assert stats[400]["skin"] == pytest.approx(stats[0]["skin"] * 400 / 350, rel=1e-5)
    assert stats[400]["rebuild_every"] > stats[0]["rebuild_every"]


def _format_run(design, cfg, prec, fmt, steps, ctx=LATE, seed=11, **opts):
    e = _list_engine(design, cfg, prec, list_format=fmt, **opts)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.set_context(ctx)
    e.run(steps, first_step=ctx["step"], temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
    return e.get_positions(), e.list_stats()


@precisions
@pytest.mark.parametrize("fmt", [1, 2])
def test_list_formats_bitwise_c1(c1_design, prec, fmt):
    """GCS_OPT_LIST_FORMAT: plane-relative 16-bit slots (1, kernels.hip ListRel16) and 32-bit slots (2) hold the same
    pairs in the same order as the default absolute 16-bit slots (0): the trajectory (list rebuilds included) is
    bitwise the same, with the same particles searched exactly"""
    cfg = InterphaseConfig()
    x0, s0 = _format_run(c1_design, cfg, prec, 0, 60)
    x1, s1 = _format_run(c1_design, cfg, prec, fmt, 60)
    assert s0["builds"] == s1["builds"] and s0["builds"] >= 2, (s0, s1)
    assert s0["fallback_particle_steps"] == s1["fallback_particle_steps"]
    assert np.array_equal(x0, x1)


@precisions
def test_relative_entries_c5_bitwise(prec):
    """N > 65,536 (C5, 606,248 particles, its dense synthetic start): the plane-relative 16-bit slots (the default
    there) against 32-bit slots -- every partner within the plane span (no escape to the exact search), so bitwise
    the same"""
    cfg = resolution_scaled(InterphaseConfig(), 10.0)
    design = synthetic.make_c5()
    ctx = {"step": 0, "time": 0.0, "core_scale": 1.0, "bond_scale": 1.0, "wall_semiaxes": LATE["wall_semiaxes"]}
    x2, s2 = _format_run(design, cfg, prec, 2, 20, ctx=ctx)
    x1, s1 = _format_run(design, cfg, prec, 1, 20, ctx=ctx)
    assert s1["fallback_particle_steps"] == s2["fallback_particle_steps"], (s1, s2)
    assert np.array_equal(x1, x2)


@precisions
def test_relative_entries_escape_to_exact_search(prec):
    """A 100,000-particle rod (cross-section of two or three list cells: cell rows of ~11,000-25,000 slots) puts a
    particle's partners in the row above up to ~22,000 slots past its plane base, beyond the 14-bit offset: those
    lists are marked overflowed and the particles searched exactly.  Same bound vs the oracle (softcore only, 5
    steps), and the exact searches happened.  (Lengths at a tenth of the nucleus' scale -- cutoff 0.03, rod 10 long
    -- so coordinates stay below 10, where the fp32 bound applies; timestep scaled to move particles alike.)"""
    n = 100000
    rng = np.random.default_rng(7)
    x = np.column_stack([rng.uniform(0, 10, n), rng.uniform(0, 0.13, n), rng.uniform(0, 0.13, n)])
    sysd = {}
    for name, cls in (("e", Engine), ("o", oracle.OracleSystem)):
        s = cls(n, precision=prec)
        s.add_neighbor_softcore(2.5, 0.03, 2.5, 0.024, 0.03, mix=False, scaled=False)
        s.set_positions(x)
        if name == "e":
            s.set_option(A.OPT_FUSED_STEP, 3)
            s.set_option(A.OPT_DENSE_NEIGHBORS, 0)
            s.set_option(A.OPT_LIST_FORMAT, 1)
        sysd[name] = s
    for s in sysd.values():
        s.run(5, seed=3, timestep=1e-7)
    st = sysd["e"].list_stats()
    assert st["active"] == 1 and st["fallback_particle_steps"] > 0, st
    assert np.abs(sysd["e"].get_positions() - sysd["o"].get_positions()).max() <= TOL_X[prec]


@precisions
def test_skin_follows_core_scale(c1_design, prec):
    """GCS_OPT_LIST_SKIN 0: the skin follows the scheduled core scale (engine.hip skin_level: 250 per mille at core
    scale 0.5 for fp64's 350 (x sqrt(cs)) and for fp32's 500 (x cs)), changing at steps fixed by the schedule -- each change re-primes
    and rebuilds.  A fast core-scale schedule (0.5 -> 0.93 over 120 steps) crosses several skin levels: the run in
    three chunks is bitwise the run in one, both within the bound of the oracle, and the skin ends larger"""
    cfg = InterphaseConfig()
    sched = dict(interphase.interphase_schedule(cfg), core_scale_tau=100 * cfg.timestep / 2.0)
    ctx0 = interphase.initial_context(cfg)
    runs = []
    for chunks in ((120,), (37, 50, 33)):
        e = _list_engine(c1_design, cfg, prec)
        e.set_schedule(**sched)
        e.set_context(ctx0)
        e.run(1, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=21)
        skin0 = e.list_stats()["skin"]
        first = 1
        for c in chunks:
            e.run(c, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep, seed=21)
            first += c
        runs.append((e.get_positions(), skin0, e.list_stats()))
    (x1, skin0, st1), (x3, _, st3) = runs
    assert skin0 == pytest.approx({64: 0.250, 32: 0.250}[prec] * cfg.a_core_diameter, rel=1e-6)
    assert st1["skin"] > skin0 and st1["skin"] == st3["skin"] and st1["builds"] == st3["builds"], (st1, st3)
    assert np.array_equal(x1, x3)
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=prec)
    o.set_schedule(**sched)
    o.set_context(ctx0)
    o.run(121, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=21)
    assert np.abs(x1 - o.get_positions()).max() <= TOL_X[prec]


def _classes_system(cls, n, nclass, prec, rng_seed=5, **opts):
    """n particles in a cube at ~C2's density, softcore A/B with `nclass` distinct (a, b) factor pairs (continuous
    values, as chains TSVs give: stage_prepare/chains.cpp:55-56) and an ellipsoid wall"""
    rng = np.random.default_rng(rng_seed)
    side = (n / 220.0) ** (1.0 / 3.0)
    x = rng.uniform(0, side, (n, 3))
    table = rng.uniform(0.4, 1.6, (nclass, 2))
    ab = table[rng.integers(0, nclass, n)]
    ab[:nclass] = table  # every class present
    s = cls(n, ab_factors=ab, precision=prec)
    s.add_neighbor_softcore(2.0, 0.3, 1.5, 0.24, 0.3, mix=True, scaled=False)
    s.add_ellipsoid_inward(5.0, 0.3, 0.0, 1.0, center=(side / 2,) * 3)
    s.set_context({"core_scale": 1.0, "bond_scale": 1.0, "wall_semiaxes": [0.45 * side] * 3})
    s.set_positions(x)
    for k, v in opts.items():
        s.set_option(getattr(A, "OPT_" + k.upper()), v)
    return s


@precisions
def test_many_pair_classes_take_the_cell_list_step(prec):
    """More than 256 distinct (a, b) pair classes (1,500 continuous factor pairs): the list step does not admit the
    system; the default engine then runs its cell-list step (fp64: k_eval64 + k_red64 + k_update + k_tail; fp32: the
    rebuild step) instead of failing, within the precision's bound of the oracle"""
    n = 1500
    e = _classes_system(Engine, n, 1500, prec)
    o = _classes_system(oracle.OracleSystem, n, 1500, prec)
    for s in (e, o):
        s.run(25, seed=9, timestep=1e-5, temperature=1.0)
    assert e.list_stats()["active"] == 0
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X[prec]
