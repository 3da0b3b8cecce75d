"""GPU, long horizon: the persistent small-system step (kernels.hip k_pstep, the default for every mitotic stage)
against the list step (GCS_OPT_SMALL_STEP 0) over the reference's stage lengths' order of magnitude (VERDICT r5 item
5; the reference runs 200k + 50k anaphase/telophase and 400k prometaphase steps per cycle,
common/simulation_config.hpp:20-22, stage_anatelophase/simulation_driver.cpp:262-268, 303-309,
stage_prometaphase/simulation_driver.cpp:230-236).

Both paths compute the same pair set with sums in another order, so their trajectories separate (the dynamics is
chaotic) and agree only in distribution: per seed the time-averaged bond length, radius of gyration, energy per
particle and kinetochore-to-pole distance over 50,000 steps (samples every 2,500 after the first 10,000), then the seed
means of the two paths within 3.5 standard errors of their difference.  A stalled hand-off fails the run (GCS_ESTATE,
engine.hip run_small), so every completed run also proves that no workgroup gave up."""
import dataclasses

import numpy as np
import pytest

from gcs import _abi as A
from gcs import mitotic, synthetic
from gcs.config import MitoticPhaseConfig
from gcs.engine import Engine

pytestmark = pytest.mark.gpu

NSEED, STEPS, EVERY, SKIP = 6, 50000, 2500, 10000
NAMES = ["bond", "rg", "energy_per_particle", "kinetochore_pole"]


def _observables(s, design, kin_pole):
    x = s.get_positions()
    b = np.concatenate([np.linalg.norm(x[a + 1:t] - x[a:t - 1], axis=1) for _, a, t, _ in design.chains])
    rg = float(np.sqrt(((x - x.mean(axis=0)) ** 2).sum(axis=1).mean()))
    en, _ = s.compute_energy()
    kp = float(np.mean([np.linalg.norm(x[k] - p) for k, p in kin_pole]))
    return [float(b.mean()), rg, en / design.n, kp]


def _series(s, design, kin_pole, seed, cfg):
    out, done = [], 0
    while done < STEPS:
        s.run(EVERY, first_step=done, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed)
        done += EVERY
        if done > SKIP:
            out.append(_observables(s, design, kin_pole))
    assert np.isfinite(s.get_positions()).all()
    return np.mean(out, axis=0)


def _compare(res):
    m1, m0 = np.mean(res[1], axis=0), np.mean(res[0], axis=0)
    s1 = np.std(res[1], axis=0, ddof=1) / np.sqrt(NSEED)
    s0 = np.std(res[0], axis=0, ddof=1) / np.sqrt(NSEED)
    zs = np.abs(m1 - m0) / np.sqrt(s1 ** 2 + s0 ** 2 + 1e-30)
    print({n: (float(a), float(b), float(c)) for n, a, b, c in zip(NAMES, m1, m0, zs)})
    assert (zs <= 3.5).all(), dict(zip(NAMES, zs.tolist()))
    assert (s1 > 0).all() and (s0 > 0).all()  # the seeds do differ


def test_anaphase_small_step_vs_list_step_long():
    """586-bead anaphase (rods init, kinetochore fibers dragging to the pole), fp64: 6 seeds x 50,000 steps through
    k_pstep and through the list step"""
    cfg = MitoticPhaseConfig()
    idesign = synthetic.make_c2()
    pole = np.asarray(cfg.anaphase_spindle_shift, dtype=np.float64)
    res = {1: [], 0: []}
    for k in range(NSEED):
        a = mitotic.anatelophase_design(idesign, cfg, master_seed=101 + k)
        kin_pole = [(kin, pole) for _, _, _, kin in a.chains]
        for small in res:
            s, h = mitotic.build_anatelophase(Engine, a, cfg)
            s.set_option(A.OPT_SMALL_STEP, small)
            drv = mitotic.AnatelophaseDriver(s, h, a, cfg, log=None)
            drv.run_initialization()  # the same rods on both paths (the design's mt19937_64 stream)
            specs = mitotic._kfiber_specs(a, cfg, range(len(a.chains)), cfg.kfiber_decay_rate_anaphase,
                                          cfg.kfiber_length_anaphase)
            s.add_kinetochore_fiber(pole, specs)  # run_dragging_stage's field (:232-262)
            res[small].append(_series(s, a, kin_pole, drv.random(), cfg))
            st = s.run_stats()
            assert (st["eager_steps"] >= STEPS) if small else (st["graph_steps"] > 0), st
            s.close()
    _compare(res)


def test_prometaphase_small_step_vs_list_step_long():
    """1,172-bead prometaphase (sister bonds, fibers to both poles, polar ejection on), fp64: 6 seeds x 50,000
    steps through k_pstep and through the list step, from the sister-pair structure of the C3 parity test"""
    cfg = dataclasses.replace(MitoticPhaseConfig(), polar_ejection_force=0.5, polar_ejection_cross_section=0.09,
                              kfiber_length_prometaphase=1.0)
    i = synthetic.make_c2()
    a = mitotic.anatelophase_design(i, cfg)
    p = mitotic.prometaphase_design(a, cfg, i.master_seed)
    tp, sp = p.pole_positions
    kin_pole = [(p.chains[t][3], tp) for t, _ in p.sister_chromatids] + \
               [(p.chains[s_][3], sp) for _, s_ in p.sister_chromatids]
    rng = np.random.default_rng(11)
    x0 = np.zeros((p.n, 3))
    for (_, ts, te, _), (_, ss, se, _) in zip(p.chains[0::2], p.chains[1::2]):
        c = rng.normal(scale=1.0, size=3)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        for k in range(te - ts):
            x0[ts + k] = c + (k - (te - ts) / 2) * cfg.bond_length * d
            x0[ss + k] = x0[ts + k] + [0.0, cfg.sister_separation, 0.0]
    res = {1: [], 0: []}
    for k in range(NSEED):
        for small in res:
            s, _ = mitotic.build_prometaphase(Engine, p, cfg)
            s.set_option(A.OPT_SMALL_STEP, small)
            s.set_positions(x0)
            res[small].append(_series(s, p, kin_pole, 5000 + k, cfg))
            s.close()
    _compare(res)
