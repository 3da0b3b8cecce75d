"""GPU: the spatial domain decomposition (C5, gcs/domain.py + csrc/domain.hip) with HIP engines, several domains in
one process on one device (LocalTransport), against the undecomposed engine and the fp64 oracle.

Tolerances: positions |dx| <= 2e-5 after 30 steps (fp32; the domains' cell lists order the pair sums differently
from the single engine's), wall semiaxes relative 1e-7; the protocol flags (bond beyond the halo, band over
capacity) must stay clear."""
import numpy as np
import pytest

from gcs import domain, interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine

import oracle

pytestmark = pytest.mark.gpu

STEPS = 30
SEED = 99


def _engine(design, cfg):
    e, _ = interphase.build_interphase(Engine, design, cfg, device=0)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    return e


def _decomposed(design, cfg, ndom, steps, cap=None, halo=None):
    halo = halo or domain.domain_halo(cfg)
    slabs = domain.plan_slabs(design.positions[:, 2], ndom)
    sh = domain.shared_particles(design)
    doms = [domain.EngineDomain(_engine(design, cfg), d, slabs, halo, cap=cap, device=0, shared=sh)
            for d in range(ndom)]
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    run.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    return run, doms, slabs


@pytest.mark.parametrize("ndom,halo", [(2, None), (4, None), (3, 0.45)])
def test_decomposed_engines_match_single_engine_c1(c1_design, ndom, halo):
    cfg = InterphaseConfig()
    single = _engine(c1_design, cfg)
    single.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1, c1 = single.get_positions(), single.get_context()
    run, doms, slabs = _decomposed(c1_design, cfg, ndom, STEPS, halo=halo)
    run.check()
    x = domain.gather_positions(run, c1_design.n)
    assert np.abs(x - x1).max() <= 2e-5
    for d in doms:
        c = d.context()
        assert c["step"] == c1["step"]
        assert np.allclose(c["wall_semiaxes"], c1["wall_semiaxes"], rtol=1e-7, atol=0)
    # and against the fp64 oracle's undecomposed run
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert np.abs(x - o.get_positions()).max() <= 2e-5


def test_decomposed_engines_c2_four_domains():
    cfg = InterphaseConfig()
    design = synthetic.make_c2()
    single = _engine(design, cfg)
    single.run(20, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1 = single.get_positions()
    run, doms, _ = _decomposed(design, cfg, 4, 20)
    run.check()
    x = domain.gather_positions(run, design.n)
    assert np.abs(x - x1).max() <= 2e-5


def test_band_capacity_overflow_is_reported(c1_design):
    cfg = InterphaseConfig()
    run, _, _ = _decomposed(c1_design, cfg, 2, 2, cap=8)
    with pytest.raises(domain.DomainError):
        run.check()


def test_bond_beyond_halo_is_reported(c1_design):
    """A halo below the chain bonds' length (C1 starts with every bond 0.1 long): the pack kernel flags it."""
    cfg = InterphaseConfig()
    run, _, _ = _decomposed(c1_design, cfg, 2, 2, halo=0.09)
    with pytest.raises(domain.DomainError, match="bond"):
        run.check()


def test_decomposed_c5_scaled_two_domains():
    """C5 (606,248 beads, the 10 kb force field and timestep of config.resolution_scaled), 2 domains and one engine,
    each against the fp64 oracle under the absolute C5 bound of tests/test_gpu_parity_long.py (2e-5 after 10
    steps; the derivation is there and in DESIGN.md §6)."""
    from gcs.config import resolution_scaled
    cfg = resolution_scaled(InterphaseConfig(), 10.0)
    design = synthetic.make_c5()
    steps = 10
    single = _engine(design, cfg)
    single.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1 = single.get_positions()
    run, doms, _ = _decomposed(design, cfg, 2, steps)
    run.check()
    x = domain.gather_positions(run, design.n)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.set_positions(np.asarray(design.positions, dtype=np.float32).astype(np.float64))
    o.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    xo = o.get_positions()
    e_single = np.abs(x1 - xo).max()
    e_dec = np.abs(x - xo).max()
    assert np.isfinite(x).all()
    assert e_single <= 2e-5 and e_dec <= 2e-5, (e_dec, e_single)
