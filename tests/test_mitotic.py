"""Mitotic stages (C3) on the CPU: prepare's coarse-graining (prepare.cpp:279-372), the libstdc++ normal stream of
the anaphase initialisation (stage_anatelophase/simulation_driver.cpp:25-32, pinned by the g++ fixtures), and the drivers' stage
order / field swap on the oracle backend."""
import json
from pathlib import Path

import numpy as np
import pytest

from gcs import mitotic, synthetic
from gcs.config import MitoticPhaseConfig
from gcs.seeds import MT19937_64

import oracle

FIX = json.loads((Path(__file__).parent / "golden" / "rng_fixtures.json").read_text())


@pytest.fixture(scope="module")
def c3():
    cfg = MitoticPhaseConfig()
    i = synthetic.make_c2()
    a = mitotic.anatelophase_design(i, cfg)
    p = mitotic.prometaphase_design(a, cfg, i.master_seed)
    return cfg, i, a, p


def test_coarse_grained_designs(c3):
    cfg, i, a, p = c3
    assert a.n == sum((e - s) // cfg.coarse_graining for _, s, e in i.chains) == 586
    assert p.n == 2 * a.n == 1172
    assert len(a.chains) == 46 and len(p.chains) == 92 and len(p.sister_chromatids) == 46
    for (_, s, e, k), (_, istart, _), (cs, ce) in zip(a.chains, i.chains, i.centromeres):
        assert s <= k < e and a.particle_types[k] == mitotic.T_KINETOCHORE
        assert k - s == ((cs + ce) // 2 - istart) // cfg.coarse_graining  # prepare.cpp:289-291
    assert (a.particle_types == mitotic.T_KINETOCHORE).sum() == 46
    for (t, sis), ((_, ts, te, tk), (_, ss, se, sk)) in zip(p.sister_chromatids, zip(p.chains[0::2], p.chains[1::2])):
        assert p.chains[t][3] == tk and p.chains[sis][3] == sk
        assert te == ss and tk - ts == sk - ss
    assert np.allclose(p.pole_positions, [[0, -5, 0], [0, 5, 0]])


def test_std_normal_matches_libstdcxx(c3):
    for case in FIX["normal_distribution"]:
        nd = mitotic.StdNormal(MT19937_64(case["seed"]))
        got = [nd() for _ in range(len(case["values"]))]
        assert got == case["values"]


def test_normal_vector_uses_a_fresh_distribution():
    """each normal_vector() builds its own normal_distribution: the cached 4th value is dropped"""
    stream = oracle.reference_normals(123, 8)
    g = MT19937_64(123)
    v1 = mitotic.normal_vector(g)
    v2 = mitotic.normal_vector(g)
    assert v1.tolist() == list(stream[:3]) and v2.tolist() == list(stream[4:7])


def test_anatelophase_driver_on_oracle(c3):
    cfg, _, a, _ = c3
    o, h = mitotic.build_anatelophase(oracle.OracleSystem, a, cfg)
    drv = mitotic.AnatelophaseDriver(o, h, a, cfg, log=None)
    drv.run(anaphase_steps=20, telophase_steps=20)
    x = o.get_positions()
    assert np.isfinite(x).all()
    assert set(drv.h) == {"repulsion", "packing", "telophase_bonds", "telophase_bending"}
    # the rods start around -spindle_axis
    drv2 = mitotic.AnatelophaseDriver(o, h, a, cfg, log=None)
    r = drv2.initial_rods()
    assert abs(r[:, 1].mean() + 5.0) < 1.0
    for _, s, e, _ in a.chains:
        d = np.linalg.norm(np.diff(r[s:e], axis=0), axis=1)
        assert np.allclose(d, cfg.bond_length)


def test_prometaphase_driver_on_oracle(c3):
    cfg, _, a, p = c3
    o, _ = mitotic.build_prometaphase(oracle.OracleSystem, p, cfg)
    x0 = np.concatenate([np.random.default_rng(1).normal(scale=1.0, size=(p.n, 3))])
    drv = mitotic.PrometaphaseDriver(o, p, cfg, log=None)
    drv.run(x0, steps=10)
    assert np.isfinite(o.get_positions()).all() and drv.time == pytest.approx(10 * cfg.timestep)
    with pytest.raises(RuntimeError):
        drv.run(x0[:-1], steps=1)
