"""GPU: the HIP engine (through the C ABI) against the committed golden vectors (tests/golden/oracle_golden.npz, the
fp64 oracle's outputs on the cases of tests/golden_cases.py; tests/test_golden.py pins them on the CPU). The only
oracle code used here is the reference-order noise stream (mt19937_64 + libstdc++ normal_distribution, itself pinned
by tests/golden/rng_fixtures.json); every expected value comes from the committed vectors.

Tolerances, fp64 engine (default) / fp32 engine vs the fp64 vectors: two-particle KATs |dE| <= 1e-10 / 1e-5 max|E|
+ 1e-12 / 1e-6, |dF| <= 1e-10 / 1e-5 max|F| + 1e-10 / 1e-5; C1 forces, energies and positions after 1 and 10 steps
with the injected reference noise as tests/tolerances.py; pair sets bit-exact (the strict predicate in the engine's
precision: c1_pairs64_* / c1_pairs_*); quantize bit-exact."""
import functools
from pathlib import Path

import numpy as np
import pytest

import golden_cases as G
from gcs.engine import Engine
from tolerances import E_ABS, E_REL, WALL_REL, X, assert_forces_close, precisions

pytestmark = pytest.mark.gpu

GOLD = np.load(Path(__file__).parent / "golden" / "oracle_golden.npz")


KAT_TOL = {64: (1e-10, 1e-12, 1e-10, 1e-10), 32: (1e-5, 1e-6, 1e-5, 1e-5)}  # energy rel, abs; force rel, abs


@precisions
@pytest.mark.parametrize("name", sorted(G.KATS))
def test_kats(name, prec):
    e, f = G.kat_eval(G.KATS[name], functools.partial(Engine, precision=prec))
    ge, gf = GOLD[f"kat_{name}_e"], GOLD[f"kat_{name}_f"]
    er, ea, fr, fa = KAT_TOL[prec]
    assert np.abs(e - ge).max() <= er * np.abs(ge).max() + ea, (e, ge)
    assert np.abs(f - gf).max() <= fr * np.abs(gf).max() + fa, (f, gf)


@precisions
def test_c1_pairs(prec):
    e = Engine(16, precision=prec)
    key = "c1_pairs64" if prec == 64 else "c1_pairs"
    for d in G.PAIR_DISTANCES:
        got = e.search_neighbors(d, points=GOLD["c1_x0"])
        assert np.array_equal(got.astype(np.int32), GOLD[f"{key}_{int(round(d * 100)):03d}"])


@precisions
def test_c1_forces_and_energy(prec):
    s, _, _ = G.c1_system(functools.partial(Engine, precision=prec))
    assert_forces_close(s.compute_forces(), GOLD["c1_forces"], prec)
    tot, parts = s.compute_energy()
    assert tot == pytest.approx(float(GOLD["c1_energy"][0]), rel=E_REL[prec])
    assert np.allclose(parts, GOLD["c1_energy_parts"], rtol=E_REL[prec], atol=E_ABS[prec])


@precisions
@pytest.mark.parametrize("steps,key", [(1, "c1_step1"), (G.TRAJ_STEPS, "c1_traj10")])
def test_c1_trajectory_injected_noise(steps, key, prec):
    s, design, cfg = G.c1_system(functools.partial(Engine, precision=prec))
    x, c = G.c1_run(s, cfg, G.c1_noise(design.n)[:steps], steps)
    assert np.abs(x - GOLD[key]).max() <= X[prec]
    if steps == G.TRAJ_STEPS:
        assert np.allclose(c["wall_semiaxes"], GOLD["c1_traj10_wall"], rtol=max(WALL_REL[prec], 1e-9))
        assert c["core_scale"] == pytest.approx(float(GOLD["c1_traj10_core_scale"][0]), rel=1e-12)


@precisions
def test_quantize_table(prec):
    q = GOLD["quantize_in"]
    e = Engine(q.size // 3 + 1, precision=prec)
    x = np.zeros((e.n, 3))
    x.ravel()[:q.size] = q
    e.set_positions(x)
    got = e.sample_positions().astype(np.float64).ravel()[:q.size]
    # the store writes f32 after quantising (simulation_store.cpp:192-216): the fp64 table cast to f32
    assert np.array_equal(got, GOLD["quantize_out"].astype(np.float32).astype(np.float64))
