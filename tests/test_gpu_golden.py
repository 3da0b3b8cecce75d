"""GPU: the HIP engine (through the C ABI) against the committed golden vectors (tests/golden/oracle_golden.npz, the
fp64 oracle's outputs on the cases of tests/golden_cases.py; tests/test_golden.py pins them on the CPU). The only
oracle code used here is the reference-order noise stream (mt19937_64 + libstdc++ normal_distribution, itself pinned
by tests/golden/rng_fixtures.json); every expected value comes from the committed vectors.

Tolerances (fp32 device vs fp64 vectors): two-particle KATs |dE| <= 1e-5 max|E| + 1e-6, |dF| <= 1e-5 max|F| + 1e-5;
C1 forces |dF| <= 1e-4 max|F| + 1e-3 (tests/test_gpu_parity.py), energy relative 1e-5; pair sets bit-exact (strict
fp32 predicate); positions after 1 and 10 steps with the injected reference noise |dx| <= 2e-5, wall semiaxes
relative 1e-9; quantize bit-exact."""
from pathlib import Path

import numpy as np
import pytest

import golden_cases as G
from gcs.engine import Engine

pytestmark = pytest.mark.gpu

GOLD = np.load(Path(__file__).parent / "golden" / "oracle_golden.npz")


@pytest.mark.parametrize("name", sorted(G.KATS))
def test_kats(name):
    e, f = G.kat_eval(G.KATS[name], Engine)
    ge, gf = GOLD[f"kat_{name}_e"], GOLD[f"kat_{name}_f"]
    assert np.abs(e - ge).max() <= 1e-5 * np.abs(ge).max() + 1e-6, (e, ge)
    assert np.abs(f - gf).max() <= 1e-5 * np.abs(gf).max() + 1e-5, (f, gf)


def test_c1_pairs():
    e = Engine(16)
    for d in G.PAIR_DISTANCES:
        got = e.search_neighbors(d, points=GOLD["c1_x0"])
        assert np.array_equal(got.astype(np.int32), GOLD[f"c1_pairs_{int(round(d * 100)):03d}"])


def test_c1_forces_and_energy():
    s, _, _ = G.c1_system(Engine)
    f = s.compute_forces()
    scale = np.abs(GOLD["c1_forces"]).max()
    assert np.abs(f - GOLD["c1_forces"]).max() <= 1e-4 * scale + 1e-3
    tot, parts = s.compute_energy()
    assert tot == pytest.approx(float(GOLD["c1_energy"][0]), rel=1e-5)
    assert np.allclose(parts, GOLD["c1_energy_parts"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("steps,key", [(1, "c1_step1"), (G.TRAJ_STEPS, "c1_traj10")])
def test_c1_trajectory_injected_noise(steps, key):
    s, design, cfg = G.c1_system(Engine)
    x, c = G.c1_run(s, cfg, G.c1_noise(design.n)[:steps], steps)
    assert np.abs(x - GOLD[key]).max() <= 2e-5
    if steps == G.TRAJ_STEPS:
        assert np.allclose(c["wall_semiaxes"], GOLD["c1_traj10_wall"], rtol=1e-9)
        assert c["core_scale"] == pytest.approx(float(GOLD["c1_traj10_core_scale"][0]), rel=1e-12)


def test_quantize_table():
    q = GOLD["quantize_in"]
    e = Engine(q.size // 3 + 1)
    x = np.zeros((e.n, 3))
    x.ravel()[:q.size] = q
    e.set_positions(x)
    got = e.sample_positions().astype(np.float64).ravel()[:q.size]
    # the store writes f32 after quantising (simulation_store.cpp:192-216): the fp64 table cast to f32
    assert np.array_equal(got, GOLD["quantize_out"].astype(np.float32).astype(np.float64))
