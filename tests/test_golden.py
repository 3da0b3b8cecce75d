"""CPU: the committed golden vectors (tests/golden/oracle_golden.npz) against closed forms of the
reference's potentials (for the two-particle KATs) and against a fresh run of the oracle (every item: the oracle
must not drift from the vectors the engine is checked against in tests/test_gpu_golden.py).

Tolerances: closed forms relative 1e-12; oracle re-runs relative 1e-9 (the same fp64 code; the library is built
with -funsafe-math-optimizations, so a different compiler may reassociate)."""
import math
from pathlib import Path

import numpy as np
import pytest

import golden_cases as G
import oracle

GOLD = np.load(Path(__file__).parent / "golden" / "oracle_golden.npz")


def test_kat_closed_forms():
    r = GOLD["kat_r"]
    assert np.array_equal(r, G.KAT_R)
    # softcore A/B (simulation_driver_forcefield.cpp:32-47), pair means a = 0.75, b = 0.25
    a, b = 0.75, 0.25
    e = np.where(r < 0.3, a * 2.5 * (1 - (r / 0.3) ** 2) ** 3, 0) + np.where(r < 0.24, b * 2.5 * (1 - (r / 0.24) ** 8) ** 3, 0)
    f = (np.where(r < 0.3, a * 2.5 * 3 * (1 - (r / 0.3) ** 2) ** 2 * 2 * r / 0.3 ** 2, 0)
         + np.where(r < 0.24, b * 2.5 * 3 * (1 - (r / 0.24) ** 8) ** 2 * 8 * r ** 7 / 0.24 ** 8, 0))
    assert np.allclose(GOLD["kat_softcore_e"], e, rtol=1e-12, atol=1e-14)
    assert np.allclose(GOLD["kat_softcore_f"], f, rtol=1e-12, atol=1e-12)
    # semispring K = 100, l = 0.1, one-sided
    assert np.allclose(GOLD["kat_semispring_e"], np.where(r > 0.1, 50 * (r - 0.1) ** 2, 0), rtol=1e-12, atol=1e-14)
    assert np.allclose(GOLD["kat_semispring_f"], np.where(r > 0.1, -100 * (r - 0.1), 0), rtol=1e-12, atol=1e-12)
    # softwell<6>(0.3, 0.2) truncated at 0.4 without shift
    u = (r / 0.2) ** 6
    assert np.allclose(GOLD["kat_softwell_e"], np.where(r < 0.4, -0.3 / (1 + u), 0), rtol=1e-12, atol=1e-14)
    fw = np.where(r < 0.4, -0.3 * 6 * u / r.clip(1e-300) / (1 + u) ** 2, 0)
    assert np.allclose(GOLD["kat_softwell_f"], fw, rtol=1e-12, atol=1e-12)
    # force flux (force_flux_potential.hpp:24-37): U = b f atan2(b, r), F = f b^2 / (b^2 r + r^3) r_vec
    # (particle 0 sits on the source and adds its own constant b f atan2(b, 0))
    assert np.allclose(GOLD["kat_force_flux_e"], 0.4 * 0.7 * (np.arctan2(0.4, r) + math.pi / 2), rtol=1e-12)
    ff = np.where(r > 0, 0.7 * 0.16 / (0.16 * r + r ** 3).clip(1e-300) * r, 0)
    assert np.allclose(GOLD["kat_force_flux_f"], ff, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", sorted(G.KATS))
def test_oracle_reproduces_kats(name):
    e, f = G.kat_eval(G.KATS[name], oracle.OracleSystem)
    assert np.allclose(e, GOLD[f"kat_{name}_e"], rtol=1e-9, atol=1e-13)
    assert np.allclose(f, GOLD[f"kat_{name}_f"], rtol=1e-9, atol=1e-12)


def test_oracle_reproduces_c1():
    s, design, cfg = G.c1_system(oracle.OracleSystem)
    assert np.array_equal(np.asarray(design.positions, dtype=np.float64), GOLD["c1_x0"])
    for d in G.PAIR_DISTANCES:
        exp = GOLD[f"c1_pairs_{int(round(d * 100)):03d}"]
        assert np.array_equal(oracle.search_neighbors(GOLD["c1_x0"], d, 32), exp)
        exp64 = GOLD[f"c1_pairs64_{int(round(d * 100)):03d}"]
        assert np.array_equal(oracle.search_neighbors(GOLD["c1_x0"], d, 64), exp64)
    assert np.allclose(s.compute_forces(), GOLD["c1_forces"], rtol=1e-9, atol=1e-9)
    tot, parts = s.compute_energy()
    assert tot == pytest.approx(float(GOLD["c1_energy"][0]), rel=1e-10)
    assert np.allclose(parts, GOLD["c1_energy_parts"], rtol=1e-10, atol=1e-12)
    xi = G.c1_noise(design.n)
    x10, c10 = G.c1_run(s, cfg, xi, G.TRAJ_STEPS)
    assert np.allclose(x10, GOLD["c1_traj10"], rtol=0, atol=1e-11)
    assert np.allclose(c10["wall_semiaxes"], GOLD["c1_traj10_wall"], rtol=1e-12)


def test_quantize_table():
    # simulation_store.cpp:22-33: frexp mantissa rounded to 16 fraction bits
    for v, q in zip(GOLD["quantize_in"], GOLD["quantize_out"]):
        assert oracle.quantize(v) == q
        if v != 0:
            m, _ = math.frexp(q)
            assert float(m * 2 ** 16).is_integer()
