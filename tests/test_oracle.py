"""CPU tests of the oracle (test infrastructure) against golden vectors and closed forms.

Golden vectors: tests/golden/rng_fixtures.json (libstdc++ outputs, tests/golden/make_fixtures.sh) and the
Random123 Philox4x32-10 known-answer vectors.  Potential/force-field forms are micromd restatements
("parity unpinned"): they are checked for internal consistency (F = -grad U by central differences,
Newton's third law) and against closed forms computed here.
"""
import json
import math
from pathlib import Path

import numpy as np
import pytest

import oracle

GOLDEN = Path(__file__).resolve().parent / "golden" / "rng_fixtures.json"


@pytest.fixture(scope="module")
def fx():
    return json.loads(GOLDEN.read_text())


# ---- random numbers ----------------------------------------------------------------------------------

def test_philox_random123_kat():
    # Random123 kat_vectors, philox4x32 10 rounds
    assert oracle.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                          0x6D5451FD]
    assert oracle.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_seed_seq_matches_libstdcxx(fx):
    for rec in fx["seed_seq"]:
        assert oracle.seed_seq_generate([rec["master"]], 3) == rec["stage_seeds"]
    lng = fx["seed_seq_long"]
    assert oracle.seed_seq_generate(lng["seeds"], len(lng["out"])) == lng["out"]


def test_reference_normals_match_libstdcxx(fx):
    for rec in fx["normal_distribution"]:
        got = oracle.reference_normals(rec["seed"], len(rec["values"]))
        assert np.array_equal(got, np.array(rec["values"])), (got, rec["values"])


def test_philox_normals_statistics():
    z = oracle.philox_normals(12345, 7, 200_000).ravel()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    # different steps / seeds give different streams; the same arguments the same stream
    assert not np.array_equal(oracle.philox_normals(1, 1, 10), oracle.philox_normals(1, 2, 10))
    assert np.array_equal(oracle.philox_normals(1, 1, 10), oracle.philox_normals(1, 1, 10))


def test_quantize():
    # simulation_store.cpp:22-33: 16 fraction bits of the frexp mantissa
    assert oracle.quantize(1.0) == 1.0
    assert oracle.quantize(0.0) == 0.0
    v = 1.0 / 3.0
    assert oracle.quantize(v) == round(2 ** 16 * (2.0 / 3.0)) * 2.0 ** -17
    for x in np.random.default_rng(0).normal(size=100) * 3:
        q = oracle.quantize(x)
        m, e = math.frexp(q)
        assert float(m * 2 ** 16).is_integer()
        assert abs(q - x) <= abs(x) * 2.0 ** -16


# ---- force fields ------------------------------------------------------------------------------------

def _fd_check(sys_, x0, idx, h=1e-6, rtol=2e-5, atol=2e-4):
    sys_.set_positions(x0)
    F = sys_.compute_forces()
    for i in idx:
        for k in range(3):
            xp = x0.copy()
            xp[i, k] += h
            sys_.set_positions(xp)
            ep, _ = sys_.compute_energy()
            xm = x0.copy()
            xm[i, k] -= h
            sys_.set_positions(xm)
            em, _ = sys_.compute_energy()
            fd = -(ep - em) / (2 * h)
            assert abs(fd - F[i, k]) <= atol + rtol * abs(F[i, k]), (i, k, fd, F[i, k])
    sys_.set_positions(x0)
    return F


def test_interphase_forces_are_minus_grad_energy(c1_design, interphase_cfg):
    from gcs import interphase
    s, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, interphase_cfg)
    F = _fd_check(s, c1_design.positions.copy(), [0, 1, 99, 500, 999, 1000, 1001])
    # everything but the walls is internal: the net force vanishes (Newton's third law)
    assert np.abs(F.sum(axis=0)).max() < 1e-8 * np.abs(F).sum()


def test_wall_forces_and_reaction():
    """Sphere wall (semiaxes equal): the Sampson distance is exact, so the closed form applies."""
    rng = np.random.default_rng(3)
    n = 400
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    radii = rng.uniform(1.85, 2.1, size=n)
    x = dirs * radii[:, None]
    ab = np.tile([0.5, 0.5], (n, 1))
    s = oracle.OracleSystem(n, ab_factors=ab)
    s.add_ellipsoid_inward(a_energy=2.5, a_diameter=0.15, b_energy=2.5, b_diameter=0.12, wall_a=0.0, wall_b=10.0,
                           mix=True, scaled=False)
    s.add_ellipsoid_outward(spring=1000.0)
    s.set_context({"wall_semiaxes": [2.0, 2.0, 2.0]})
    F = _fd_check(s, x, list(range(0, n, 37)))
    # closed form of the outward harmonic wall: F = -K (r - R) r_hat
    out = radii > 2.0
    exp = -1000.0 * (radii[out] - 2.0)[:, None] * dirs[out]
    inside_contact = (radii < 2.0) & (radii > 2.0 - 0.15)
    assert np.allclose(F[out], exp, rtol=1e-10, atol=1e-10)
    c = s.get_context()
    # reaction = per-axis sum of |force on the particles from each wall|
    assert np.allclose(c["outward_reaction"], np.abs(exp).sum(axis=0))
    assert np.all(np.array(c["inward_reaction"]) > 0) and inside_contact.any()


def test_mitotic_fields_consistent():
    """bending, kinetochore fiber, point sources (semispring, force flux), plain softcore<2,3>"""
    rng = np.random.default_rng(7)
    n = 60
    x = np.cumsum(rng.normal(scale=0.2, size=(n, 3)), axis=0)
    s = oracle.OracleSystem(n, mobilities=np.full(n, 0.1))
    s.add_neighbor_softcore(a_energy=2.0, a_diameter=0.3, neighbor_distance=0.3, mix=False, scaled=False)
    s.add_bonded_pairwise(0, a_spring=1000.0, a_length=0.3, ranges=[(0, 30), (30, 60)])
    s.add_bonded_triplewise(1.0, ranges=[(0, 12), (13, 30), (30, 60)])
    s.add_kinetochore_fiber([0.0, 5.0, 0.0], [(12, 0.1 / 30, 1.0, 0.5), (42, 0.1 / 30, 1.0, 0.0)])
    s.add_point_source(0, [0.0, 0.0, 0.0], spring=100.0, length=1.5)
    s.add_point_source(3, [0.0, -5.0, 0.0], force=0.7, reactive_distance=0.4)
    s.add_bonded_pairwise(0, a_spring=1000.0, a_length=0.3, pairs=[(12, 42)])
    _fd_check(s, x, [0, 5, 12, 13, 29, 30, 42, 59])


def test_force_flux_closed_form():
    """common/potentials/force_flux_potential.hpp:24-37 (in-repo): U = b f atan2(b, r),
    F = f b^2 / (b^2 r + r^3) r_vec."""
    s = oracle.OracleSystem(1)
    s.add_point_source(3, [0.0, 0.0, 0.0], force=0.7, reactive_distance=0.4)
    for r in (0.05, 0.4, 1.0, 3.0):
        s.set_positions([[r, 0.0, 0.0]])
        e, _ = s.compute_energy()
        assert e == pytest.approx(0.4 * 0.7 * math.atan2(0.4, r), rel=1e-12)
        f = s.compute_forces()[0]
        assert f[0] == pytest.approx(0.7 * 0.16 / (0.16 * r + r ** 3) * r, rel=1e-12)


@pytest.mark.parametrize("r", [0.0, 0.05, 0.1, 0.149, 0.2, 0.239, 0.25, 0.299, 0.31])
def test_softcore_closed_form(r):
    """U = a SC<2,3> + b SC<8,3> with SC<p,q> = eps (1 - (r/s)^p)^q (r < s); pair means of the ab factors."""
    s = oracle.OracleSystem(2, ab_factors=[[1.0, 0.0], [0.5, 0.5]])
    s.add_neighbor_softcore(a_energy=2.5, a_diameter=0.3, b_energy=2.5, b_diameter=0.24, neighbor_distance=0.3,
                            mix=True, scaled=False)
    s.set_positions([[0, 0, 0], [r, 0, 0]])
    e, _ = s.compute_energy()
    a, b = 0.75, 0.25
    exp = 0.0
    if r < 0.3:
        exp += a * 2.5 * (1 - (r / 0.3) ** 2) ** 3
    if r < 0.24:
        exp += b * 2.5 * (1 - (r / 0.24) ** 8) ** 3
    assert e == pytest.approx(exp, rel=1e-12, abs=1e-14)


def test_softwell_cutoff_and_form():
    s = oracle.OracleSystem(3, ab_factors=[[0, 10]] * 3)
    s.add_neighbor_softwell(energy=0.3, decay_distance=0.2, cutoff=0.4, targets=[0, 2])
    s.set_positions([[0, 0, 0], [0.1, 0, 0], [0.3, 0, 0]])
    e, _ = s.compute_energy()
    assert e == pytest.approx(-0.3 / (1 + (0.3 / 0.2) ** 6))
    s.set_positions([[0, 0, 0], [0.1, 0, 0], [0.41, 0, 0]])
    assert s.compute_energy()[0] == 0.0


def test_schedule_closed_form():
    s = oracle.OracleSystem(1)
    s.set_context({"wall_semiaxes": [2.0, 2.1, 2.2], "core_scale": 0.5, "bond_scale": 0.5})
    s.set_schedule(update_time=1, update_scales=1, update_wall=1, timestep=1e-5, core_scale_init=0.5,
                   core_scale_tau=0.5, bond_scale_init=0.4, bond_scale_tau=0.25,
                   wall_semiaxes_spring=[3e4, 3e4, 3e4], wall_mobility=2e-4)
    s.apply_schedule(1000)
    c = s.get_context()
    t = 1000 * 1e-5
    assert c["time"] == pytest.approx(t)
    assert c["core_scale"] == pytest.approx(1 - 0.5 * math.exp(-t / 0.5))
    assert c["bond_scale"] == pytest.approx(1 - 0.6 * math.exp(-t / 0.25))
    for k, a in enumerate([2.0, 2.1, 2.2]):
        assert c["wall_semiaxes"][k] == pytest.approx(a + 1e-5 * 2e-4 * (0 - 3e4 * a))


def test_bd_step_closed_form():
    """One Euler-Maruyama step with injected noise: x' = x + mu dt F + sqrt(2 T mu dt) xi."""
    rng = np.random.default_rng(11)
    n = 5
    x = rng.normal(size=(n, 3))
    mu = rng.uniform(0.5, 2.0, size=n)
    s = oracle.OracleSystem(n, mobilities=mu)
    s.add_point_source(1, [0.0, 0.0, 0.0], spring=3.0)
    s.set_positions(x)
    xi = rng.normal(size=(1, n, 3))
    s.set_noise(xi)
    s.run(1, temperature=0.7, timestep=1e-3, noise=1)
    exp = x + mu[:, None] * 1e-3 * (-3.0 * x) + np.sqrt(2 * 0.7 * mu[:, None] * 1e-3) * xi[0]
    assert np.allclose(s.get_positions(), exp, rtol=1e-13, atol=1e-14)


def test_spacestep_limits_drift():
    n = 4
    s = oracle.OracleSystem(n)
    s.add_point_source(1, [0.0, 0.0, 0.0], spring=1e4)
    x = np.array([[1.0, 0, 0], [0, 0.5, 0], [0, 0, 0.1], [0.2, 0.2, 0.2]])
    s.set_positions(x)
    s.run(1, timestep=1e-3, spacestep=1e-3, noise=2)
    moved = np.linalg.norm(s.get_positions() - x, axis=1)
    assert moved.max() == pytest.approx(1e-3, rel=1e-12)
    assert s.get_context()["last_timestep"] == pytest.approx(1e-3 / 1e4, rel=1e-12)


# ---- neighbor search ---------------------------------------------------------------------------------

def _brute_pairs(x, d):
    p = x.astype(np.float32)
    out = []
    rc2 = np.float32(d) * np.float32(d)
    for i in range(len(p)):
        diff = (p[i] - p[i + 1:]).astype(np.float32)
        sq = (diff * diff).astype(np.float32)
        r2 = ((sq[:, 0] + sq[:, 1]).astype(np.float32) + sq[:, 2]).astype(np.float32)
        for j in np.nonzero(r2 < rc2)[0]:
            out.append((i, i + 1 + j))
    return np.array(out, dtype=np.uint32).reshape(-1, 2)


def test_neighbor_search_matches_brute_force(c1_design):
    x = c1_design.positions
    for d in (0.12, 0.24, 0.3):
        got = oracle.search_neighbors(x, d)
        exp = _brute_pairs(x, d)
        assert np.array_equal(got, exp)


def test_neighbor_search_edge_cases():
    assert oracle.search_neighbors(np.zeros((0, 3)), 0.3).shape == (0, 2)
    assert oracle.search_neighbors(np.zeros((1, 3)), 0.3).shape == (0, 2)
    # coincident points, points exactly at the cutoff, degenerate (planar) extents
    x = np.array([[0, 0, 0], [0, 0, 0], [0.25, 0, 0], [0.5, 0, 0], [5.0, 0, 0]])
    got = oracle.search_neighbors(x, 0.25)
    assert got.tolist() == [[0, 1]]  # 0.25 apart is not "closer than 0.25"
    assert np.array_equal(got, _brute_pairs(x, 0.25))
    assert oracle.search_neighbors(x, 0.2500001).tolist() == [[0, 1], [0, 2], [1, 2], [2, 3]]


def test_driver_contact_schedule_on_the_oracle(c1_design):
    """InterphaseDriver's contact-map cadence (simulation_driver_interphase.cpp:38-45, 68-76) on the oracle backend:
    updates every 20 steps with 0.24 x core_scale of the previous step, none at callback(0), output + clear at
    the window end."""
    from gcs import interphase
    from gcs.config import InterphaseConfig
    cfg = InterphaseConfig()
    cfg.logging_interval = 40
    cfg.sampling_interval = 40
    cfg.contactmap_output_window = 1
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg)
    drv = interphase.InterphaseDriver(o, c1_design, cfg, log=None)
    assert drv.contact_distance(0) == 0.0
    assert drv.contact_distance(1) == pytest.approx(0.24 * cfg.core_scale_init)
    t21 = 20 * cfg.timestep
    assert drv.contact_distance(21) == pytest.approx(
        0.24 * (1 - (1 - cfg.core_scale_init) * np.exp(-t21 / cfg.core_scale_tau)))
    drv.run_simulation(steps=40)
    t = drv.last_contacts
    assert t.dtype == np.uint32 and t.shape[1] == 3 and t.shape[0] > 0
    assert (t[:, 0] < t[:, 1]).all() and 1 <= t[:, 2].max() <= 2  # updates at steps 20 and 40
    keys = t[:, 0].astype(np.uint64) << np.uint64(32) | t[:, 1].astype(np.uint64)
    assert (np.diff(keys.astype(np.int64)) > 0).all()
