"""GPU parity: the HIP engine (libgcs.so, through the C ABI) against the fp64 CPU oracle, at both engine
precisions (the fp64 engine -- the reference's arithmetic, the default -- and the fp32 engine).

Tolerances per precision (tests/tolerances.py; fp64 / fp32):
  forces        |dF| <= 1e-10 / 1e-4 * max|F| + 1e-10 / 1e-3 per component
  energies      relative 1e-10 / 1e-5 per kind (absolute 1e-9 / 1e-4 for kinds near zero)
  trajectories  |dx| <= 1e-9 / 2e-5 after <= 50 steps with identical noise (injected or Philox)
  neighbor sets bit-exact (the strict predicate in the engine's precision on both sides)
The fp32-only step shapes (unfused tile step, rebuild step; their tiling options) are tested on fp32 engines.
"""
import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine
from tolerances import E_ABS, E_REL, REACT, REACT_FORCES, WALL_REL, X, assert_forces_close, precisions

import oracle

pytestmark = pytest.mark.gpu


def both(design, cfg, prec=64):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg, precision=prec)
    return e, o


@pytest.fixture(scope="module")
def c2_design():
    return synthetic.make_c2()


@precisions
def test_forces_c1(c1_design, interphase_cfg, prec):
    e, o = both(c1_design, interphase_cfg, prec)
    assert_forces_close(e.compute_forces(), o.compute_forces(), prec)
    ce, co = e.get_context(), o.get_context()
    rt, at = REACT_FORCES[prec]
    assert np.allclose(ce["inward_reaction"], co["inward_reaction"], rtol=rt, atol=at)


@precisions
def test_forces_c1_full_scale(c1_design, interphase_cfg, prec):
    e, o = both(c1_design, interphase_cfg, prec)
    ctx = {"core_scale": 1.0, "bond_scale": 1.0, "wall_semiaxes": [1.25, 1.3, 1.2]}
    e.set_context(ctx)
    o.set_context(ctx)
    assert_forces_close(e.compute_forces(), o.compute_forces(), prec)
    ce, co = e.get_context(), o.get_context()
    rt, at = REACT_FORCES[prec]
    for k in ("inward_reaction", "outward_reaction"):
        assert np.allclose(ce[k], co[k], rtol=rt, atol=10 * at), (k, ce[k], co[k])
    assert max(co["inward_reaction"]) > 0 and max(co["outward_reaction"]) > 0


@precisions
def test_energy_c1(c1_design, interphase_cfg, prec):
    e, o = both(c1_design, interphase_cfg, prec)
    te, pe = e.compute_energy()
    to, po = o.compute_energy()
    assert te == pytest.approx(to, rel=E_REL[prec])
    assert np.allclose(pe, po, rtol=E_REL[prec], atol=E_ABS[prec]), (pe, po)


@precisions
def test_forces_c2(c2_design, interphase_cfg, prec):
    e, o = both(c2_design, interphase_cfg, prec)
    assert_forces_close(e.compute_forces(), o.compute_forces(), prec)
    ctx = {"core_scale": 1.0, "bond_scale": 1.0, "wall_semiaxes": [1.9, 1.9, 1.9]}
    e.set_context(ctx)
    o.set_context(ctx)
    assert_forces_close(e.compute_forces(), o.compute_forces(), prec)
    te, pe = e.compute_energy()
    to, po = o.compute_energy()
    assert te == pytest.approx(to, rel=E_REL[prec])


@precisions
def test_trajectory_injected_reference_noise(c1_design, interphase_cfg, prec):
    """Reference-order normals (std::mt19937_64 + libstdc++ normal_distribution, particle-major x,y,z)
    injected into both: the engine reproduces the reference integrator's noise stream exactly."""
    cfg = interphase_cfg
    e, o = both(c1_design, cfg, prec)
    steps = 20
    xi = oracle.reference_normals(123, steps * c1_design.n * 3).reshape(steps, c1_design.n, 3)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
        s.set_noise(xi)
        s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, noise=A.NOISE_INJECTED)
    xe, xo = e.get_positions(), o.get_positions()
    assert np.abs(xe - xo).max() <= X[prec]
    ce, co = e.get_context(), o.get_context()
    assert ce["step"] == co["step"] == steps
    assert ce["core_scale"] == pytest.approx(co["core_scale"], rel=1e-12)
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=max(WALL_REL[prec], 1e-9))


@precisions
def test_trajectory_philox_c1(c1_design, interphase_cfg, prec):
    cfg = interphase_cfg
    e, o = both(c1_design, cfg, prec)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
        s.run(50, temperature=cfg.temperature, timestep=cfg.timestep, seed=987654321)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= X[prec]


@precisions
def test_trajectory_philox_c1_wall_contact(c1_design, interphase_cfg, prec):
    """Late-schedule window with the wall in contact: reactions drive the wall ODE on both sides."""
    cfg = interphase_cfg
    e, o = both(c1_design, cfg, prec)
    ctx = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}
    for s in (e, o):
        s.set_context(ctx)
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.run(40, first_step=200000, temperature=cfg.temperature, timestep=cfg.timestep, seed=5)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= X[prec]
    ce, co = e.get_context(), o.get_context()
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=WALL_REL[prec])
    rt, at = REACT[prec]
    assert np.allclose(ce["inward_reaction"], co["inward_reaction"], rtol=rt, atol=at)
    assert ce["step"] == 200040


@precisions
@pytest.mark.parametrize("fused", [3, 0], ids=["list", "cells"])
def test_relaxation_spacestep(c1_design, interphase_cfg, prec, fused):
    """spacestep 1e-3 (simulation_driver_relaxation.cpp:48-55), injected reference noise: the relaxation step on the
    lists (default) and on a fresh cell list every step (GCS_OPT_FUSED_STEP 0: fp32 k_force + k_adapt + k_update, fp64
    k_eval64 + k_red64 + k_update)"""
    cfg = interphase_cfg
    e, o = both(c1_design, cfg, prec)
    e.set_option(A.OPT_FUSED_STEP, fused)
    steps = 10
    xi = oracle.reference_normals(7, steps * c1_design.n * 3).reshape(steps, c1_design.n, 3)
    for s in (e, o):
        s.set_noise(xi)
        s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, spacestep=cfg.relaxation_spacestep,
              noise=A.NOISE_INJECTED)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= X[prec]
    assert e.get_context()["last_timestep"] == pytest.approx(o.get_context()["last_timestep"],
                                                             rel={64: 1e-10, 32: 1e-4}[prec])
    builds = e.list_stats()["builds"]
    assert (builds >= 1) if fused == 3 else (builds == 0)  # (the rebuild period depends on the precision's skin)


@precisions
def test_graph_and_eager_bitwise_identical(c1_design, interphase_cfg, prec):
    cfg = interphase_cfg
    runs = []
    for g in (0, 8, 32):
        e, _ = interphase.build_interphase(Engine, c1_design, cfg, precision=prec)
        e.set_option(A.OPT_GRAPH_STEPS, g)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.apply_schedule(0)
        e.run(70, seed=11)
        runs.append((e.get_positions(), e.get_context()))
    for x, c in runs[1:]:
        assert np.array_equal(x, runs[0][0])
        assert c == runs[0][1]


@pytest.mark.parametrize("waves", [1, 2, 4, 8])
@pytest.mark.parametrize("order", [0, 1])
def test_waves_per_tile_equivalent(c1_design, interphase_cfg, waves, order):
    """the fp32 tile kernel's wave / chunk options (the fp32 engine's force and energy evaluations)"""
    e, o = both(c1_design, interphase_cfg, 32)
    e.set_option(A.OPT_WAVES_PER_TILE, waves)
    e.set_option(A.OPT_CHUNK_ORDER, order)
    assert_forces_close(e.compute_forces(), o.compute_forces(), 32)
    te, pe = e.compute_energy()
    to, po = o.compute_energy()
    assert te == pytest.approx(to, rel=1e-5)


@pytest.mark.parametrize("fused", [0, 2])
@pytest.mark.parametrize("mode", [1, 2])
def test_split_tiles_agree(c2_design, interphase_cfg, fused, mode):
    """Splitting tiles' candidates over two workgroups (mode 1: every tile; mode 2: the heavy tiles the cell scan
    picks) only regroups the fp32 pair sums: the C2 trajectory stays within fp32 tolerance of the unsplit one,
    and the split run is bitwise reproducible."""
    out = []
    for split in (0, mode, mode):
        e, _ = interphase.build_interphase(Engine, c2_design, interphase_cfg, precision=32)
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_option(A.OPT_SPLIT_TILES, split)
        e.set_schedule(**interphase.interphase_schedule(interphase_cfg))
        e.apply_schedule(0)
        e.run(20, seed=11)
        out.append(e.get_positions())
        e.close()
    assert np.abs(out[0] - out[1]).max() <= 2e-5
    assert np.array_equal(out[1], out[2])


@pytest.mark.parametrize("prec,fused", [(32, 0), (32, 2), (64, 3)])
def test_scan_blocks_agree(c2_design, interphase_cfg, prec, fused):
    """The multi-block look-back cell scan builds the same cstart / tile tables as the one-workgroup scan, so
    the C2 trajectories are bitwise equal (the tile step, the rebuild step's first cell list, the list builds)."""
    out = []
    for mb in (0, 1):
        e, _ = interphase.build_interphase(Engine, c2_design, interphase_cfg, precision=prec)
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_option(A.OPT_SCAN_BLOCKS, mb)
        e.set_schedule(**interphase.interphase_schedule(interphase_cfg))
        e.apply_schedule(0)
        e.run(30, seed=5)
        out.append(e.get_positions())
        e.close()
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("squeeze", [1.0, 0.08])
def test_step_shapes_bitwise_equal(c2_design, interphase_cfg, squeeze):
    """The fp32 2-launch rebuild step (cell list rebuilt from the force kernel's per-cell buckets) is bitwise
    reproducible and, across a run split in two, equal to itself; the unfused step bins with its own grid (fp32 sums
    in another order): within tolerance.  squeeze < 1 packs the beads into a small ball: cells far over the bucket
    capacity (overflow list) and blocks over the LDS staging capacity (global staging path)."""
    x0 = c2_design.positions
    x0 = x0.mean(0) + squeeze * (x0 - x0.mean(0))
    out = []
    for fused in (0, 2, 2):
        e, _ = interphase.build_interphase(Engine, c2_design, interphase_cfg, precision=32)
        e.set_positions(x0)
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_schedule(**interphase.interphase_schedule(interphase_cfg))
        e.apply_schedule(0)
        e.run(12, seed=9)
        e.run(8, first_step=12, seed=9)
        out.append(e.get_positions())
        e.close()
    assert np.all(np.isfinite(out[2]))
    assert np.array_equal(out[1], out[2])
    if squeeze == 1.0:
        assert np.abs(out[0] - out[1]).max() <= 2e-5


@pytest.mark.parametrize("mb", [0, 1])
@pytest.mark.parametrize("shape", ["x_line", "z_line", "slab"])
@precisions
def test_neighbor_search_grid_shapes(mb, shape, prec):
    """Degenerate grids for the cell scan: rows wider than one scan block (nx > 2048, chunked), one-cell rows
    (nx = 1, 2048 rows per block) and a thin slab; pair sets bit-exact vs the oracle for both scan kinds."""
    rng = np.random.default_rng(7)
    d = 0.25
    if shape == "x_line":
        pts = np.stack([rng.uniform(0, 3000 * d, 3000), rng.uniform(0, 0.1, 3000), rng.uniform(0, 0.1, 3000)], 1)
    elif shape == "z_line":
        pts = np.stack([rng.uniform(0, 0.1, 3000), rng.uniform(0, 0.1, 3000), rng.uniform(0, 2500 * d, 3000)], 1)
    else:
        pts = np.stack([rng.uniform(0, 60, 5000), rng.uniform(0, 60, 5000), rng.uniform(0, 0.3, 5000)], 1)
    e = Engine(4, precision=prec)
    e.set_option(A.OPT_SCAN_BLOCKS, mb)
    got = e.search_neighbors(d, points=pts)
    exp = oracle.search_neighbors(pts, d, prec)
    assert got.shape == exp.shape and np.array_equal(got, exp)


@pytest.mark.parametrize("prec,fused", [(32, 0), (32, 2), (32, 3), (64, 3)])
def test_chunked_runs_equal_one_run(c1_design, interphase_cfg, prec, fused):
    """The Philox counter is the absolute step: 3 chunks == 1 run, bit for bit (every step shape; the fused
    steps carry their cell list / lists across runs that continue at the next step)."""
    cfg = interphase_cfg
    a, _ = interphase.build_interphase(Engine, c1_design, cfg, precision=prec)
    b, _ = interphase.build_interphase(Engine, c1_design, cfg, precision=prec)
    for s in (a, b):
        s.set_option(A.OPT_FUSED_STEP, fused)
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
    a.run(60, seed=3)
    b.run(25, first_step=0, seed=3)
    b.run(20, first_step=25, seed=3)
    b.run(15, first_step=45, seed=3)
    assert np.array_equal(a.get_positions(), b.get_positions())


@precisions
def test_neighbor_search_near_cutoff_far_from_origin(prec):
    """Pairs just inside the cutoff (d (1 - 1e-6) along a coordinate axis) in a box 1,000 away from the origin,
    where the fp32 roundings the binning works on (~6e-5) exceed 1e-4 of the cell edge (d = 0.1): without a margin
    that scales with the coordinates some such pairs bin two cells apart and are lost (kernels.hip make_grid; ADVICE
    r4).  The pair set is bit-exact vs the oracle predicate"""
    rng = np.random.default_rng(13)
    d = 0.1
    m = 20000
    a = 1000.0 + rng.uniform(0, 3.0, size=(m, 3))
    u = np.zeros((m, 3))
    u[np.arange(m), rng.integers(0, 3, m)] = rng.choice([-1.0, 1.0], m)
    pts = np.concatenate([a, a + u * d * (1 - 1e-6)])
    e = Engine(4, precision=prec)
    got = e.search_neighbors(d, points=pts)
    exp = oracle.search_neighbors(pts, d, prec)
    assert exp.shape[0] >= m // 2  # (most placed pairs are within d in the engine's precision)
    assert got.shape == exp.shape and np.array_equal(got, exp)


@precisions
def test_neighbor_search_bitexact_c1(c1_design, prec):
    e = Engine(c1_design.n, precision=prec)
    e.set_positions(c1_design.positions)
    for d in (0.12, 0.24, 0.3, 0.5):
        assert np.array_equal(e.search_neighbors(d), oracle.search_neighbors(c1_design.positions, d, prec))


@precisions
def test_neighbor_search_bitexact_c2(c2_design, prec):
    e = Engine(16, precision=prec)
    for d in (0.12, 0.24):
        got = e.search_neighbors(d, points=c2_design.positions)
        exp = oracle.search_neighbors(c2_design.positions, d, prec)
        assert got.shape == exp.shape and np.array_equal(got, exp)


@precisions
def test_neighbor_search_edge_cases(prec):
    e = Engine(4, precision=prec)
    pts = np.array([[0, 0, 0], [0, 0, 0], [0.25, 0, 0], [0.5, 0, 0], [5.0, 0, 0]], dtype=float)
    assert e.search_neighbors(0.25, points=pts).tolist() == oracle.search_neighbors(pts, 0.25, prec).tolist()
    assert (e.search_neighbors(0.2500001, points=pts).tolist()
            == oracle.search_neighbors(pts, 0.2500001, prec).tolist())
    # ties at the cutoff in fp64 that round together in fp32: 0.25 + 1 ulp (fp64) is a pair only for fp64 at 0.25+
    tie = np.array([[0.0, 0.0, 0.0], [np.nextafter(0.25, 1.0), 0.0, 0.0]])
    assert (e.search_neighbors(np.nextafter(np.nextafter(0.25, 1.0), 1.0), points=tie).tolist()
            == oracle.search_neighbors(tie, np.nextafter(np.nextafter(0.25, 1.0), 1.0), prec).tolist())
    assert e.search_neighbors(0.3, points=np.zeros((1, 3))).shape == (0, 2)
    # all points coincident (degenerate bounding box)
    same = np.zeros((70, 3))
    got = e.search_neighbors(0.1, points=same)
    assert got.shape == (70 * 69 // 2, 2)
    assert np.array_equal(got, oracle.search_neighbors(same, 0.1, prec))


@precisions
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 200])
def test_small_and_ragged_sizes(n, prec):
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
        sysd[name] = s
    assert_forces_close(sysd["e"].compute_forces(), sysd["o"].compute_forces(), prec)
    for s in sysd.values():
        s.run(5, seed=1, timestep=1e-4)
    assert np.abs(sysd["e"].get_positions() - sysd["o"].get_positions()).max() <= X[prec]


@precisions
def test_particles_far_outside_and_coincident(prec):
    n = 130
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, size=(n, 3))
    x[:10] = 0.0          # coincident
    x[10:15] += 50.0      # far away cluster
    x[15] = [-80, 3, 3]   # isolated
    res = []
    for cls in (Engine, oracle.OracleSystem):
        s = cls(n, ab_factors=np.tile([1.0, 0.0], (n, 1)), precision=prec)
        s.add_neighbor_softcore(2.0, 0.3, neighbor_distance=0.3, mix=False)
        s.set_positions(x)
        res.append(s.compute_forces())
    assert_forces_close(res[0], res[1], prec)


@precisions
def test_mitotic_fields_parity(prec):
    rng = np.random.default_rng(7)
    n = 120
    x = np.cumsum(rng.normal(scale=0.15, size=(n, 3)), axis=0)
    mu = np.full(n, 0.1)
    out = []
    for cls in (Engine, oracle.OracleSystem):
        s = cls(n, mobilities=mu, precision=prec)
        s.add_neighbor_softcore(a_energy=2.0, a_diameter=0.3, neighbor_distance=0.3, mix=False)
        s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=1000.0, a_length=0.3, ranges=[(0, 60), (60, 120)])
        s.add_bonded_triplewise(1.0, ranges=[(0, 20), (21, 60), (60, 80), (81, 120)])
        s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=1000.0, a_length=0.3, pairs=[(20, 80)])
        s.add_kinetochore_fiber([0.0, -5.0, 0.0], [(20, 0.1 / 60, 1.0, 0.0)])
        s.add_kinetochore_fiber([0.0, 5.0, 0.0], [(80, 0.1 / 60, 1.0, 0.2)])
        s.add_point_source(A.POT_FORCE_FLUX, [0.0, -5.0, 0.0], force=0.5, reactive_distance=0.3)
        s.add_point_source(A.POT_FORCE_FLUX, [0.0, 5.0, 0.0], force=0.5, reactive_distance=0.3)
        s.add_point_source(A.POT_SEMISPRING, [0.0, 0.0, 0.0], spring=100.0, length=1.5)
        s.set_positions(x)
        f = s.compute_forces()
        en = s.compute_energy()
        xi = oracle.reference_normals(99, 10 * n * 3).reshape(10, n, 3)
        s.set_noise(xi)
        s.run(10, timestep=1e-4, noise=A.NOISE_INJECTED)
        out.append((f, en, s.get_positions()))
    assert_forces_close(out[0][0], out[1][0], prec)
    assert out[0][1][0] == pytest.approx(out[1][1][0], rel=E_REL[prec])
    assert np.allclose(out[0][1][1], out[1][1][1], rtol=E_REL[prec], atol=E_ABS[prec])
    assert np.abs(out[0][2] - out[1][2]).max() <= X[prec]


@precisions
def test_remove_forcefield_swaps_like_anatelophase(prec):
    """stage_anatelophase/simulation_driver.cpp:277-285: remove the anaphase bonds/bending, add telophase ones"""
    n = 90
    rng = np.random.default_rng(3)
    x = np.cumsum(rng.normal(scale=0.2, size=(n, 3)), axis=0)
    res = []
    for cls in (Engine, oracle.OracleSystem):
        s = cls(n, mobilities=np.full(n, 0.1), precision=prec)
        s.add_neighbor_softcore(2.0, 0.3, neighbor_distance=0.3, mix=False)
        hb = s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=1000.0, a_length=0.3, ranges=[(0, 90)])
        hk = s.add_bonded_triplewise(1.0, ranges=[(0, 90)])
        s.set_positions(x)
        s.run(5, timestep=1e-4, seed=4)
        s.remove_forcefield(hb)
        s.remove_forcefield(hk)
        s.add_bonded_pairwise(A.POT_SEMISPRING, a_spring=500.0, a_length=0.3, ranges=[(0, 90)])
        s.add_bonded_triplewise(3.0, ranges=[(0, 90)])
        s.add_point_source(A.POT_SEMISPRING, [0, 0, 0], spring=100.0, length=1.5)
        s.run(5, first_step=5, timestep=1e-4, seed=4)
        res.append((s.get_positions(), s.compute_forces()))
    assert np.abs(res[0][0] - res[1][0]).max() <= X[prec]
    assert_forces_close(res[0][1], res[1][1], prec)


def test_c2_window_properties(c2_design, interphase_cfg):
    """Full C2 size: a production window stays finite, the schedule advances and the step is deterministic."""
    cfg = interphase_cfg
    e1, _ = interphase.build_interphase(Engine, c2_design, cfg)
    e2, _ = interphase.build_interphase(Engine, c2_design, cfg)
    for s in (e1, e2):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
        s.run(64, seed=17)
    x1, x2 = e1.get_positions(), e2.get_positions()
    assert np.isfinite(x1).all()
    assert np.array_equal(x1, x2)
    c = e1.get_context()
    assert c["step"] == 64 and c["time"] == pytest.approx(64 * cfg.timestep)
    disp = np.linalg.norm(x1 - c2_design.positions, axis=1)
    assert disp.mean() < 0.2


def test_fused_and_unfused_steps_agree(c1_design, interphase_cfg):
    """The fp32 rebuild step (binning into the next grid inside the force kernel, the cell list rebuilt from its
    buckets) and the 6-launch step give the same trajectory within fp32 tolerance (their cell grids, hence summation
    orders, differ)."""
    cfg = interphase_cfg
    out = []
    for fused in (0, 2):
        e, _ = interphase.build_interphase(Engine, c1_design, cfg, precision=32)
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.apply_schedule(0)
        e.run(50, seed=21)
        out.append((e.get_positions(), e.get_context()))
    assert np.abs(out[0][0] - out[1][0]).max() <= 2e-5
    assert out[0][1]["step"] == out[1][1]["step"] == 50
    assert np.allclose(out[0][1]["wall_semiaxes"], out[1][1]["wall_semiaxes"], rtol=1e-9)


@precisions
def test_fused_c2_matches_oracle_forces_after_run(c2_design, interphase_cfg, prec):
    """After a fused run the engine's cell list must still describe its positions: forces at the final state
    match the oracle's on the same positions/context."""
    cfg = interphase_cfg
    e, _ = interphase.build_interphase(Engine, c2_design, cfg, precision=prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.set_context({"step": 300000, "time": 3.0, "core_scale": 0.9988, "bond_scale": 0.9988,
                   "wall_semiaxes": [2.0, 2.0, 2.0]})
    e.run(96, first_step=300000, seed=8)
    o, _ = interphase.build_interphase(oracle.OracleSystem, c2_design, cfg)
    o.set_positions(e.get_positions())
    ctx = e.get_context()
    o.set_context(ctx)
    assert_forces_close(e.compute_forces(), o.compute_forces(), prec)


# ---- C3: the mitotic stages through the drivers (gcs.mitotic), engine vs oracle, Philox noise -------------------

def _c3():
    from gcs import mitotic
    from gcs.config import MitoticPhaseConfig
    cfg = MitoticPhaseConfig()
    i = synthetic.make_c2()
    a = mitotic.anatelophase_design(i, cfg)
    p = mitotic.prometaphase_design(a, cfg, i.master_seed)
    return mitotic, cfg, a, p


@precisions
def test_c3_anatelophase_stages_match_oracle(prec):
    """586 beads: rods init (same mt19937_64 draws), 40 anaphase steps with kinetochore fibers, field swap,
    40 telophase steps with the packing well; positions and energies within the precision's bounds."""
    mitotic, cfg, a, _ = _c3()
    res = []
    for cls in (Engine, oracle.OracleSystem):
        s, h = mitotic.build_anatelophase(cls, a, cfg, precision=prec)
        drv = mitotic.AnatelophaseDriver(s, h, a, cfg, log=None)
        drv.run(anaphase_steps=40, telophase_steps=40)
        res.append((s.get_positions(), s.compute_energy()[0], s.compute_forces()))
    assert np.abs(res[0][0] - res[1][0]).max() <= X[prec]
    assert res[0][1] == pytest.approx(res[1][1], rel=E_REL[prec])
    assert_forces_close(res[0][2], res[1][2], prec)


@precisions
def test_c3_prometaphase_matches_oracle(prec):
    """1,172 beads: sister bonds, fibers to both poles, force-flux point sources (polar ejection switched on)."""
    import dataclasses
    mitotic, cfg, a, p = _c3()
    cfg = dataclasses.replace(cfg, polar_ejection_force=0.5, polar_ejection_cross_section=0.09,
                              kfiber_length_prometaphase=1.0)
    # a structure like the one transition writes: each sister pair side by side around the metaphase plate
    rng = np.random.default_rng(11)
    x0 = np.zeros((p.n, 3))
    for (_, ts, te, _), (_, ss, se, _) in zip(p.chains[0::2], p.chains[1::2]):
        c = rng.normal(scale=1.0, size=3)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        for k in range(te - ts):
            x0[ts + k] = c + (k - (te - ts) / 2) * cfg.bond_length * d
            x0[ss + k] = x0[ts + k] + [0.0, cfg.sister_separation, 0.0]
    res = []
    for cls in (Engine, oracle.OracleSystem):
        s, _ = mitotic.build_prometaphase(cls, p, cfg, precision=prec)
        mitotic.PrometaphaseDriver(s, p, cfg, log=None).run(x0, steps=50)
        res.append((s.get_positions(), s.compute_forces()))
    assert np.abs(res[0][0] - res[1][0]).max() <= X[prec]
    assert_forces_close(res[0][1], res[1][1], prec)
