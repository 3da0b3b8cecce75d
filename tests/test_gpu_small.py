"""GPU parity of the small-system path (GCS_OPT_SMALL_PATH, kernels.hip k_small: systems of <= 2,048 particles run a
whole chunk of steps in one single-workgroup launch, Verlet lists rebuilt by displacement) against the fp64 oracle,
through the C ABI.  Opt-in (default off: measured slower than the list step's graphs on prometaphase and
telophase); every engine here turns it on.

Bounds as DESIGN.md §6 states for every step shape: positions within 2e-5 absolute after k steps, wall semiaxes
rel 1e-7.  The path changes only the order of the fp32 pair sums (lists in cell-scan order), never the pair set."""
import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, mitotic, synthetic
from gcs.config import InterphaseConfig, MitoticPhaseConfig
from gcs.engine import Engine as _Engine

import oracle

pytestmark = pytest.mark.gpu

TOL_X = 2e-5


class Engine(_Engine):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.set_option(A.OPT_SMALL_PATH, 1)

LATE = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}


def _pair(design, cfg, ctx=None):
    e, _ = interphase.build_interphase(Engine, design, cfg)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        if ctx is not None:
            s.set_context(ctx)
        else:
            s.apply_schedule(0)
    return e, o


def _run(s, steps, first, cfg, seed, **kw):
    s.run(steps, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep, seed=seed, **kw)


def test_small_c1_from_step0(c1_design):
    """production start (core scale 0.5, growing cutoff), 80 steps, Philox noise; one launch"""
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg)
    for s in (e, o):
        _run(s, 80, 0, cfg, 987654321)
    rs = e.run_stats()
    assert rs["small_launches"] == 1 and rs["small_steps"] == 80, rs
    assert e.list_stats()["builds"] >= 1
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X
    ce, co = e.get_context(), o.get_context()
    assert ce["step"] == co["step"] == 80
    assert ce["core_scale"] == pytest.approx(co["core_scale"], rel=1e-12)


def test_small_c1_wall_contact(c1_design):
    cfg = InterphaseConfig()
    e, o = _pair(c1_design, cfg, ctx=LATE)
    for s in (e, o):
        _run(s, 40, LATE["step"], cfg, 5)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X
    ce, co = e.get_context(), o.get_context()
    assert np.allclose(ce["wall_semiaxes"], co["wall_semiaxes"], rtol=1e-7)
    assert np.allclose(ce["inward_reaction"], co["inward_reaction"], rtol=1e-3, atol=1e-2)


def test_small_injected_reference_noise(c1_design):
    cfg = InterphaseConfig()
    steps = 12
    xi = oracle.reference_normals(c1_design.seed, steps * c1_design.n * 3).reshape(steps, c1_design.n, 3)
    e, o = _pair(c1_design, cfg)
    for s in (e, o):
        s.set_noise(xi)
        _run(s, steps, 0, cfg, 0, noise=A.NOISE_INJECTED)
    assert np.abs(e.get_positions() - o.get_positions()).max() <= TOL_X


def test_small_chunks_bitwise_equal_one_run(c1_design):
    """the list state persists across launches: chunks rebuild where one run does, bit for bit; and the list step
    gives the same trajectory within fp32 tolerance"""
    cfg = InterphaseConfig()
    out = []
    for chunks, small in (([90], 1), ([7, 40, 1, 42], 1), ([90], 0)):
        e, _ = interphase.build_interphase(Engine, c1_design, cfg)
        e.set_option(A.OPT_SMALL_PATH, small)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_context(LATE)
        first = LATE["step"]
        for c in chunks:
            _run(e, c, first, cfg, 11)
            first += c
        out.append((e.get_positions(), e.get_context()))
        e.close()
    assert np.array_equal(out[0][0], out[1][0]) and out[0][1] == out[1][1]
    assert np.abs(out[0][0] - out[2][0]).max() <= TOL_X


def test_small_overflowed_lists_match_oracle():
    """300 particles packed into a ball far smaller than the cutoff: every list overflows its 256 entries and every
    particle is evaluated by the scan of the build's cells; same bound against the oracle"""
    rng = np.random.default_rng(5)
    n = 300
    x = rng.normal(scale=0.03, size=(n, 3))
    sysd = {}
    for name, cls in (("e", Engine), ("o", oracle.OracleSystem)):
        s = cls(n, mobilities=np.full(n, 0.1))
        s.add_neighbor_softcore(2.0, 0.3, neighbor_distance=0.3, mix=False)
        s.set_positions(x)
        sysd[name] = s
    for s in sysd.values():
        s.run(10, seed=2, timestep=1e-5)
    assert sysd["e"].list_stats()["fallback_particle_steps"] >= n
    assert np.abs(sysd["e"].get_positions() - sysd["o"].get_positions()).max() <= TOL_X


def _chains_walk(design, seed=3):
    """a start structure for the prometaphase chains: each chain a random walk of bond-length steps"""
    rng = np.random.default_rng(seed)
    x = np.zeros((design.n, 3))
    for _, a, b, _ in design.chains:
        p = rng.uniform(-1.5, 1.5, 3)
        for i in range(a, b):
            x[i] = p
            v = rng.normal(size=3)
            p = p + 0.3 * v / np.linalg.norm(v)
    return x


@pytest.mark.parametrize("stage", ["anaphase", "prometaphase"])
def test_small_mitotic_stage_matches_oracle(stage):
    """C3's mitotic fields (bending, kinetochore fibers, point sources / force-flux, sister bonds) on the small
    path: 200 steps through the stage drivers' force-field composition vs the oracle"""
    cfg = MitoticPhaseConfig()
    d = synthetic.make_c2(1)
    ad = mitotic.anatelophase_design(d, cfg)
    out = {}
    for name, cls in (("e", Engine), ("o", oracle.OracleSystem)):
        if stage == "anaphase":
            s, h = mitotic.build_anatelophase(cls, ad, cfg)
            drv = mitotic.AnatelophaseDriver(s, h, ad, cfg, log=None)
            drv.run_initialization()
            drv.run_dragging_stage(200)
        else:
            pd = mitotic.prometaphase_design(ad, cfg, 1)
            s, _ = mitotic.build_prometaphase(cls, pd, cfg)
            mitotic.PrometaphaseDriver(s, pd, cfg, log=None).run(_chains_walk(pd), 200)
        out[name] = s
    assert out["e"].run_stats()["small_steps"] == 200
    assert np.abs(out["e"].get_positions() - out["o"].get_positions()).max() <= TOL_X
