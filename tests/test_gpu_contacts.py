"""GPU parity of the interphase driver's off-step-loop device work against the oracle.

* contact map (stage_interphase/contact_map.cpp:33-85): the device hash map's sorted (i, j, count) table is
  BIT-EXACT against counting the oracle's strict neighbour pairs (in the engine's precision: fp64 by default, fp32
  for an fp32 engine) of the same positions at every update;
* sampled positions (simulation_store.cpp:22-33, 192-216): the device quantisation is BIT-EXACT against the
  oracle's fp64 quantize() of the same coordinates (the fp64 engine's own, or the fp32 engine's);
* contact updates between run chunks leave the trajectory bitwise unchanged.
"""
import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine
from tolerances import precisions

import oracle

pytestmark = pytest.mark.gpu

STEPS_PER_UPDATE = 20  # contactmap_update_interval (simulation_config.hpp:76)


def expected_table(snapshots, distance, prec=64):
    counts = {}
    for x in snapshots:
        for i, j in oracle.search_neighbors(x, distance, prec):
            counts[(int(i), int(j))] = counts.get((int(i), int(j)), 0) + 1
    return np.array([(i, j, c) for (i, j), c in sorted(counts.items())], dtype=np.uint32).reshape(-1, 3)


def engine_for(design, cfg, prec=64):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    return e


@precisions
@pytest.mark.parametrize("distance", [0.12, 0.24, 0.5])
def test_contact_map_matches_oracle_c1(c1_design, interphase_cfg, distance, prec):
    e = engine_for(c1_design, interphase_cfg, prec)
    snaps = []
    step = 0
    for _ in range(6):
        e.run(STEPS_PER_UPDATE, first_step=step, seed=7)
        step += STEPS_PER_UPDATE
        e.contacts_update(distance)
        snaps.append(e.get_positions())
    got = e.contacts_accumulate()
    exp = expected_table(snaps, distance, prec)
    assert got.shape == exp.shape and np.array_equal(got, exp)
    assert got[:, 2].max() <= 6 and (got[:, 0] < got[:, 1]).all()
    e.contacts_clear()
    assert e.contacts_accumulate().shape == (0, 3)


@precisions
def test_contact_map_matches_oracle_c2(interphase_cfg, prec):
    design = synthetic.make_c2()
    e = engine_for(design, interphase_cfg, prec)
    snaps = []
    step = 0
    for _ in range(2):
        e.run(STEPS_PER_UPDATE, first_step=step, seed=3)
        step += STEPS_PER_UPDATE
        e.contacts_update(0.24 * 0.5)
        snaps.append(e.get_positions())
    got = e.contacts_accumulate()
    exp = expected_table(snaps, 0.24 * 0.5, prec)
    assert got.shape == exp.shape and np.array_equal(got, exp)


def test_contact_updates_leave_the_trajectory_unchanged(c1_design, interphase_cfg):
    a = engine_for(c1_design, interphase_cfg)
    b = engine_for(c1_design, interphase_cfg)
    for k in range(5):
        a.run(STEPS_PER_UPDATE, first_step=k * STEPS_PER_UPDATE, seed=11)
        b.run(STEPS_PER_UPDATE, first_step=k * STEPS_PER_UPDATE, seed=11)
        b.contacts_update(0.24)
    assert np.array_equal(a.get_positions(), b.get_positions())
    assert a.get_context() == b.get_context()


def test_contact_map_overflow_is_reported(c1_design):
    e = Engine(c1_design.n)
    e.set_option(A.OPT_CONTACT_BITS, 10)  # 1,024 slots
    e.set_positions(c1_design.positions)
    e.contacts_update(0.5)  # far more than 1,024 distinct pairs
    with pytest.raises(A.GcsError):
        e.contacts_accumulate()
    e.contacts_clear()
    e.contacts_update(0.01)
    assert e.contacts_accumulate().shape[1] == 3


def test_contact_map_driver_window(c1_design):
    """InterphaseDriver: updates every 20 steps, the table at the window end holds every update's pairs."""
    cfg = InterphaseConfig()
    cfg.logging_interval = 100
    cfg.sampling_interval = 100
    cfg.contactmap_output_window = 1
    e = engine_for(c1_design, cfg)
    drv = interphase.InterphaseDriver(e, c1_design, cfg, log=None)
    drv.run_simulation(steps=100)
    t = drv.last_contacts
    assert t.shape[0] > 0 and (t[:, 0] < t[:, 1]).all()
    # updates at steps 20, 40, 60, 80, 100 (callback(0) has distance 0)
    assert 1 <= t[:, 2].max() <= 5


@precisions
def test_sample_positions_bitexact(c1_design, interphase_cfg, prec):
    e = engine_for(c1_design, interphase_cfg, prec)
    e.run(30, first_step=0, seed=5)
    x = e.get_positions()  # the device coordinates (fp64, or fp64 copies of the fp32 ones)
    for bits in (16, 8, 23):
        got = e.sample_positions(bits)
        exp = np.vectorize(lambda v: oracle.quantize(v, bits))(x).astype(np.float32)
        assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), exp.view(np.uint32)), bits


@pytest.mark.parametrize("fused", [2, 0])
def test_contact_map_engine_cell_list_matches_oracle(c1_design, interphase_cfg, fused):
    """fp32 tile-step shapes: after a rebuild-step run the update reads the engine's own cell list; after the unfused
    step it builds a search list: both tables equal the oracle's counts of the same positions."""
    a = engine_for(c1_design, interphase_cfg, 32)
    a.set_option(A.OPT_FUSED_STEP, fused)
    snaps = []
    for k in range(4):
        a.run(STEPS_PER_UPDATE, first_step=k * STEPS_PER_UPDATE, seed=13)
        snaps.append(a.get_positions())
        a.contacts_update(0.24 * 0.6)
    assert np.array_equal(a.contacts_accumulate(), expected_table(snaps, 0.24 * 0.6, 32))


@precisions
def test_deferred_contact_update_flushes_before_position_changes(c1_design, interphase_cfg, prec):
    """after a list-step run the update is counted inside the next step; a set_positions (or a read) in between
    counts it first, from the positions it was asked for"""
    e = engine_for(c1_design, interphase_cfg, prec)
    e.run(STEPS_PER_UPDATE, first_step=0, seed=3)
    x0 = e.get_positions()
    e.contacts_update(0.24)
    e.set_positions(x0 + 0.05)   # the pending update must see x0, not these
    e.run(STEPS_PER_UPDATE, first_step=STEPS_PER_UPDATE, seed=3)
    x1 = e.get_positions()
    e.contacts_update(0.24)      # pending again: the read flushes it
    got = e.contacts_accumulate()
    assert np.array_equal(got, expected_table([x0, x1], 0.24, prec))
    e.contacts_update(0.24)
    e.contacts_clear()           # a pending update followed by a clear: an empty table
    assert e.contacts_accumulate().shape == (0, 3)


# ---- the production path: the update counted INSIDE the next list step (k_lstep<..., CT>) ------------------------
#
# After a list-step run, contacts_update only records the distance; the next run's first step counts the pairs of
# its start positions from its neighbour lists (partners within the contact distance), or, for particles whose
# lists do not cover that distance (skin outrun, overflowed list, distance beyond cutoff + skin), by a contact-only
# cell search.  InterphaseDriver and the bench take exactly this path (update, then run, no read in between).
# Each snapshot is read BEFORE its update, when nothing is pending, so no read flushes the update through the
# standalone k_contact_insert: every count below comes from the fused step.  Reference: contact_map.cpp:33-85,
# simulation_driver_interphase.cpp:38-45.

def _bench_state():
    from pathlib import Path
    z = np.load(Path(__file__).resolve().parents[1] / "benchdata" / "c2_interphase_step300000.npz")
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    return np.asarray(z["positions"], dtype=np.float32).astype(np.float64), ctx


LATE = {"step": 200000, "time": 2.0, "core_scale": 0.99, "bond_scale": 0.99, "wall_semiaxes": [1.5, 1.55, 1.6]}


def _fused_contacts(design, cfg, ctx, distance, updates, seed, x=None, prec=64, **opts):
    e = engine_for(design, cfg, prec)
    e.set_option(A.OPT_FUSED_STEP, 3)
    e.set_option(A.OPT_DENSE_NEIGHBORS, 0)  # at any density (C1 at core scale 0.99 is dense)
    for k, v in opts.items():
        e.set_option(getattr(A, "OPT_" + k.upper()), v)
    if x is not None:
        e.set_positions(x)
    e.set_context(ctx)
    step = ctx["step"]
    e.run(STEPS_PER_UPDATE, first_step=step, seed=seed)
    step += STEPS_PER_UPDATE
    before = e.run_stats()
    snaps = []
    for _ in range(updates):
        snaps.append(e.get_positions())  # nothing pending: a plain read
        e.contacts_update(distance)      # deferred
        e.run(STEPS_PER_UPDATE, first_step=step, seed=seed)  # counted by this run's first step
        step += STEPS_PER_UPDATE
    after = e.run_stats()
    st = e.list_stats()
    got = e.contacts_accumulate()
    return e, got, snaps, st, {k: after[k] - before[k] for k in before}


def _check_fused(got, snaps, distance, runs, updates, prec=64):
    exp = expected_table(snaps, distance, prec)
    # every update was counted inside a list step (the contact-counting instantiation, replayed from graphs)
    assert runs["fused_contact_steps"] == updates and runs["eager_steps"] == 0, runs
    assert got.shape == exp.shape and np.array_equal(got, exp)
    assert (got[:, 0] < got[:, 1]).all() and got[:, 2].max() <= updates


@precisions
@pytest.mark.parametrize("frac", [0.24, 0.5])
def test_fused_contacts_c1_match_oracle(c1_design, frac, prec):
    """C1, late schedule: 0.24 cs (inside the lists) and 0.5 cs (beyond cutoff + skin: the contact-only search)"""
    cfg = InterphaseConfig()
    d = frac * LATE["core_scale"]
    e, got, snaps, st, runs = _fused_contacts(c1_design, cfg, LATE, d, 5, 31, prec=prec)
    assert st["active"] == 1
    _check_fused(got, snaps, d, runs, 5, prec)


@precisions
@pytest.mark.parametrize("frac", [0.24, 0.5])
def test_fused_contacts_c2_match_oracle(frac, prec):
    """C2 (60,662 particles) from the bench state (step 300,000)"""
    design, cfg = synthetic.make_c2(), InterphaseConfig()
    x, ctx = _bench_state()
    d = frac * ctx["core_scale"]
    e, got, snaps, st, runs = _fused_contacts(design, cfg, ctx, d, 2, 41, x=x, prec=prec, contact_bits=25)
    assert st["active"] == 1
    _check_fused(got, snaps, d, runs, 2, prec)


@precisions
def test_fused_contacts_forced_fallbacks_match_oracle(c1_design, prec):
    """skin 30 per mille with a 200-step rebuild period: particles outrun the skin and are searched exactly, for
    their forces and for their contacts"""
    cfg = InterphaseConfig()
    d = 0.24 * LATE["core_scale"]
    e, got, snaps, st, runs = _fused_contacts(c1_design, cfg, LATE, d, 5, 43, prec=prec, list_skin=30,
                                              list_every=200)
    assert st["fallback_particle_steps"] > 0, st
    _check_fused(got, snaps, d, runs, 5, prec)


@precisions
def test_fused_contacts_overflowed_lists_match_oracle(c1_design, prec):
    """32-entry lists: the overflowed particles' contacts come from the contact-only search"""
    cfg = InterphaseConfig()
    d = 0.24 * LATE["core_scale"]
    e, got, snaps, st, runs = _fused_contacts(c1_design, cfg, LATE, d, 4, 47, prec=prec, list_cap=32)
    assert st["fallback_particle_steps"] > 0, st
    _check_fused(got, snaps, d, runs, 4, prec)


@precisions
def test_fused_contacts_leave_the_trajectory_unchanged(c1_design, prec):
    """the contact-counting step computes the same forces bit for bit: a run with fused updates equals one without"""
    cfg = InterphaseConfig()
    a, _, _, _, _ = _fused_contacts(c1_design, cfg, LATE, 0.5, 3, 53, prec=prec)
    b = engine_for(c1_design, cfg, prec)
    b.set_option(A.OPT_FUSED_STEP, 3)
    b.set_option(A.OPT_DENSE_NEIGHBORS, 0)
    b.set_context(LATE)
    b.run(4 * STEPS_PER_UPDATE, first_step=LATE["step"], seed=53)
    assert np.array_equal(a.get_positions(), b.get_positions())

