"""GPU parity of the interphase driver's off-step-loop device work against the oracle.

* contact map (stage_interphase/contact_map.cpp:33-85): the device hash map's sorted (i, j, count) table is
  BIT-EXACT against counting the oracle's strict-fp32 neighbour pairs of the same positions at every update;
* sampled positions (simulation_store.cpp:22-33, 192-216): the device quantisation is BIT-EXACT against the
  oracle's fp64 quantize() of the same (fp32) coordinates;
* contact updates between run chunks leave the trajectory bitwise unchanged.
"""
import numpy as np
import pytest

from gcs import _abi as A
from gcs import interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine

import oracle

pytestmark = pytest.mark.gpu

STEPS_PER_UPDATE = 20  # contactmap_update_interval (simulation_config.hpp:76)


def expected_table(snapshots, distance):
    counts = {}
    for x in snapshots:
        for i, j in oracle.search_neighbors(x, distance):
            counts[(int(i), int(j))] = counts.get((int(i), int(j)), 0) + 1
    return np.array([(i, j, c) for (i, j), c in sorted(counts.items())], dtype=np.uint32).reshape(-1, 3)


def engine_for(design, cfg):
    e, _ = interphase.build_interphase(Engine, design, cfg)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    return e


@pytest.mark.parametrize("distance", [0.12, 0.24, 0.5])
def test_contact_map_matches_oracle_c1(c1_design, interphase_cfg, distance):
    e = engine_for(c1_design, interphase_cfg)
    snaps = []
    step = 0
    for _ in range(6):
        e.run(STEPS_PER_UPDATE, first_step=step, seed=7)
        step += STEPS_PER_UPDATE
        e.contacts_update(distance)
        snaps.append(e.get_positions())
    got = e.contacts_accumulate()
    exp = expected_table(snaps, distance)
    assert got.shape == exp.shape and np.array_equal(got, exp)
    assert got[:, 2].max() <= 6 and (got[:, 0] < got[:, 1]).all()
    e.contacts_clear()
    assert e.contacts_accumulate().shape == (0, 3)


def test_contact_map_matches_oracle_c2(interphase_cfg):
    design = synthetic.make_c2()
    e = engine_for(design, interphase_cfg)
    snaps = []
    step = 0
    for _ in range(2):
        e.run(STEPS_PER_UPDATE, first_step=step, seed=3)
        step += STEPS_PER_UPDATE
        e.contacts_update(0.24 * 0.5)
        snaps.append(e.get_positions())
    got = e.contacts_accumulate()
    exp = expected_table(snaps, 0.24 * 0.5)
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


def test_sample_positions_bitexact(c1_design, interphase_cfg):
    e = engine_for(c1_design, interphase_cfg)
    e.run(30, first_step=0, seed=5)
    x = e.get_positions()  # fp64 copies of the fp32 device coordinates
    for bits in (16, 8, 23):
        got = e.sample_positions(bits)
        exp = np.vectorize(lambda v: oracle.quantize(v, bits))(x).astype(np.float32)
        assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), exp.view(np.uint32)), bits


def test_contact_map_engine_cell_list_equals_search_cell_list(c1_design, interphase_cfg):
    """After a rebuild-step run the update reads the engine's own cell list; otherwise (4-launch step) it builds a
    search list: the tables are identical."""
    a = engine_for(c1_design, interphase_cfg)
    a.set_option(A.OPT_FUSED_STEP, 2)
    b = engine_for(c1_design, interphase_cfg)
    b.set_option(A.OPT_FUSED_STEP, 1)
    for k in range(4):
        for e in (a, b):
            e.run(STEPS_PER_UPDATE, first_step=k * STEPS_PER_UPDATE, seed=13)
            e.contacts_update(0.24 * 0.6)
    assert np.array_equal(a.get_positions(), b.get_positions())
    assert np.array_equal(a.contacts_accumulate(), b.contacts_accumulate())


def test_deferred_contact_update_flushes_before_position_changes(c1_design, interphase_cfg):
    """after a list-step run the update is counted inside the next step; a set_positions (or a read) in between
    counts it first, from the positions it was asked for"""
    e = engine_for(c1_design, interphase_cfg)
    e.run(STEPS_PER_UPDATE, first_step=0, seed=3)
    x0 = e.get_positions()
    e.contacts_update(0.24)
    e.set_positions(x0 + 0.05)   # the pending update must see x0, not these
    e.run(STEPS_PER_UPDATE, first_step=STEPS_PER_UPDATE, seed=3)
    x1 = e.get_positions()
    e.contacts_update(0.24)      # pending again: the read flushes it
    got = e.contacts_accumulate()
    assert np.array_equal(got, expected_table([x0, x1], 0.24))
    e.contacts_update(0.24)
    e.contacts_clear()           # a pending update followed by a clear: an empty table
    assert e.contacts_accumulate().shape == (0, 3)
