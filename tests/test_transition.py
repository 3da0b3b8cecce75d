"""Stage transitions (gcs/transition.py; stage_transition/*.cpp) on the CPU, through the HDF5 store."""
import numpy as np
import pytest

from gcs import mitotic, store, synthetic, transition
from gcs.config import SimulationConfig


def test_resample_reproduces_cubic_data():
    """the not-a-knot spline is exact on cubic data: resampling at the knots' own parameters is the identity, and a
    cubic curve is reproduced at any sample count"""
    n = 9
    t = (0.5 + np.arange(n)) / n
    curve = lambda u: np.stack([u, u ** 2 - u, 2 * u ** 3 + 0.5], axis=1)
    x = curve(t)
    assert np.allclose(transition.resample_chain(x, n), x, atol=1e-12)
    u = (0.5 + np.arange(37)) / 37
    assert np.allclose(transition.resample_chain(x, 37), curve(u), atol=1e-12)


@pytest.fixture
def cycle_file(tmp_path):
    cfg = SimulationConfig()
    d = synthetic.make_c2()
    a = mitotic.anatelophase_design(d, cfg.mitotic_phase)
    p = mitotic.prometaphase_design(a, cfg.mitotic_phase, d.master_seed)
    path = tmp_path / "cycle.h5"
    store.write_prepared(path, cfg, d, d.master_seed, anatelophase=a, prometaphase=p)
    return path, cfg, d, a, p


def test_interphase_transition(cycle_file):
    path, cfg, d, a, _ = cycle_file
    rng = np.random.default_rng(0)
    tel = np.cumsum(rng.normal(scale=0.3, size=(a.n, 3)), axis=0)
    with store.SimulationStore(path) as st:
        st.set_stage("telophase")
        st.save_positions(0, tel * 0.5)
        st.save_positions(50, tel)
        st.append_frame(0)
        st.append_frame(50)  # the last frame is the one refined
        transition.transition_interphase(st)
        st.set_stage("relaxation")
        x = st.load_positions(0)
    assert x.shape == (d.n, 3)
    for (_, ts, te, _), (_, s, e) in zip(a.chains, d.chains):
        # the refined chain passes near the coarse beads it interpolates (ends are extrapolated half a bin)
        mid = s + ((np.arange(te - ts) + 0.5) * (e - s) / (te - ts)).astype(int)
        assert np.abs(x[mid] - store.quantize_positions(tel[ts:te])).max() < 0.2
    for nor, nuc in d.nucleolar_bonds:
        assert np.array_equal(x[nuc], x[nor])


def test_prometaphase_and_cycle_transitions(cycle_file, tmp_path):
    path, cfg, d, a, p = cycle_file
    xi = np.random.default_rng(1).normal(size=(d.n, 3))
    with store.SimulationStore(path) as st:
        st.set_stage("interphase")
        st.save_positions(400, xi)
        st.append_frame(400)
        transition.transition_prometaphase(st)
        st.set_stage("prometaphase")
        xp = st.load_positions(0)
    xq = store.quantize_positions(xi).astype(np.float64)
    cg = cfg.mitotic_phase.coarse_graining
    (_, ts, te, _), (_, ss, se, _) = p.chains[0], p.chains[1]
    _, s0, _ = d.chains[0]
    assert np.allclose(xp[ts + 3], store.quantize_positions(xq[s0 + 3 * cg: s0 + 4 * cg].mean(axis=0)))
    disp = -cfg.mitotic_phase.sister_separation * np.array(cfg.mitotic_phase.spindle_axis) / 5.0
    assert np.abs(xp[ss:se] - xp[ts:te] - disp).max() < 1e-4
    # cycle: the target chromatids, shifted by -spindle_axis, into a daughter file's anaphase step 0
    nxt = tmp_path / "daughter.h5"
    store.write_prepared(nxt, cfg, d, d.master_seed + 1, anatelophase=a, prometaphase=p)
    with store.SimulationStore(path) as prev, store.SimulationStore(nxt) as st:
        prev.set_stage("prometaphase")
        prev.append_frame(0)
        transition.transition_cycle(prev, st)
        st.set_stage("anaphase")
        xa = st.load_positions(0)
    assert np.allclose(xa[a.chains[0][1]:a.chains[0][2]], xp[ts:te] - [0, 5, 0], atol=1e-4)
