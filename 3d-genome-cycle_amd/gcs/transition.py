"""Stage transitions (stage_transition/*.cpp): host-only O(N) conversions between stages that
close the cell-cycle loop (prepare -> anatelophase -> transition interphase -> interphase -> transition
prometaphase -> prometaphase -> transition cycle -> the daughter's anatelophase).

The refinement uses the cubic spline with not-a-knot end conditions of snsinfu/cxx-spline (an un-vendored
submodule, version unpinned: .gitmodules:16-18); its published algorithm is the unique not-a-knot C2 interpolant,
restated here with scipy.interpolate.CubicSpline(bc_type="not-a-knot") (parity unpinned: no fixture of the
reference's spline exists).
"""
from __future__ import annotations

import numpy as np


def _last_positions(store, stage):
    store.set_stage(stage)
    steps = store.load_steps()
    if not steps:
        raise RuntimeError(f"no frames in stage {stage}")
    return store.load_positions(steps[-1])


def resample_chain(chain: np.ndarray, n_new: int) -> np.ndarray:
    """transition_interphase.cpp:14-41: knots t_k = (k + 0.5) / n, samples at (i + 0.5) / n_new."""
    from scipy.interpolate import CubicSpline
    n = chain.shape[0]
    t = (0.5 + np.arange(n)) / n
    u = (0.5 + np.arange(n_new)) / n_new
    if n == 1:
        return np.repeat(chain, n_new, axis=0)
    return CubicSpline(t, chain, axis=0, bc_type="not-a-knot")(u)


def transition_interphase(store):
    """transition_interphase.cpp:46-84: refine the final telophase frame into the relaxation stage's step 0."""
    tdesign = store.load_anatelophase_design()
    idesign = store.load_interphase_design()
    tpos = _last_positions(store, "telophase")
    ipos = np.zeros((idesign.n, 3))
    for tc, ic in zip(tdesign.chains, idesign.chains):
        ipos[ic[1]:ic[2]] = resample_chain(tpos[tc[1]:tc[2]], ic[2] - ic[1])
    for nor, nuc in idesign.nucleolar_bonds:
        ipos[nuc] = ipos[nor]
    store.set_stage("relaxation")
    store.save_positions(0, ipos)


def transition_prometaphase(store):
    """transition_prometaphase.cpp:43-105: coarse-grain the final interphase frame (centroids of coarse_graining
    beads) into the target chromatids; each sister is its target displaced by -sister_separation along the
    spindle axis."""
    cfg = store.load_config().mitotic_phase
    idesign = store.load_interphase_design()
    pdesign = store.load_prometaphase_design()
    ipos = _last_positions(store, "interphase")
    n = sum(c[2] - c[1] for c in pdesign.chains)
    ppos = np.zeros((n, 3))
    axis = np.asarray(cfg.spindle_axis, dtype=np.float64)
    disp = -cfg.sister_separation * axis / np.linalg.norm(axis)
    cg = cfg.coarse_graining
    for k, src in enumerate(idesign.chains):
        t_i, s_i = pdesign.sister_chromatids[k]
        tch, sch = pdesign.chains[t_i], pdesign.chains[s_i]
        src_len = src[2] - src[1]
        for off in range(tch[2] - tch[1]):
            a = src[1] + cg * off
            b = min(a + cg, a + src_len)  # (the reference's bound: a + min(cg, source length))
            c = ipos[a:b].mean(axis=0)
            ppos[tch[1] + off] = c
            ppos[sch[1] + off] = c + disp
    store.set_stage("prometaphase")
    store.save_positions(0, ppos)


def transition_cycle(prev, nxt):
    """transition_cycle.cpp:25-76: the target chromatids of the final prometaphase frame of `prev`, shifted by
    -spindle_axis (their pole becomes the origin), become `nxt`'s initial anaphase structure."""
    mdesign = prev.load_prometaphase_design()
    adesign = nxt.load_anatelophase_design()
    cfg = nxt.load_config().mitotic_phase
    mpos = _last_positions(prev, "prometaphase")
    n = sum(c[2] - c[1] for c in adesign.chains)
    apos = np.zeros((n, 3))
    disp = -np.asarray(cfg.spindle_axis, dtype=np.float64)
    for k, ach in enumerate(adesign.chains):
        t_i, _ = mdesign.sister_chromatids[k]
        mch = mdesign.chains[t_i]
        ln = mch[2] - mch[1]
        apos[ach[1]:ach[1] + ln] = mpos[mch[1]:mch[2]] + disp
    nxt.set_stage("anaphase")
    nxt.save_positions(0, apos)
