"""GPU: long-horizon C2 statistics of the engine's production step against the fp64 oracle's ensemble (SURVEY.md
§4.6; the regime of simulation_driver_interphase.cpp:57-63).

Trajectories are chaotic, so beyond a few hundred steps fp32 vs fp64 parity is statistical: the engine's list step
(the default: lists + skin + exact fallback, Philox noise) runs the protocol of tests/ensemble_protocol.py for
NSEED seeds of its own and the time-averaged observables (mean chain-bond length, Rg, E/N, wall semiaxes) are
compared with the oracle ensemble committed in tests/golden/c2_oracle_ensemble.npz (tests/golden/gen_c2_ensemble.py)
within 3 standard errors of the difference of the seed means.  The two ensembles share no code beyond the
force-field composition and no noise stream (different seeds)."""
from pathlib import Path

import numpy as np
import pytest

import ensemble_protocol as P
from gcs.engine import Engine

pytestmark = pytest.mark.gpu

FIXTURE = Path(__file__).resolve().parent / "golden" / "c2_oracle_ensemble.npz"


def test_c2_long_horizon_ensemble_matches_oracle():
    ref = np.load(FIXTURE, allow_pickle=False)
    assert int(ref["steps"]) == P.STEPS and int(ref["every"]) == P.EVERY and int(ref["skip"]) == P.SKIP
    oracle_means = ref["samples"].mean(axis=1)  # [seed][observable], time averages
    engine_means = []
    for k in range(P.NSEED):
        s = P.build(Engine)
        samples = np.array(P.trajectory(s, P.ENGINE_SEED0 + k))
        assert np.isfinite(s.get_positions()).all()
        st = s.list_stats()
        assert st["active"] == 1 and st["sync_stalls"] == 0, st
        engine_means.append(samples.mean(axis=0))
        s.close()
    engine_means = np.array(engine_means)
    me, mo = engine_means.mean(axis=0), oracle_means.mean(axis=0)
    se = engine_means.std(axis=0, ddof=1) / np.sqrt(len(engine_means))
    so = oracle_means.std(axis=0, ddof=1) / np.sqrt(len(oracle_means))
    z = np.abs(me - mo) / np.sqrt(se ** 2 + so ** 2 + 1e-30)
    report = {n: (float(a), float(b), float(c)) for n, a, b, c in zip(P.NAMES, me, mo, z)}
    print({"ensemble engine/oracle/z": report})
    assert (z <= 3.0).all(), report
    assert (se[:3] > 0).all() and (so[:3] > 0).all()
