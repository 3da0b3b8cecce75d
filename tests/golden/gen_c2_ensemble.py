"""Writes tests/golden/c2_oracle_ensemble.npz: the fp64 oracle's C2 ensemble over a long horizon (TEST
INFRASTRUCTURE: the fixture `tests/test_gpu_ensemble.py` compares the engine's Philox ensemble with).

Protocol (shared with the test through `tests/ensemble_protocol.py`): C2 (60,662 particles) from the committed bench
state (benchdata/c2_interphase_step300000.npz, step 300,000), the full interphase force field and schedule
(simulation_driver_interphase.cpp:57-63, 67-90), Philox noise; `NSEED` trajectories of `STEPS` steps, observables
(mean chain-bond length, radius of gyration, energy per particle, wall semiaxes) sampled every `EVERY` steps after
`SKIP`.  One process per seed (the oracle is single-threaded, like the reference).

    python tests/golden/gen_c2_ensemble.py [--procs 8]
"""
from __future__ import annotations

import argparse
import sys
import time
from multiprocessing import Pool
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))

import ensemble_protocol as P  # noqa: E402


def one(k):
    import oracle
    t0 = time.time()
    s = P.build(oracle.OracleSystem)
    samples = P.trajectory(s, P.ORACLE_SEED0 + k)
    print(f"seed {k}: {len(samples)} samples, {time.time() - t0:.0f} s", flush=True)
    return np.array(samples)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "c2_oracle_ensemble.npz"))
    a = ap.parse_args()
    with Pool(a.procs) as pool:
        res = pool.map(one, range(P.NSEED))
    np.savez_compressed(a.out, samples=np.stack(res), names=np.array(P.NAMES), nseed=P.NSEED, steps=P.STEPS,
                        every=P.EVERY, skip=P.SKIP, seed0=P.ORACLE_SEED0)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
