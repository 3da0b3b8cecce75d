"""Step-shape crossover: single-trajectory bead-updates/s of the list step (GCS_OPT_FUSED_STEP 3) and the unfused tile
step (0) on states of different density -- C2's synthetic start, C2's bench window (step 300,000), C5's synthetic
start -- with the mean neighbour count within the cutoff.  The data behind GCS_OPT_DENSE_NEIGHBORS.

usage: python tools/shape_probe.py [warm_steps] [timed_steps]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi as A  # noqa: E402
from gcs import interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig, resolution_scaled  # noqa: E402
from gcs.engine import Engine  # noqa: E402

warm = int(sys.argv[1]) if len(sys.argv) > 1 else 64
timed = int(sys.argv[2]) if len(sys.argv) > 2 else 256


def c2_window():
    z = np.load(ROOT / "benchdata" / "c2_interphase_step300000.npz")
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    return synthetic.make_c2(), InterphaseConfig(), z["positions"], ctx


cases = {
    "c2_start": lambda: (synthetic.make_c2(), InterphaseConfig(), None, None),
    "c2_window": c2_window,
    "c5_start": lambda: (synthetic.make_c5(), resolution_scaled(InterphaseConfig(), 10.0), None, None),
}
for name, make in cases.items():
    design, cfg, x, ctx = make()
    for fused in (3, 0):
        e, _ = interphase.build_interphase(Engine, design, cfg)
        e.set_schedule(**interphase.interphase_schedule(cfg))
        e.set_option(A.OPT_FUSED_STEP, fused)
        e.set_option(A.OPT_DENSE_NEIGHBORS, 0)
        if x is not None:
            e.set_positions(x)
        if ctx is not None:
            e.set_context(ctx)
        else:
            e.apply_schedule(0)
        first = e.get_context()["step"]
        e.run(warm, first_step=first, temperature=cfg.temperature, timestep=cfg.timestep, seed=5)
        e.synchronize()
        t0 = time.perf_counter()
        e.run(timed, first_step=first + warm, temperature=cfg.temperature, timestep=cfg.timestep, seed=5)
        e.synchronize()
        dt = time.perf_counter() - t0
        rc = max(cfg.a_core_diameter, cfg.b_core_diameter) * e.get_context()["core_scale"]
        nb = 2.0 * len(e.search_neighbors(rc)) / design.n
        print(f"{name:10s} fused={fused} {design.n * timed / dt:.3e} bead-updates/s  {dt / timed * 1e6:.1f} us/step  "
              f"neighbours {nb:.1f}", flush=True)
        e.close()
