#!/usr/bin/env python3
"""Generate the benchmark's starting state: the synthetic C2 system (gcs/synthetic.py, master seed 1) run through
the interphase schedule from step 0 to step 300,000 (t = 3: core_scale 0.9988, the wall expanded by the wall
ODE), i.e. the state of a real trajectory in the regime of >90 % of the reference's 700,000 interphase steps.

    python tools/make_bench_state.py [out.npz]      (on a GPU; ~20 s)

Positions are stored as float32 (the engine's device precision) with the context; bench.py loads them.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))

from gcs import interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

STEPS = 300_000
SEED = 20251015


def main():
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "benchdata" / "c2_interphase_step300000.npz"
    cfg = InterphaseConfig()
    design = synthetic.make_c2(master_seed=1)
    e, _ = interphase.build_interphase(Engine, design, cfg)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.apply_schedule(0)
    e.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    e.synchronize()
    x = e.get_positions().astype(np.float32)
    c = e.get_context()
    prof = e.profile(10, first_step=STEPS, seed=SEED)
    np.savez_compressed(out, positions=x, step=np.int64(STEPS), time=np.float64(c["time"]),
                        core_scale=np.float64(c["core_scale"]), bond_scale=np.float64(c["bond_scale"]),
                        wall_semiaxes=np.asarray(c["wall_semiaxes"], np.float64), master_seed=np.int64(1),
                        noise_seed=np.int64(SEED), mean_neighbors=np.float64(prof["mean_neighbors"]))
    print(f"{out}: step {STEPS}, core_scale {c['core_scale']:.6f}, wall {c['wall_semiaxes']}, "
          f"mean neighbours {prof['mean_neighbors']:.2f}, finite {bool(np.isfinite(x).all())}")


if __name__ == "__main__":
    main()
