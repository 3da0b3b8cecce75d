"""Steps/s of the persistent small-system step alone (fp64, anatelophase and prometaphase systems), for same-box A/B
of library variants (GCS_LIB): usage python tools/pstep_time.py [steps] [label]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import mitotic, synthetic  # noqa: E402
from gcs.config import MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
label = sys.argv[2] if len(sys.argv) > 2 else ""
cfg = MitoticPhaseConfig()
d = synthetic.make_c2()
a = mitotic.anatelophase_design(d, cfg)
p = mitotic.prometaphase_design(a, cfg, d.master_seed)
out = []
for stage, design, build in (("anatelophase", a, mitotic.build_anatelophase),
                             ("prometaphase", p, mitotic.build_prometaphase)):
    s, h = build(Engine, design, cfg, precision=64)
    if stage == "anatelophase":
        mitotic.AnatelophaseDriver(s, h, design, cfg, log=None).run_initialization()
    else:
        s.set_positions(np.random.default_rng(1).normal(scale=2.0, size=(design.n, 3)))
    bd = dict(temperature=cfg.temperature, timestep=cfg.timestep, seed=3)
    s.run(2000, **bd)
    s.synchronize()
    best = 0.0
    for rep in range(3):
        t0 = time.perf_counter()
        s.run(steps, first_step=2000 + rep * steps, **bd)
        s.synchronize()
        best = max(best, steps / (time.perf_counter() - t0))
    out.append(f"{stage} {best:9.0f} steps/s ({1e6 / best:5.2f} us)")
    s.close()
print(label, " | ".join(out), flush=True)
