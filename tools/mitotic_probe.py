"""Timing of the mitotic stages (C3, 586 / 1,172 particles) through the stage drivers, no store: steps/s of the
anaphase, telophase and prometaphase stages at the reference's cadence (sampling / logging every 1,000 / 10,000
steps).  Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

usage: python tools/mitotic_probe.py [steps_per_stage] [small_path 0|1]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi, mitotic, synthetic  # noqa: E402
from gcs.config import MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
small = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # GCS_OPT_SMALL_PATH for both systems
cfg = MitoticPhaseConfig()
d = synthetic.make_c2(1)
ad = mitotic.anatelophase_design(d, cfg)
pd = mitotic.prometaphase_design(ad, cfg, 1)
s, h = mitotic.build_anatelophase(Engine, ad, cfg)
s.set_option(_abi.OPT_SMALL_PATH, small)
drv = mitotic.AnatelophaseDriver(s, h, ad, cfg, log=None)
drv.run_initialization()
t0 = time.perf_counter()
drv.run_dragging_stage(steps)
s.synchronize()
t1 = time.perf_counter()
drv.run_packing_stage(steps // 4)
s.synchronize()
t2 = time.perf_counter()
x = s.get_positions()
print(f"anaphase {ad.n} particles: {steps / (t1 - t0):.0f} steps/s; telophase: {steps // 4 / (t2 - t1):.0f} steps/s",
      flush=True)
p, _ = mitotic.build_prometaphase(Engine, pd, cfg)
import numpy as np  # noqa: E402
xp = np.concatenate([x, x + 0.3])[: pd.n]  # any start structure of the right size (timing only)
p.set_option(_abi.OPT_SMALL_PATH, small)
pdrv = mitotic.PrometaphaseDriver(p, pd, cfg, log=None)
t0 = time.perf_counter()
pdrv.run(xp, steps)
p.synchronize()
t1 = time.perf_counter()
print(f"prometaphase {pd.n} particles: {steps / (t1 - t0):.0f} steps/s", flush=True)
print("run stats", s.run_stats(), p.run_stats(), s.list_stats()["rebuild_every"], flush=True)
