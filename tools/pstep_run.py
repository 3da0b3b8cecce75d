"""A bare run of the persistent small-system step on the anatelophase system (fp64), for profilers:
usage: python tools/pstep_run.py [steps] [precision]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import mitotic, synthetic  # noqa: E402
from gcs.config import MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = MitoticPhaseConfig()
a = mitotic.anatelophase_design(synthetic.make_c2(), cfg)
s, h = mitotic.build_anatelophase(Engine, a, cfg, precision=prec)
mitotic.AnatelophaseDriver(s, h, a, cfg, log=None).run_initialization()
s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, seed=3)
s.synchronize()
if os.environ.get("GCS_MAPS_OUT"):  # (diagnostics) the mappings, to symbolise a crash at exit (tools/symbolize_trace.py)
    with open("/proc/self/maps") as src, open(os.environ["GCS_MAPS_OUT"], "w") as dst:
        dst.write(src.read())
s.close()
print("done", steps, flush=True)
