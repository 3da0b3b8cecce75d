"""One profiled launch of the bench workload with per-block debug stamps (GCS_DEBUG_TIMES), then force_times.py."""
import os
import subprocess
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
out = str(ROOT / "gpurun_out" / "force_times.bin")
os.environ["GCS_DEBUG_TIMES"] = out
import bench  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs import synthetic  # noqa: E402
cfg = InterphaseConfig()
st = bench.load_state()
e = bench.make_engine(synthetic.make_c2(), cfg, 0, bench.WINDOW_START, st)
e.run(200, first_step=bench.WINDOW_START, seed=5)
p = e.profile(20, first_step=bench.WINDOW_START + 200, seed=5)
print(p)
subprocess.run([sys.executable, str(ROOT / "tools" / "force_times.py"), out], check=True)
