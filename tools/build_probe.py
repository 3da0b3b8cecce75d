"""k_lbuild timeline on the bench workload (one trajectory): per-workgroup wall-clock stamps of the last list build
in a profiled window (GCS_DEBUG_BUILD; wall_clock64 = 100 MHz): start, each wave's candidate-sweep end, tile end,
the tile's candidate count.

usage: python tools/build_probe.py [config=c2|c5] [list_waves=2|4] [other engine options as NAME=VALUE ...]
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
out = str(ROOT / "gpurun_out" / "build_times.bin")
os.environ["GCS_DEBUG_BUILD"] = out
import bench  # noqa: E402
from gcs import _abi as A  # noqa: E402

opts = dict(a.split("=") for a in sys.argv[1:])
name = opts.pop("config", "c2")
cfg = bench.bench_config(name)
st = bench.load_state() if name == "c2" else None
w0 = bench.WINDOW_START if name == "c2" else 0
e = bench.make_engine(bench.design_maker(name)(), cfg, 0, w0, st)
for k, v in opts.items():
    e.set_option(getattr(A, "OPT_" + k.upper()), int(v))
e.run(200, first_step=w0, seed=5, timestep=cfg.timestep)
p = e.profile(40, first_step=w0 + 200, seed=5, timestep=cfg.timestep)
print({k: (round(v * 1e3, 2) if k.endswith("_ms") else v) for k, v in p.items()}, "(us)")
t = np.fromfile(out, dtype=np.uint64).astype(np.int64).reshape(-1, 8)
act = t[:, 1] > 0
f = t[act]
t0 = f[:, 0].min()
us = lambda v: (v - t0) / 100.0
q = lambda a: f"med {np.median(a):7.2f} p90 {np.percentile(a, 90):7.2f} max {a.max():7.2f}"
W = int(opts.get("list_waves", 4))
print(f"workgroups with a tile {act.sum()} of {t.shape[0]}")
print("start            ", q(us(f[:, 0])))
for w in range(W):
    print(f"wave {w} sweep end ", q(us(f[:, 2 + w])))
print("tile end         ", q(us(f[:, 1])))
dur = (f[:, 1] - f[:, 0]) / 100.0
print("tile duration    ", q(dur))
print("candidates/group ", q(f[:, 6].astype(float)))
c = np.corrcoef(f[:, 6], dur)[0, 1]
print(f"corr(candidates, duration) {c:.2f}; us per 32-candidate chunk per wave ~ "
      f"{np.median(dur / np.maximum(f[:, 6] / 32.0 / W, 1)):.2f}")
