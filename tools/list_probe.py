"""List step timing on the bench workload (C2 at step 300,000, one trajectory): profile() per-kernel times and the
per-workgroup wall-clock stamps of the last profiled k_lstep (GCS_DEBUG_TIMES; wall_clock64 = 100 MHz).

usage: python tools/list_probe.py [fused=3] [extra engine options as NAME=VALUE ...]
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
out = str(ROOT / "gpurun_out" / "list_times.bin")
os.environ["GCS_DEBUG_TIMES"] = out
import bench  # noqa: E402
from gcs import _abi as A  # noqa: E402
from gcs import synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402

opts = dict(a.split("=") for a in sys.argv[1:])
name = opts.pop("config", "c2")  # c5: C5 from its synthetic start (the bench's C5 window)
cfg = bench.bench_config(name)
start = int(opts.pop("start", 0)) or name != "c2"  # 1: the production start window (step 0, core_scale 0.5)
st = None if start else bench.load_state()
w0 = 0 if start else bench.WINDOW_START
e = bench.make_engine(bench.design_maker(name)(), cfg, 0, w0, st,
                      precision=int(os.environ.get("GCS_PROBE_PRECISION", "64")))
e.set_option(A.OPT_FUSED_STEP, int(opts.pop("fused", 3)))
for k, v in opts.items():
    e.set_option(getattr(A, "OPT_" + k.upper()), int(v))
e.run(200, first_step=w0, seed=5, timestep=cfg.timestep)
p = e.profile(40, first_step=w0 + 200, seed=5, timestep=cfg.timestep)
print({k: (round(v * 1e3, 2) if k.endswith("_ms") else v) for k, v in p.items()}, "(us)")
print(e.list_stats())
n = e.n
t = np.fromfile(out, dtype=np.uint64).astype(np.int64)
fb = (n + 63) // 64  # list step workgroups (force_blocks)
f = t[: 8 * fb].reshape(fb, 8)
t0 = f[:, 0].min()
us = lambda v: (v - t0) / 100.0
q = lambda a: f"med {np.median(a):6.2f} p90 {np.percentile(a, 90):6.2f} max {a.max():6.2f}"
act = f[:, 1] > 0
print(f"workgroups {fb}, with a tile {act.sum()}")
print("start             ", q(us(f[:, 0])))
print("pair loop start   ", q(us(f[act, 1])))
print("pair loop end     ", q(us(f[act, 2])))
print("reduced           ", q(us(f[act, 3])))
print("integrated        ", q(us(f[act, 4])))
print("workgroup end     ", q(us(f[:, 5])))
print("ticket            ", q(us(f[:, 6])))
last = f[:, 7] > 0
print("tail end          ", q(us(f[last, 7])), "(last workgroup)")
print("pair loop length  ", q((f[act, 2] - f[act, 1]) / 100.0))
print("local+integrate   ", q((f[act, 4] - f[act, 3]) / 100.0))
order = np.argsort(-f[:, 6])[:6]
print("slowest workgroups (ticket, pair start, pair len, reduce wait, integrate):")
for b in order:
    r = f[b]
    print(f"  wg {b:5d}: {us(r[6]):6.2f}  {us(r[1]):6.2f}  {(r[2]-r[1])/100:6.2f}  {(r[3]-r[2])/100:6.2f}  {(r[4]-r[3])/100:6.2f}")
tt = t[8 * fb: 8 * fb + 2]
print(f"final workgroup: top ticket -> {us(tt[0]):.2f}, rows reduced {us(tt[1]):.2f}, tail end {us(f[last, 7].max()):.2f}")
