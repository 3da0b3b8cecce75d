"""Positions after a run of the default engine, for comparing two builds of libgcs.so bit for bit (GCS_LIB picks
the library).  usage: GCS_LIB=<lib> python tools/lib_bitwise.py <config c1|c2|c5> <precision> <steps> <out.npy>"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

name, prec, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
cfg = bench.bench_config(name)
st = bench.load_state() if name == "c2" else None
w0 = bench.WINDOW_START if name == "c2" else 0
e = bench.make_engine(bench.design_maker(name)(), cfg, 0, w0, st, precision=prec)
e.run(steps, first_step=w0, seed=7, timestep=cfg.timestep, temperature=cfg.temperature)
np.save(out, e.get_positions())
print(name, prec, steps, e.list_stats())
