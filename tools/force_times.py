"""Summarise a GCS_DEBUG_TIMES dump of the force kernel (per block: start, end, smid << 32 | candidates, first tile;
then per block the wave-0 stamps pair start, pair end, local start, local end; wall_clock64 = 100 MHz).

usage: python tools/force_times.py gpurun_out/times.bin [N]
"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60662
ncm = min(1 << 21, max(4096, 4 * n))
rb = 1 + ncm // 128 + 2
fb = (len(t) - 2 * rb) // 8
f = t[: 4 * fb].reshape(fb, 4)
ph = t[4 * fb: 8 * fb].reshape(fb, 4)
act = f[:, 2] != -1
t0 = f[act, 0].min()
us = lambda v: (v - t0) / 100.0
start, end = us(f[act, 0]), us(f[act, 1])
cand = (f[act, 2] & 0xFFFFFFFF).astype(np.int64)
dur = end - start
p = ph[act]
pair = (p[:, 1] - p[:, 0]) / 100.0
loc = (p[:, 3] - p[:, 2]) / 100.0
pre = (p[:, 0] - f[act, 0]) / 100.0
post = (f[act, 1] - p[:, 3]) / 100.0
q = lambda a: f"med {np.median(a):.2f} p90 {np.percentile(a, 90):.2f} max {a.max():.2f}"
print(f"active blocks {act.sum()} of {fb}; kernel span {end.max():.2f} us; last start {start.max():.2f}")
print("block duration", q(dur))
print("  before pair loop", q(pre))
print("  pair loop (wave 0)", q(pair))
print("  local+integrate (wave 0)", q(loc))
print("  after", q(post))
print("candidates per group (max of the tile's groups)", q(cand.astype(float)))
c = np.corrcoef(cand, pair)[0, 1]
print(f"corr(candidates, pair time) {c:.2f}; pair us per 1000 candidates {1000 * np.median(pair / np.maximum(cand, 1)):.2f}")
order = np.argsort(-end)[:5]
print("latest blocks (end, start, cand):", [(round(end[i], 2), round(start[i], 2), int(cand[i])) for i in order])
