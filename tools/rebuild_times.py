"""Summarise a GCS_DEBUG_TIMES dump of the rebuild step (force per-block words, then rebuild {start, end} pairs).

usage: python tools/rebuild_times.py gpurun_out/times.bin [N] [kRbCells]
"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60662
ncm = min(1 << 21, max(4096, 4 * n))
rb = 1 + ncm // (int(sys.argv[3]) // 2 if len(sys.argv) > 3 else 128) + 2  # rebuild_blocks(): kRbCells / 2
fb = (len(t) - 2 * rb) // 8
f = t[: 4 * fb].reshape(fb, 4)
act = f[:, 2] != -1
t0 = f[act, 0].min()
r = t[8 * fb: 8 * fb + 2 * rb].reshape(rb, 2)
s = (r[:, 0] - t0) / 100.0
e = (r[:, 1] - t0) / 100.0
fe = (f[act, 1].max() - t0) / 100.0
print(f"force: last start {(f[act, 0].max() - t0) / 100:.2f}  last end {fe:.2f} us  ({act.sum()} active blocks)")
print(f"rebuild: first start {s.min():.2f} (gap {s.min() - fe:.2f})  tail block {s[0]:.2f}..{e[0]:.2f}  last end {e.max():.2f} us")
d = e[1:] - s[1:]
work = d > 1.0
print(f"rebuild blocks with work: {work.sum()}, duration median {np.median(d[work]):.2f} max {d[work].max():.2f} us")
print("latest ends:", [(int(i), round(float(e[i]), 2)) for i in np.argsort(-e)[:6]])
