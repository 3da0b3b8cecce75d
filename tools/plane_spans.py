"""Plane spans of the plane-relative list entries (kernels.hip ListRel16) at C5's synthetic start, no GPU: for the list
build's cell grid (x edge r/2, y/z edge r, r = cutoff(cs) + skin) the largest span from a particle's plane base (cell
(x - 2, y - 1) of plane z + dz) to the end of its last partner cell (x + 2, y + 1): must stay below 2^14 slots; and
the largest 5-cell row span.  usage: python tools/plane_spans.py"""
import sys, numpy as np
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1] / "3d-genome-cycle_amd"))
from gcs import synthetic
from gcs.config import InterphaseConfig, resolution_scaled
d = synthetic.make_c5(); cfg = resolution_scaled(InterphaseConfig(), 10.0)
x = d.positions.astype(np.float64); n = len(x)
pd = max(cfg.a_core_diameter, cfg.b_core_diameter)
lo, hi = x.min(0), x.max(0)
for skin in (0.35, 0.5):
  for cs in (0.5, 1.0):
    rc = pd*cs + skin*pd
    edge = np.array([rc/2, rc, rc]); ng = np.maximum(1, np.minimum(1024, ((hi-lo)/(edge*1.0001)).astype(int)))
    while ng.prod() > min(1<<21, max(4096, 4*n)):
        k = int(np.argmax(ng)); ng[k] = max(1, ng[k]//2)
    c = np.minimum(((x-lo)*ng/(hi-lo)).astype(int), ng-1)
    cid = c[:,0] + ng[0]*(c[:,1] + ng[1]*c[:,2])
    cnt = np.bincount(cid, minlength=ng.prod()); cst = np.concatenate([[0], np.cumsum(cnt)])
    def cs_at(cx, cy, cz): return cst[cx + ng[0]*(cy + ng[1]*cz)]
    span_plane = 0; span_row = 0
    for dz in (-1, 0, 1):
        z = c[:,2] + dz; ok = (z >= 0) & (z < ng[2])
        zc = np.clip(z, 0, ng[2]-1)
        ylo = np.maximum(c[:,1]-1, 0); yhi = np.minimum(c[:,1]+1, ng[1]-1)
        xlo = np.maximum(c[:,0]-2, 0); xhi = np.minimum(c[:,0]+2, ng[0]-1)
        sp = cs_at(xhi, yhi, zc) + cnt[xhi + ng[0]*(yhi + ng[1]*zc)] - cs_at(xlo, ylo, zc)
        span_plane = max(span_plane, int(sp[ok].max()))
        for dy in (-1, 0, 1):
            y = c[:,1] + dy; ok2 = ok & (y >= 0) & (y < ng[1]); yc = np.clip(y, 0, ng[1]-1)
            sr = cs_at(xhi, yc, zc) + cnt[xhi + ng[0]*(yc + ng[1]*zc)] - cs_at(xlo, yc, zc)
            span_row = max(span_row, int(sr[ok2].max()))
    print(f"skin {skin} cs {cs}: grid {ng}, max cell {cnt.max()}, max 3-row plane span {span_plane}, max 5-cell row span {span_row}")
