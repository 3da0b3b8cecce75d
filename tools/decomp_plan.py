"""Decomposition geometry of a configuration (no GPU): per rank the owned beads, the region's binned beads (owned +
ghosts), the peers, the band records per peer (owned beads inside the peer's region: what the owner sends each step,
16 B each) and the binning halo's share of the binned set, for recursive-bisection boxes and for z-slabs.  The numbers
DESIGN.md §8 quotes for 8 ranks.

usage: python tools/decomp_plan.py [c2|c5] [ranks...]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import domain, synthetic  # noqa: E402
from gcs.config import InterphaseConfig, resolution_scaled  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "c5"
ranks = [int(v) for v in sys.argv[2:]] or [2, 4, 8]
if config == "c5":
    design, cfg = synthetic.make_c5(), resolution_scaled(InterphaseConfig(), 10.0)
else:
    design, cfg = synthetic.make_c2(), InterphaseConfig()
x = design.positions
n = x.shape[0]
halo = domain.domain_halo(cfg)
rc = max(cfg.a_core_diameter, cfg.b_core_diameter)
bin_halo = min(halo, rc * (1 + 2 * domain.LIST_SKIN))  # the engine's binning halo (engine.hip dom_bin_halo)
print(f"{config}: {n} beads, exchange halo {halo:.3f}, binning halo {bin_halo:.3f} (list radius "
      f"{rc * (1 + domain.LIST_SKIN):.3f})")
for kind in ("boxes", "slabs"):
    for k in ranks:
        boxes = domain.plan_boxes(x, k) if kind == "boxes" else domain.plan_slabs(x[:, 2], k)
        rows = []
        for d in range(k):
            own = domain.in_box(x, boxes[d])
            binned = domain.in_box(x, domain.region(boxes[d], bin_halo))
            peers = domain.peers_of(d, boxes, halo)
            bands = [int((own & domain.in_box(x, domain.region(boxes[p], halo))).sum()) for p in peers]
            rows.append((int(own.sum()), int(binned.sum()), len(peers), sum(bands), max(bands, default=0)))
        r = np.array(rows)
        print(f"  {kind:5s} x{k}: owned {r[:, 0].min()}-{r[:, 0].max()}, binned (owned + ghosts) max {r[:, 1].max()} "
              f"({r[:, 1].max() / r[:, 0].max():.2f} x owned), peers max {r[:, 2].max()}, band records per rank per "
              f"step max {r[:, 3].max()} ({16 * r[:, 3].max() / 1e6:.2f} MB sent), largest band {r[:, 4].max()}")
