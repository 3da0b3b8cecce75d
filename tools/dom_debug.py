"""Probe of a decomposed run (in-process domains on one GPU): per step the allreduced totals (owned particles,
fallbacks, largest displacement), the flags, owned counts by position vs counted by the step, large jumps, and the
copies of one particle (WATCH=index) in every domain.

usage: python tools/dom_debug.py [slabs|boxes] [domains] [c1|c2] [steps]   (env FUSED, EVERY: engine options)"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi as A  # noqa: E402
from gcs import domain, interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

cfg = InterphaseConfig()
kind = sys.argv[1] if len(sys.argv) > 1 else "slabs"
ndom = int(sys.argv[2]) if len(sys.argv) > 2 else 2
design = synthetic.make_c2() if (len(sys.argv) > 3 and sys.argv[3] == "c2") else synthetic.make_c1()
nsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
boxes = domain.plan_slabs(design.positions[:, 2], ndom) if kind == "slabs" else domain.plan_boxes(design.positions, ndom)
halo = domain.domain_halo(cfg)
doms = []
for d in range(ndom):
    e, _ = interphase.build_interphase(Engine, design, cfg, device=0)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    if os.environ.get("FUSED"):
        e.set_option(A.OPT_FUSED_STEP, int(os.environ["FUSED"]))
    if os.environ.get("EVERY"):
        e.set_option(A.OPT_LIST_EVERY, int(os.environ["EVERY"]))
    doms.append(domain.EngineDomain(e, d, boxes, halo, shared=domain.shared_particles(design)))
run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
for st in range(nsteps):
    pre = [int(d.owned_mask(d.positions()).sum()) for d in doms]
    xpre = [d.positions() for d in doms]
    gpre = domain.gather_positions(run, design.n)
    run.run(1, first_step=st, temperature=cfg.temperature, timestep=cfg.timestep, seed=99)
    post = [int(d.red[7]) for d in doms]
    watch = int(os.environ.get("WATCH", "-1"))
    if watch >= 0:
        for d in doms:
            xw = d.positions()[watch]
            print(st, "nown watch", watch, "dom", d.index, xw, "in box", bool(d.owned_mask(xw[None])[0]),
                  "in region", bool(domain.in_box(xw[None], domain.region(d.box, halo))[0]), flush=True)
    if pre != post:
        print(st, "nown owned by position", pre, "counted by k_lstep", post, flush=True)
    xs = [d.positions() for d in doms]
    try:
        g = domain.gather_positions(run, design.n)
        dx = np.linalg.norm(g - gpre, axis=1)
        i = int(np.argmax(dx))
        if dx[i] > 0.5:
            print(st, "nown jump", dx[i], "particle", i, flush=True)
            for d, a, b in zip(doms, xpre, xs):
                print(st, "nown   dom", d.index, "box", d.box[0], d.box[1], "pre", a[i], "post", b[i],
                      "own pre", bool(d.owned_mask(a[i:i + 1])[0]), flush=True)
    except domain.DomainError as ex:
        print(st, "nown gather", ex, flush=True)
    for d in doms:
        d.synchronize()
    print(st, "nown", int(doms[0].glob[7]), "nfb", int(doms[0].glob[8]), "D", round(doms[0].glob[-ndom:].max(), 4),
          "flags", max(d.flag_bits() for d in doms), "owned", [int(d.red[7]) for d in doms], flush=True)
    xs = [d.positions() for d in doms]
    own = np.array([d.owned_mask(x) for d, x in zip(doms, xs)])
    cnt = own.sum(axis=0)
    bad = np.nonzero(cnt != 1)[0]
    if bad.size:
        i = int(bad[0])
        print("  particles owned != once:", bad.size, "first", i, "owners", np.nonzero(own[:, i])[0].tolist(), flush=True)
        for d, x in zip(doms, xs):
            print("   dom", d.index, "copy", x[i], "in box", bool(d.owned_mask(x[i:i + 1])[0]),
                  "in region", bool(domain.in_box(x[i:i + 1], domain.region(d.box, halo))[0]), flush=True)
        break
