"""Decomposed engines vs one engine, step by step (GPU box debugging aid)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-genome-cycle_amd"))
import torch
torch.zeros(1, device="cuda")
import numpy as np
from gcs import domain, interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine

cfg = InterphaseConfig()
design = synthetic.make_c1()


def eng():
    e, _ = interphase.build_interphase(Engine, design, cfg, device=0)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    return e


for ndom, halo_over in ((2, 10.0), (2, None)):
    single = eng()
    halo = halo_over or domain.domain_halo(cfg)
    slabs = domain.plan_slabs(design.positions[:, 2], ndom)
    doms = [domain.EngineDomain(eng(), d, slabs, halo, device=0) for d in range(ndom)]
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    for st in range(2):
        single.run(1, first_step=st, seed=99)
        run.run(1, first_step=st, seed=99)
        x1 = single.get_positions()
        x, m = run.local_positions(design.n)
        err = np.abs(x - x1).max(axis=1)
        bad = np.argsort(err)[-3:]
        own0 = doms[0].owned_mask(x)
        print("slab0 err", err[own0].max(), "slab1 err", err[~own0].max(), "cut", slabs[0][1])
        print(ndom, halo, st, "max err", err.max(), "owned all", m.all(), "worst", bad, x1[bad, 2],
              [d.context()["wall_semiaxes"][0] for d in doms], single.get_context()["wall_semiaxes"][0], flush=True)
