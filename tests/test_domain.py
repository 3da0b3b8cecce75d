"""Spatial domain decomposition (C5; gcs/domain.py) on the CPU oracle: the decomposed trajectory
of one system (box ownership: z-slabs or recursive-bisection blocks, band exchange, allreduced wall reaction) equals
the undecomposed oracle run.

Tolerance: positions within 1e-9 and wall semiaxes within 1e-12 after 30 steps (fp64 on both sides; only the
order of the pair-force summation may differ), in-process (2-8 domains) and over gloo with world_size 2 and 4."""
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

from gcs import domain, interphase
from gcs.config import InterphaseConfig

import oracle
from oracle_domain import OracleDomain

ROOT = Path(__file__).resolve().parents[1]
STEPS = 30
SEED = 99


def _single(design, cfg):
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    return o.get_positions(), o.get_context()


def _domains(design, cfg, boxes, halo, only=None):
    doms = []
    for d in range(len(boxes)):
        if only is not None and d != only:
            continue
        o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
        doms.append(OracleDomain(o, d, boxes, halo, interphase.interphase_schedule(cfg),
                                 shared=domain.shared_particles(design)))
    return doms


def _plan(kind, x, ndom):
    return domain.plan_slabs(x[:, 2], ndom) if kind == "slabs" else domain.plan_boxes(x, ndom)


def test_halo_and_shared_particles(c1_design, interphase_cfg):
    from gcs.config import resolution_scaled
    h = domain.domain_halo(interphase_cfg)
    assert h == pytest.approx(7.5 * (1 / 50) ** 0.5 + 0.05)  # the B-type chain bond's reach dominates
    h10 = domain.domain_halo(resolution_scaled(interphase_cfg, 10.0))
    assert h10 == pytest.approx(h * 10 ** (-1 / 3) - 0.05 * 10 ** (-1 / 3) + 0.05)
    sh = domain.shared_particles(c1_design)
    assert set(sh.tolist()) == {500, 1000, 1001}


def test_plan_slabs_partition_and_peers(c1_design, interphase_cfg):
    x = c1_design.positions
    z = x[:, 2]
    halo = domain.domain_halo(interphase_cfg)
    for nd in (1, 2, 3, 8):
        slabs = domain.plan_slabs(z, nd)
        assert slabs[0][0][2] == -np.inf and slabs[-1][1][2] == np.inf
        assert all(slabs[k][1][2] == slabs[k + 1][0][2] for k in range(nd - 1))
        assert all(np.isinf(b[0][:2]).all() and np.isinf(b[1][:2]).all() for b in slabs)
        owners = sum(domain.in_box(x, b).astype(int) for b in slabs)
        assert (owners == 1).all()
        for d in range(nd):
            for p in domain.peers_of(d, slabs, halo):
                assert d in domain.peers_of(p, slabs, halo)
    # thin slabs reach past their neighbours: the peer set grows beyond +-1
    slabs = domain.plan_slabs(z, 8)
    assert max(len(domain.peers_of(d, slabs, halo)) for d in range(8)) > 2


@pytest.mark.parametrize("nd", [1, 2, 3, 4, 5, 7, 8])
def test_plan_boxes_partition_counts_and_peers(nd):
    """recursive bisection: a partition of space (every particle in exactly one box, also points off the start
    structure), equal counts within one particle per cut level, symmetric peers; 8 domains of a compact nucleus
    are 2 x 2 x 2 blocks whose sides stay thicker than the halo (8 slabs are not)"""
    from gcs import synthetic
    d = synthetic.make_c2(1)
    x = d.positions
    boxes = domain.plan_boxes(x, nd)
    assert len(boxes) == nd
    owners = sum(domain.in_box(x, b).astype(int) for b in boxes)
    assert (owners == 1).all()
    rng = np.random.default_rng(1)
    y = rng.normal(scale=5.0, size=(2000, 3))
    assert (sum(domain.in_box(y, b).astype(int) for b in boxes) == 1).all()
    counts = np.array([domain.in_box(x, b).sum() for b in boxes])
    assert counts.max() - counts.min() <= 3
    cfg = InterphaseConfig()
    halo = domain.domain_halo(cfg)
    for k in range(nd):
        for p in domain.peers_of(k, boxes, halo):
            assert k in domain.peers_of(p, boxes, halo)
    if nd == 8:
        # every block is cut once along each axis: 2 x 2 x 2
        for b in boxes:
            assert int(np.isfinite(b[0]).sum() + np.isfinite(b[1]).sum()) == 3
        for b in boxes:
            inside = x[domain.in_box(x, b)]
            side = np.minimum(inside.max(axis=0), b[1]) - np.maximum(inside.min(axis=0), b[0])
            assert (side > halo).all()
        assert max(len(domain.peers_of(k, boxes, halo)) for k in range(8)) == 7


@pytest.mark.parametrize("kind,ndom,halo", [("slabs", 2, None), ("slabs", 3, None), ("slabs", 4, None),
                                            ("slabs", 4, 0.45), ("boxes", 4, None), ("boxes", 8, None),
                                            ("boxes", 8, 0.45)])
def test_decomposed_oracle_matches_single(c1_design, kind, ndom, halo):
    """halo None: the default (chain-bond reach 1.11); 0.45: thin halo, so the shared nucleolar particles (bonds
    of rms 0.55) must come through the allreduce, not the bands."""
    cfg = InterphaseConfig()
    x1, c1 = _single(c1_design, cfg)
    halo = halo or domain.domain_halo(cfg)
    boxes = _plan(kind, c1_design.positions, ndom)
    doms = _domains(c1_design, cfg, boxes, halo)
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    run.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    run.check()
    x = domain.gather_positions(run, c1_design.n)
    assert np.abs(x - x1).max() <= 1e-9
    for d in doms:
        c = d.context()
        assert np.allclose(c["wall_semiaxes"], c1["wall_semiaxes"], rtol=0, atol=1e-12)
        assert c["step"] == c1["step"] and c["core_scale"] == c1["core_scale"]
    # the particles really moved between domains during the run
    x0 = c1_design.positions
    moved = sum(int((domain.in_box(x0, b) & ~domain.in_box(x, b)).sum()) for b in boxes)
    assert moved > 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir, kind):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch.distributed as dist
    from oracle_domain import OracleDomain
    from gcs import domain as D, interphase as I, synthetic
    from gcs.config import InterphaseConfig as IC
    import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    design = synthetic.make_c1()
    cfg = IC()
    halo = D.domain_halo(cfg)
    boxes = D.plan_slabs(design.positions[:, 2], world) if kind == "slabs" else D.plan_boxes(design.positions, world)
    o, _ = I.build_interphase(O.OracleSystem, design, cfg)
    d = OracleDomain(o, rank, boxes, halo, I.interphase_schedule(cfg), shared=D.shared_particles(design))
    run = D.DecomposedRun([d], D.DistTransport(d, dist))
    run.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    run.check()
    x = D.gather_positions(run, design.n, dist)
    if rank == 0:
        np.save(Path(out_dir, "x.npy"), x)
        Path(out_dir, "ctx.json").write_text(json.dumps(d.context()))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("slabs", 2), ("boxes", 4)])
def test_decomposed_oracle_gloo(tmp_path, c1_design, kind, world):
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path), kind), nprocs=world, join=True,
                       start_method="spawn")
    x = np.load(tmp_path / "x.npy")
    ctx = json.loads((tmp_path / "ctx.json").read_text())
    x1, c1 = _single(c1_design, InterphaseConfig())
    assert np.abs(x - x1).max() <= 1e-9
    assert np.allclose(ctx["wall_semiaxes"], c1["wall_semiaxes"], rtol=0, atol=1e-12)


def test_bond_longer_than_halo_is_reported(c1_design):
    """The engine flags it on the device; the oracle domain has no such check, so exercise the run-level
    check with a forced flag."""
    cfg = InterphaseConfig()
    boxes = domain.plan_slabs(c1_design.positions[:, 2], 2)
    doms = _domains(c1_design, cfg, boxes, domain.domain_halo(cfg))
    doms[1]._flags = domain.FLAG_BOND
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    with pytest.raises(domain.DomainError):
        run.check()
