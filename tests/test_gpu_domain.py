"""GPU: the spatial domain decomposition (C5, gcs/domain.py + csrc/domain.hip) with HIP engines: several domains in
one process on one device (LocalTransport: bands device-to-device), several processes on one device (DistTransport,
host-staged over gloo: RCCL refuses two ranks on one GPU), and the engine-issued RCCL sequence with one rank
(gcs_engine_domain_run: allreduce + grouped send/recv on the engine stream, graph-captured), against the undecomposed
engine, each other and the fp64 oracle.  Both decomposed step shapes: the list step (k_lstep<..., DOM>, the default)
and the tile step (GCS_OPT_FUSED_STEP 0); both geometries: z-slabs and recursive-bisection boxes (2 x 2 x 2 at 8).

Both precisions: the fp64 engine (the default) decomposes on its list step; the tile-step cases are fp32 only.
Tolerances (tests/tolerances.py, per precision): positions vs the single engine and the fp64 oracle 1e-9 (fp64) /
2e-5 (fp32) after 30 steps (the domains' cell lists order the pair sums differently from the single engine's), wall
semiaxes relative 1e-12 / 1e-7; the protocol flags (bond beyond the halo, band over capacity, lost particle,
displacement beyond the halo) must stay clear."""
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

from gcs import _abi as A
from gcs import domain, interphase, synthetic
from gcs.config import InterphaseConfig
from gcs.engine import Engine
from tolerances import WALL_REL, X

import oracle

pytestmark = pytest.mark.gpu

STEPS = 30
SEED = 99


def _engine(design, cfg, fused=None, prec=32):
    e, _ = interphase.build_interphase(Engine, design, cfg, device=0, precision=prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    if fused is not None:
        e.set_option(A.OPT_FUSED_STEP, fused)
    return e


def _plan(kind, design, ndom):
    x = design.positions
    return domain.plan_slabs(x[:, 2], ndom) if kind == "slabs" else domain.plan_boxes(x, ndom)


def _decomposed(design, cfg, ndom, steps, cap=None, halo=None, kind="slabs", fused=None, prec=32):
    halo = halo or domain.domain_halo(cfg)
    boxes = _plan(kind, design, ndom)
    sh = domain.shared_particles(design)
    doms = [domain.EngineDomain(_engine(design, cfg, fused, prec), d, boxes, halo, cap=cap, shared=sh)
            for d in range(ndom)]
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    run.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    return run, doms, boxes


@pytest.mark.parametrize("kind,ndom,halo,fused,prec", [
    ("slabs", 2, None, None, 32), ("slabs", 4, None, None, 32), ("slabs", 3, 0.5, None, 32),
    ("boxes", 4, None, None, 32), ("boxes", 8, None, None, 32), ("slabs", 2, None, 0, 32), ("boxes", 4, None, 0, 32),
    ("slabs", 2, None, None, 64), ("slabs", 3, 0.5, None, 64), ("boxes", 4, None, None, 64),
    ("boxes", 8, None, None, 64)])
def test_decomposed_engines_match_single_engine_c1(c1_design, kind, ndom, halo, fused, prec):
    cfg = InterphaseConfig()
    single = _engine(c1_design, cfg, prec=prec)
    single.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1, c1 = single.get_positions(), single.get_context()
    run, doms, boxes = _decomposed(c1_design, cfg, ndom, STEPS, halo=halo, kind=kind, fused=fused, prec=prec)
    run.check()
    # the list step ran decomposed (its builds), or the tile step (no lists)
    st = doms[0].e.list_stats()
    builds = st["builds"]
    assert (builds >= 1 + (STEPS - 1) // st["rebuild_every"]) if fused is None else builds == 0, st
    x = domain.gather_positions(run, c1_design.n)
    assert np.abs(x - x1).max() <= X[prec]
    for d in doms:
        c = d.context()
        assert c["step"] == c1["step"]
        assert np.allclose(c["wall_semiaxes"], c1["wall_semiaxes"], rtol=WALL_REL[prec], atol=0)
    # and against the fp64 oracle's undecomposed run (the oracle's predicate in the engine's precision)
    o, _ = interphase.build_interphase(oracle.OracleSystem, c1_design, cfg, precision=prec)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.run(STEPS, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert np.abs(x - o.get_positions()).max() <= X[prec]


@pytest.mark.parametrize("kind,ndom,prec", [("slabs", 4, 32), ("boxes", 8, 32), ("boxes", 8, 64)])
def test_decomposed_engines_c2(kind, ndom, prec):
    cfg = InterphaseConfig()
    design = synthetic.make_c2()
    single = _engine(design, cfg, prec=prec)
    single.run(20, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1 = single.get_positions()
    run, doms, _ = _decomposed(design, cfg, ndom, 20, kind=kind, prec=prec)
    run.check()
    x = domain.gather_positions(run, design.n)
    assert np.abs(x - x1).max() <= X[prec]


def test_motion_beyond_halo_is_reported(c1_design):
    """list step: a hot system (T x 400) rebuilt every 64 steps with a halo just above the list radius; the
    largest displacement since the build soon exceeds halo - cutoff, which the domain tail flags"""
    cfg = InterphaseConfig()
    doms = []
    boxes = domain.plan_boxes(c1_design.positions, 2)
    for d in range(2):
        e = _engine(c1_design, cfg)
        e.set_option(A.OPT_LIST_EVERY, 64)
        doms.append(domain.EngineDomain(e, d, boxes, 0.3 * 1.4 + 0.01, shared=domain.shared_particles(c1_design)))
    run = domain.DecomposedRun(doms, domain.LocalTransport(doms))
    run.run(60, first_step=0, temperature=400.0 * cfg.temperature, timestep=cfg.timestep, seed=SEED)
    with pytest.raises(domain.DomainError, match="halo"):
        run.check()


@pytest.mark.parametrize("poison", [None, "2"])
def test_band_capacity_overflow_is_reported(c1_design, poison, monkeypatch):
    """bands over capacity are flagged (the check raises).  With every allocation poisoned (GCS_DEBUG_POISON=2): the
    ghosts that miss their records keep their build's record in both parities (kernels.hip k_cell_sort) and a lane
    that integrates nothing never indexes by its record's particle -- round 6's suite faulted here once memory was
    recycled (the stale ghost's garbage index gathered by the local terms' batch padding)"""
    cfg = InterphaseConfig()
    if poison:
        monkeypatch.setenv("GCS_DEBUG_POISON", poison)
    run, doms, _ = _decomposed(c1_design, cfg, 2, 4, cap=8)
    with pytest.raises(domain.DomainError):
        run.check()
    for d in doms:
        d.e.close()


def test_bond_beyond_halo_is_reported(c1_design):
    """A halo below the chain bonds' length (C1 starts with every bond 0.1 long): the pack kernel flags it."""
    cfg = InterphaseConfig()
    run, _, _ = _decomposed(c1_design, cfg, 2, 2, halo=0.09)
    with pytest.raises(domain.DomainError, match="bond"):
        run.check()


def test_decomposed_c5_scaled_two_domains():
    """C5 (606,248 beads, the 10 kb force field and timestep of config.resolution_scaled), 2 domains and one engine,
    each against the fp64 oracle under the absolute C5 bound of tests/test_gpu_parity_long.py (2e-5 after 10
    steps; the derivation is there and in DESIGN.md §6)."""
    from gcs.config import resolution_scaled
    cfg = resolution_scaled(InterphaseConfig(), 10.0)
    design = synthetic.make_c5()
    steps = 10
    single = _engine(design, cfg)
    single.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    x1 = single.get_positions()
    run, doms, _ = _decomposed(design, cfg, 2, steps, kind="boxes")
    run.check()
    x = domain.gather_positions(run, design.n)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.set_positions(np.asarray(design.positions, dtype=np.float32).astype(np.float64))
    o.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    xo = o.get_positions()
    e_single = np.abs(x1 - xo).max()
    e_dec = np.abs(x - xo).max()
    assert np.isfinite(x).all()
    assert e_single <= 2e-5 and e_dec <= 2e-5, (e_dec, e_single)


@pytest.mark.parametrize("fused,prec", [(None, 32), (0, 32), (None, 64)])
def test_rccl_run_one_rank_equals_host_driven(c1_design, fused, prec):
    """gcs_engine_domain_run with one rank (RCCL allreduce on the engine stream; 70 steps = a priming step, two
    captured 32-step graphs (list step: whole rebuild periods, recaptured for the second call's phase) and eager
    steps) equals the host-driven step sequence of the same domain bit for bit"""
    from gcs.engine import rccl_unique_id
    cfg = InterphaseConfig()
    halo = domain.domain_halo(cfg)
    slabs = domain.plan_slabs(c1_design.positions[:, 2], 1)
    sh = domain.shared_particles(c1_design)
    ref = domain.EngineDomain(_engine(c1_design, cfg, fused, prec), 0, slabs, halo, shared=sh)
    run = domain.DecomposedRun([ref], domain.LocalTransport([ref]))
    run.run(70, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    d = domain.EngineDomain(_engine(c1_design, cfg, fused, prec), 0, slabs, halo, shared=sh)
    d.e.domain_rccl(rccl_unique_id(), 1, 0, [])
    d.e.domain_run(30, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    d.e.domain_run(40, first_step=30, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert d.flag_bits() == 0
    xd, cd = d.positions(), d.context()
    d.e.close()  # the communicator goes with the engine, before interpreter teardown
    assert np.array_equal(xd, ref.positions())
    assert cd == ref.context()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir, config, prec=32):
    """one domain per process, all on device 0, host-staged over gloo (C1: z-slabs; C2: boxes)"""
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "3d-genome-cycle_amd"))
    import torch.distributed as dist
    from gcs import domain as D, interphase as I, synthetic as S
    from gcs.config import InterphaseConfig as IC
    from gcs.engine import Engine as E
    dist.init_process_group("gloo", rank=rank, world_size=world)
    design, cfg = (S.make_c1() if config == "c1" else S.make_c2()), IC()
    e, _ = I.build_interphase(E, design, cfg, device=0, precision=prec)
    e.set_schedule(**I.interphase_schedule(cfg))
    boxes = (D.plan_slabs(design.positions[:, 2], world) if config == "c1"
             else D.plan_boxes(design.positions, world))
    d = D.EngineDomain(e, rank, boxes, D.domain_halo(cfg), shared=D.shared_particles(design))
    run = D.DecomposedRun([d], D.DistTransport(d, dist))
    run.run(_steps(config), first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    run.check()
    x = D.gather_positions(run, design.n, dist)
    if rank == 0:
        np.save(Path(out_dir, "x.npy"), x)
        Path(out_dir, "ctx.json").write_text(json.dumps(d.context()))
    dist.destroy_process_group()


def _steps(config):
    return STEPS if config == "c1" else 20


@pytest.mark.parametrize("config,world,prec", [("c1", 2, 32), ("c2", 4, 32), ("c2", 8, 32), ("c1", 2, 64),
                                               ("c2", 4, 64)])
def test_engine_domains_processes_host_staged(tmp_path, config, world, prec):
    """`world` processes, one engine domain each (device 0), reaction allreduce and bands over gloo: within 2e-5 of
    the single engine; with two domains also bit for bit the in-process run (the same kernels; a two-term sum is
    order-free; gloo's 4-term sum may associate differently from the host's)"""
    # stdlib spawn, not torch.multiprocessing: this process keeps one HIP runtime (libgcs's); torch (for gloo) is
    # imported by the ranks only, before their engines load libgcs
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, str(tmp_path), config, prec)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    x = np.load(tmp_path / "x.npy")
    ctx = json.loads((tmp_path / "ctx.json").read_text())
    cfg = InterphaseConfig()
    design = synthetic.make_c1() if config == "c1" else synthetic.make_c2()
    steps = _steps(config)
    if world == 2:
        run, doms, _ = _decomposed(design, cfg, world, steps, prec=prec)
        xl = domain.gather_positions(run, design.n)
        assert np.array_equal(x, xl)
        assert ctx["wall_semiaxes"] == doms[0].context()["wall_semiaxes"]
    single = _engine(design, cfg, prec=prec)
    single.run(steps, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert np.abs(x - single.get_positions()).max() <= X[prec]
    assert np.allclose(ctx["wall_semiaxes"], single.get_context()["wall_semiaxes"], rtol=WALL_REL[prec], atol=0)


@pytest.mark.parametrize("prec", [64, 32])
def test_decomposed_run_twice_in_one_process(c1_design, prec, monkeypatch):
    """VERDICT r5 item 1.  The round-5 fault came on the SECOND identical 2-domain run of a process: the decomposed
    step launches a workgroup per 64 of ALL n slots, but a domain's build writes only its binned slots; the others
    kept what their allocation held -- zeros on fresh pages, anything on a recycled allocation -- and the local-terms
    wave (every lane, `act` masks only the results) followed that garbage bond row (kernels.hip k_cell_sort now
    writes a harmless record there).  The same decomposed case three times in this process, the third with every
    per-slot list buffer filled with hashed garbage at allocation (GCS_DEBUG_POISON): bit for bit the same positions
    and context every time, the checks clear (the third run with EVERY allocation poisoned, GCS_DEBUG_POISON=2)"""
    cfg = InterphaseConfig()
    outs = []
    for k in range(3):
        if k == 2:
            monkeypatch.setenv("GCS_DEBUG_POISON", "2")
        run, doms, _ = _decomposed(c1_design, cfg, 2, STEPS, prec=prec)
        run.check()
        outs.append((domain.gather_positions(run, c1_design.n), doms[0].context()))
        for d in doms:
            d.e.close()
    for x, c in outs[1:]:
        assert np.array_equal(x, outs[0][0])
        assert c == outs[0][1]


@pytest.mark.parametrize("prec", [64, 32])
def test_list_step_poisoned_buffers_bitwise(c1_design, prec, monkeypatch):
    """the undecomposed list step with its per-slot buffers poisoned at allocation (GCS_DEBUG_POISON): every slot is
    rebuilt before it is read, so the trajectory is bitwise the unpoisoned one"""
    cfg = InterphaseConfig()
    xs = []
    for poison in (False, True):
        if poison:
            monkeypatch.setenv("GCS_DEBUG_POISON", "1")
        e = _engine(c1_design, cfg, 3, prec)
        e.run(40, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
        xs.append(e.get_positions())
        e.close()
    assert np.array_equal(xs[0], xs[1])


@pytest.mark.parametrize("graph", [None, 4])
@pytest.mark.parametrize("prec", [64, 32])
def test_decomposed_skin_follows_core_scale(c1_design, prec, graph):
    """the decomposed list step's skin follows the scheduled core scale as the single engine's does (engine.hip
    enqueue_dom_list_step: a re-gridded rebuild at each level change; gcs_engine_domain_run runs a stretch with a
    change eagerly).  A fast core-scale schedule crosses several levels in 70 steps: the one-rank RCCL run in two
    calls equals the host-driven sequence bit for bit, both within the precision's bound of the single engine, flags
    clear"""
    from gcs.engine import rccl_unique_id
    cfg = InterphaseConfig()
    sched = dict(interphase.interphase_schedule(cfg), core_scale_tau=100 * cfg.timestep / 2.0)
    halo = domain.domain_halo(cfg)
    slabs = domain.plan_slabs(c1_design.positions[:, 2], 1)
    sh = domain.shared_particles(c1_design)

    def eng():
        e = _engine(c1_design, cfg, None, prec)
        e.set_schedule(**sched)
        return e

    ref = domain.EngineDomain(eng(), 0, slabs, halo, shared=sh)
    run = domain.DecomposedRun([ref], domain.LocalTransport([ref]))
    run.run(70, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    run.check()
    d = domain.EngineDomain(eng(), 0, slabs, halo, shared=sh)
    d.e.domain_rccl(rccl_unique_id(), 1, 0, [])
    if graph is not None:  # 4-step graphs between the level changes (the changes' stretches eager)
        from gcs import _abi as A
        d.e.set_option(A.OPT_GRAPH_STEPS, graph)
    d.e.domain_run(30, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    d.e.domain_run(40, first_step=30, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert d.flag_bits() == 0
    xd, skin = d.positions(), d.e.list_stats()["skin"]
    d.e.close()
    assert np.array_equal(xd, ref.positions())
    assert skin > 0.25 * cfg.a_core_diameter * (1 + 1e-6)  # the skin grew with the core scale
    single = eng()
    single.run(70, first_step=0, temperature=cfg.temperature, timestep=cfg.timestep, seed=SEED)
    assert np.abs(single.get_positions() - xd).max() <= X[prec]


def test_skin_base_fixed_once_decomposed(c1_design):
    """GCS_OPT_LIST_SKIN_BASE sizes a decomposed engine's binning halo (engine.hip list_skin_max): once the engine has
    its domain a change is refused (GCS_ESTATE), setting the value it already has is not"""
    cfg = InterphaseConfig()
    run, doms, _ = _decomposed(c1_design, cfg, 2, 2, prec=64)
    e = doms[0].e
    e.set_option(A.OPT_LIST_SKIN_BASE, 0)
    with pytest.raises(A.GcsError):
        e.set_option(A.OPT_LIST_SKIN_BASE, 400)
    run.check()
    for d in doms:
        d.e.close()
