#!/usr/bin/env python3
"""Benchmark: bead-updates/s of the interphase Brownian-dynamics step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): C2 = synthetic female diploid hg38 at 100 kb, 60,662 particles, the full
interphase force field (simulation_driver_forcefield.cpp:9-244) with the device-resident schedule and wall ODE,
Philox noise.  A step = one force evaluation + Euler-Maruyama update of every particle (+ the cell-list rebuild
and the schedule tail), i.e. one iteration of md::simulate_brownian_dynamics.  The timed window starts at step
300,000 (t = 3, core_scale = 0.9988): the regime of >90 % of the reference's 700,000 production steps.
Inputs are resident in HBM before the timed region.

Multi-GPU (torchrun): one independent replica per rank (own master seed, like `scripts/simulate -s`), no data-path
collective; value = all particle updates / max-over-ranks time ("scaling": "weak").

Rank 0 prints ONE JSON line.  See DESIGN.md "Measurement" for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))

import numpy as np  # noqa: E402

from gcs import _abi as A  # noqa: E402

A.load()  # bind the engine's HIP runtime before torch loads its own copy

from gcs import interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

BYTES_PER_UPDATE = 36  # algorithmic: 12 B position read + 12 B position write + 12 B {mu, a, b}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md "Chip-level parameters")
WINDOW_START = 300_000


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo on CPU tensors: barrier + max only (no data-path collective)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local, dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, v):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_master_seed(rank: int) -> int:
    """Each rank is an independent trajectory with its own master seed (like `scripts/simulate -s <seed>`)."""
    return 1 + rank


def replica_noise_seed(rank: int) -> int:
    return 1000003 * (rank + 1)


def whole_job_value(n: int, steps: int, world: int, el_max: float) -> float:
    """bead-updates/s of the whole job: every rank advanced n particles by `steps`; the slowest rank sets the time."""
    return n * steps * world / el_max


def make_engine(design, cfg, device, start_step):
    e, _ = interphase.build_interphase(Engine, design, cfg, device=device)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    t = start_step * cfg.timestep
    cs = 1 - (1 - cfg.core_scale_init) * np.exp(-t / cfg.core_scale_tau)
    bs = 1 - (1 - cfg.bond_scale_init) * np.exp(-t / cfg.bond_scale_tau)
    e.set_context({"step": start_step, "time": t, "core_scale": cs, "bond_scale": bs,
                   "wall_semiaxes": list(cfg.wall_semiaxes_init)})
    return e


def cpu_baseline(design, cfg, start_step, budget_s):
    """The oracle (fp64, 1 thread, reference flags) on a bounded sample of the same workload."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    t = start_step * cfg.timestep
    o.set_context({"step": start_step, "time": t, "core_scale": 1 - 0.5 * np.exp(-t / 0.5),
                   "bond_scale": 1 - 0.5 * np.exp(-t / 0.5), "wall_semiaxes": list(cfg.wall_semiaxes_init)})
    t0 = time.perf_counter()
    o.run(1, first_step=start_step, seed=1)
    one = time.perf_counter() - t0
    steps = max(1, min(200, int(budget_s / max(one, 1e-6))))
    t0 = time.perf_counter()
    o.run(steps, first_step=start_step + 1, seed=1)
    el = time.perf_counter() - t0
    return {"value": design.n * steps / el, "unit": "bead-updates/s", "cores": 1, "kind": "port",
            "sample": f"C2 {design.n} particles, {steps} steps from step {start_step + 1} "
                      f"({el:.1f} s, oracle/libgcs_oracle.so fp64 single thread, -O2 -funsafe-math-optimizations)"}


def read_traffic():
    """HBM bytes per force launch from the committed rocprofv3 PMC pass (profiles/), if present."""
    p = ROOT / "profiles" / "pmc_force_traffic.json"
    if p.exists():
        try:
            return json.loads(p.read_text()).get("bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c5"])
    ap.add_argument("--graph-steps", type=int, default=32)
    ap.add_argument("--waves", type=int, default=4)
    ap.add_argument("--chunk-order", type=int, default=1)
    ap.add_argument("--split", type=int, default=0, help="1: split each tile's candidates over two workgroups")
    ap.add_argument("--prio", type=int, default=700, help="n > 0: wave priority min(3, tile candidates / n)")
    ap.add_argument("--fused", type=int, default=1, help="1: 4-launch step (force kernel bins the new positions)")
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU baseline work (0 = skip)")
    ap.add_argument("--no-start-window", action="store_true", help="skip the secondary step-0 window")
    args = ap.parse_args()

    world, rank, local, dist = dist_setup()
    cfg = InterphaseConfig()
    maker = {"c1": synthetic.make_c1, "c2": synthetic.make_c2, "c5": synthetic.make_c5}[args.config]
    design = maker(master_seed=replica_master_seed(rank))
    n = design.n

    eng = make_engine(design, cfg, local, WINDOW_START)
    eng.set_option(A.OPT_GRAPH_STEPS, args.graph_steps)
    eng.set_option(A.OPT_WAVES_PER_TILE, args.waves)
    eng.set_option(A.OPT_CHUNK_ORDER, args.chunk_order)
    eng.set_option(A.OPT_FUSED_STEP, args.fused)
    eng.set_option(A.OPT_SPLIT_TILES, args.split)
    eng.set_option(A.OPT_TILE_PRIORITY, args.prio)
    seed = replica_noise_seed(rank)

    eng.run(args.warmup, first_step=WINDOW_START, seed=seed)
    eng.synchronize()
    first = WINDOW_START + args.warmup

    barrier(dist)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.run(args.steps, first_step=first, seed=seed)
    eng.synchronize()
    el = time.perf_counter() - t0
    barrier(dist)
    el_max = max_over_ranks(dist, el)

    # per-kernel durations with HIP events on the engine's stream (after the timed region)
    prof = eng.profile(args.profile_steps, first_step=first + args.steps, seed=seed)
    force_ms = prof["force_ms"]
    achieved = n * BYTES_PER_UPDATE / (force_ms * 1e-3) / 1e9
    ctx = eng.get_context()
    x = eng.get_positions()
    finite = bool(np.isfinite(x).all())

    # secondary: the production start window (step 0, core_scale 0.5, ~7x fewer neighbours)
    start_rate = None
    if rank == 0 and not args.no_start_window:
        e0 = make_engine(design, cfg, local, 0)
        e0.set_option(A.OPT_GRAPH_STEPS, args.graph_steps)
        e0.run(64, first_step=0, seed=seed)
        e0.synchronize()
        t1 = time.perf_counter()
        k0 = max(256, args.steps // 4)
        e0.run(k0, first_step=64, seed=seed)
        e0.synchronize()
        start_rate = n * k0 / (time.perf_counter() - t1)
        e0.close()

    if rank != 0:
        eng.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    cpu = None
    if world == 1 and args.cpu_budget > 0:
        cpu = cpu_baseline(design, cfg, WINDOW_START, args.cpu_budget)

    value = whole_job_value(n, args.steps, world, el_max)
    line = {
        "metric": "bead-updates/sec (whole node), 60k-bead diploid interphase",
        "value": value,
        "unit": "bead-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el_max * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"{args.config.upper()} interphase BD step, {n} particles, window from step "
                               f"{WINDOW_START} (core_scale {ctx['core_scale']:.4f})",
                   "particles": n, "replicas": world, "parallelism": f"replicas{world}",
                   "mean_neighbors": prof["mean_neighbors"], "graph_steps": args.graph_steps,
                   "waves_per_tile": args.waves, "chunk_order": args.chunk_order, "fused": args.fused, "split_tiles": args.split, "tile_priority": args.prio, "start_window_value": start_rate, "finite": finite},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": read_traffic(),
                     "kernel": "k_force<kModeStep>", "force_ms": force_ms, "cell_ms": prof["cell_ms"],
                     "tail_ms": prof["tail_ms"], "bytes_per_launch": n * BYTES_PER_UPDATE},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
