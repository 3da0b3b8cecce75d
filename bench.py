#!/usr/bin/env python3
"""Benchmark: bead-updates/s of the interphase Brownian-dynamics step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): C2 = synthetic female diploid hg38 at 100 kb, 60,662 particles, the full
interphase force field (simulation_driver_forcefield.cpp:9-244) with the device-resident schedule and wall ODE,
Philox noise.  Arithmetic: fp64 (--precision 64, the default), the reference's own (md::scalar is double); the fp32
engine's rate on the same window is reported beside it (config.f32).  A step = one force evaluation + Euler-Maruyama update of every particle (+ the cell-list rebuild
and the schedule tail), i.e. one iteration of md::simulate_brownian_dynamics.  The timed window starts at step
300,000 (t = 3, core_scale = 0.9988): the regime of >90 % of the reference's 700,000 production steps.
Inputs are resident in HBM before the timed region.

Replicas (C4; the reference's ensemble is separate `scripts/simulate -s seed` runs, scripts/simulate:15-18): each
GPU runs --replicas-per-gpu independent trajectories (own noise seed), each with its own engine and HIP stream, so
the GPU overlaps one trajectory's latency-bound launches with another's force kernel.  The single-trajectory rate
is reported beside it (config.single_trajectory_value).

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) every rank runs its own replicas; with
`--gpus N` and no WORLD_SIZE this process is only a launcher: it makes no GPU call and starts N child ranks
(RANK = LOCAL_RANK = r, gloo rendezvous on 127.0.0.1), then exits with their status.  No data-path collective:
gloo carries the barrier, the max-over-ranks time and the per-rank rates only; value = all particle updates of
all ranks / the slowest rank's time ("scaling": "weak").

Timed window: warm-up runs passes of the timed region's own shape (>= 2 passes, >= --warmup steps), so every hipGraph
the timed passes replay is captured and instantiated before timing; then the timed region repeats passes of --steps
steps (per replica) with no host synchronisation until the end, sized to last >= --min-window-s; "steps" reports the
steps actually timed, "steps_requested" the flag, "graph_replays" / "timed_runs" how the engines issued them.

Rank 0 prints ONE JSON line.  See DESIGN.md "Measurement" for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))

import numpy as np  # noqa: E402

# algorithmic bytes per bead-update: position read + position write + {mu, a, b}, 3 scalars each:
# 36 B in fp32, 72 B in fp64
BYTES_PER_UPDATE = {32: 36, 64: 72}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md "Chip-level parameters")
WINDOW_START = 300_000
STATE_FILE = ROOT / "benchdata" / "c2_interphase_step300000.npz"


# ---------------------------------------------------------------------------------------------------------------
# process topology


def dist_setup(backend="gloo"):
    """gloo on CPU tensors: the barrier, the max over ranks and (decomposed runs) the RCCL id hand-out; the
    decomposed runs' data path (reaction allreduce, band exchange) is RCCL issued by the engine itself.
    GCS_BENCH_SAME_DEVICE=1 (tests on a one-GPU box): every rank on device 0."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("GCS_BENCH_SAME_DEVICE") == "1":
        local = 0
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, rank=rank, world_size=world)
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


def gather_over_ranks(dist, v):
    """every rank's value of v (a float), in rank order"""
    if dist is None:
        return [v]
    import torch
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(dist.get_world_size())]
    dist.all_gather(out, torch.tensor([v], dtype=torch.float64))
    return [float(t.item()) for t in out]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, poll_s: float = 0.05, grace_s: float = 5.0) -> int:
    """`bench.py --gpus N` without WORLD_SIZE: start N child ranks of this same script (one per GPU) and wait.
    This process touches no device: the children load the engine after their own environment is set.  The children
    are polled together: the first one to exit non-zero ends the run (the others would wait in their next collective
    until the gloo timeout), so they are terminated -- killed after `grace_s` -- and its exit code returned."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "bench.py")] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live and rc == 0:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = code
                break
        if live and rc == 0:
            time.sleep(poll_s)
    if rc != 0:
        for q in live:  # a rank failed: stop the rest
            q.terminate()
        deadline = time.monotonic() + grace_s
        for q in live:
            try:
                q.wait(timeout=max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    return rc


def replica_master_seed(rank: int) -> int:
    """Each trajectory is independent with its own master seed (like `scripts/simulate -s <seed>`)."""
    return 1 + rank


def replica_noise_seed(rank: int) -> int:
    return 1000003 * (rank + 1)


def whole_job_value(n: int, steps: int, world: int, el_max: float) -> float:
    """bead-updates/s of the whole job: every rank advanced n particles by `steps`; the slowest rank sets the time."""
    return n * steps * world / el_max


# ---------------------------------------------------------------------------------------------------------------
# workload


def load_state():
    """The timed window's starting state: C2 run through the interphase schedule from step 0 to 300,000
    (tools/make_bench_state.py): wall expanded by the wall ODE, ~25 neighbours per bead in the cutoff."""
    z = np.load(STATE_FILE, allow_pickle=False)
    ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
           "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
    return z["positions"].astype(np.float64), ctx


def apply_engine_opts(e, args):
    """experiments: --engine-opt list_skin=300 (gcs._abi OPT_<NAME>); list_deal=d:0120123 -> a deal pattern"""
    from gcs import _abi as A
    for kv in args.engine_opt:
        name, v = kv.split("=")
        e.set_option(getattr(A, "OPT_" + name.upper()), A.list_deal(v[2:]) if v.startswith("d:") else int(v))


def make_engine(design, cfg, device, start_step, state=None, precision=64):
    from gcs import interphase
    from gcs.engine import Engine
    e, _ = interphase.build_interphase(Engine, design, cfg, device=device, precision=precision)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    if os.environ.get("GCS_BENCH_DENSE") is not None:  # (experiments) the dense-start threshold of every engine
        from gcs import _abi as A
        e.set_option(A.OPT_DENSE_NEIGHBORS, int(os.environ["GCS_BENCH_DENSE"]))
    if state is not None:
        x, ctx = state
        e.set_positions(x)
        e.set_context(ctx)
        return e
    t = start_step * cfg.timestep
    cs = 1 - (1 - cfg.core_scale_init) * np.exp(-t / cfg.core_scale_tau)
    bs = 1 - (1 - cfg.bond_scale_init) * np.exp(-t / cfg.bond_scale_tau)
    e.set_context({"step": start_step, "time": t, "core_scale": cs, "bond_scale": bs,
                   "wall_semiaxes": list(cfg.wall_semiaxes_init)})
    return e


class StubEngine:
    """Stands in for gcs.engine.Engine in `--stub-engine` runs (CPU tests of the launcher and the aggregation):
    the same calls, a fixed sleep per step, no device."""

    STEP_S = 2e-5

    def __init__(self, n):
        self.n = n
        self.step = 0

    def set_option(self, *_):
        pass

    def run(self, steps, first_step=0, **_):
        time.sleep(self.STEP_S * steps)
        self.step = first_step + steps

    def synchronize(self):
        pass

    def profile(self, steps, first_step=0, **_):
        self.run(steps, first_step)
        return {"force_ms": 1e3 * self.STEP_S * 0.75, "cell_ms": 1e3 * self.STEP_S * 0.25, "tail_ms": 0.0,
                "mean_neighbors": 25.0}

    def get_context(self):
        return {"step": self.step, "core_scale": 1.0}

    def get_positions(self):
        return np.zeros((self.n, 3))

    def close(self):
        pass


def window_start(name):
    """C2: the committed step-300,000 trajectory state.  C1/C5: their synthetic start (step 0, core_scale 0.5) --
    a synthetic chain packed at the generator's density has ~8x the equilibrated neighbour count at core_scale 1."""
    return WINDOW_START if name == "c2" else 0


def bench_config(name):
    """The interphase defaults; C5's 10 kb beads use the force field rescaled to their size
    (gcs.config.resolution_scaled, DESIGN.md "Measurement")."""
    from gcs.config import InterphaseConfig, resolution_scaled
    cfg = InterphaseConfig()
    return resolution_scaled(cfg, 10.0) if name == "c5" else cfg


def design_maker(name):
    from gcs import synthetic
    return {"c1": synthetic.make_c1, "c2": synthetic.make_c2, "c5": synthetic.make_c5}[name]


# ---------------------------------------------------------------------------------------------------------------
# CPU baseline (the oracle: test infrastructure, used here only as the reported CPU leg)


def cpu_rate(design, cfg, start_step, budget_s, state):
    """The oracle (fp64, 1 thread, reference flags) on a bounded sample of the same workload (same state):
    one step to size the sample, then as many steps as fit `budget_s`.  Returns (bead-updates/s, steps, s)."""
    from gcs import interphase
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg)
    o.set_schedule(**interphase.interphase_schedule(cfg))
    o.set_positions(state[0])
    o.set_context(state[1])
    t0 = time.perf_counter()
    o.run(1, first_step=start_step, seed=1)
    one = time.perf_counter() - t0
    steps = max(1, min(20000, int(budget_s / max(one, 1e-6))))
    t0 = time.perf_counter()
    o.run(steps, first_step=start_step + 1, seed=1)
    el = time.perf_counter() - t0
    return design.n * steps / el, steps, el


def cpu_worker(budget_s):
    """Child-process entry (`bench.py --cpu-worker S`): one single-threaded oracle trajectory; prints its rate."""
    from gcs import synthetic
    from gcs.config import InterphaseConfig
    r, steps, el = cpu_rate(synthetic.make_c2(master_seed=1), InterphaseConfig(), WINDOW_START, budget_s, load_state())
    print(json.dumps({"value": r, "steps": steps, "seconds": el}), flush=True)


def cpu_baseline(budget_s, procs):
    """cpu_baseline of the bench line.  value: ONE oracle process on one core (the reference is single-threaded);
    `replicas_value`: `procs` independent single-threaded trajectories side by side, aggregate.
    Both legs run as child processes that never touch the device."""

    cpus = cpu_share(procs)

    def launch(k):
        env = dict(os.environ, OMP_NUM_THREADS="1")
        out = []
        for q in range(k):
            # pinned one per core (taskset -c <cpu>): the legs never share a core, so the aggregate is k cores' worth
            cmd = [sys.executable, str(ROOT / "bench.py"), "--cpu-worker", str(budget_s)]
            if shutil.which("taskset"):
                cmd = ["taskset", "-c", str(cpus[q % len(cpus)])] + cmd
            out.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env))
        return out

    def collect(ps):
        out = []
        for p in ps:
            so, _ = p.communicate()
            if p.returncode != 0:
                raise RuntimeError(f"cpu baseline worker failed (rc {p.returncode})")
            out.append(json.loads(so.strip().splitlines()[-1]))
        return out

    one = collect(launch(1))[0]
    res = {"value": one["value"], "unit": "bead-updates/s", "cores": 1, "kind": "port",
           "sample": f"C2 60662 particles from the bench state, {one['steps']} steps from step {WINDOW_START + 1} "
                     f"({one['seconds']:.1f} s, oracle/libgcs_oracle.so fp64 single thread, "
                     f"-O2 -funsafe-math-optimizations)",
           "cpu_model": _cpu_model()}
    if len(cpus) > 1:
        many = collect(launch(len(cpus)))
        res["replicas_value"] = sum(m["value"] for m in many)
        res["replicas_cores"] = len(cpus)
        res["replicas_cpus"] = cpus
        res["replicas_sample"] = (f"{len(cpus)} independent single-threaded oracle trajectories run side by side, "
                                  f"each pinned to its own core (taskset -c), "
                                  f"{min(m['steps'] for m in many)}-{max(m['steps'] for m in many)} steps each")
    return res


def cpu_share(limit):
    """The cores this process may use (its affinity set; SURVEY 8d (ii) `nproc`), at most `limit` (the GPU box's CPU
    share is 16 cores per GPU, while its affinity set may show the whole machine)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    return cpus[:max(1, limit)]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


STEP_KERNEL = {(3, 64): ("k_lstep<..., double>", "pmc_lstep64_traffic.json"),
               (3, 32): ("k_lstep<..., float>", "pmc_lstep_traffic.json"),
               (2, 32): ("k_force<kModeStep, FUSED>", "pmc_force_traffic.json"), (0, 32): ("k_force<kModeStep>", None)}


def read_traffic(fused=3, precision=64):
    """The committed rocprofv3 record of the step's dominant kernel (profiles/): HBM bytes per launch from the PMC
    passes (2 x FETCH_SIZE + WRITE_SIZE: reads and writes) and the kernel-trace average duration of the same run."""
    name = STEP_KERNEL.get((fused, precision), (None, None))[1]
    if name is None:
        return None
    p = ROOT / "profiles" / name
    if p.exists():
        try:
            return json.loads(p.read_text())
        except Exception:
            return None
    return None


# ---------------------------------------------------------------------------------------------------------------
# secondary legs of the default line: C5 on one GPU, the C3 cell cycle


def c5_leg(local, seed, steps, precision=64, log=sys.stderr):
    """C5 (606,248 particles, BASELINE configs[4]'s system) as ONE trajectory on this GPU, from its synthetic start
    (step 0, core_scale 0.5 and growing; gcs.config.resolution_scaled force field): the fp64 engine (its list step),
    and the fp32 engine's default step and explicit step shapes (list step, 2-launch rebuild step, 6-launch unfused
    tile step), each warmed by 64 steps (graphs captured)."""
    from gcs import _abi as A
    from gcs import synthetic
    cfg = bench_config("c5")
    d = synthetic.make_c5(master_seed=1)
    bd = {"temperature": cfg.temperature, "timestep": cfg.timestep, "seed": seed}
    out = {"particles": d.n, "window": f"steps 64..{64 + steps} from the synthetic start", "steps": steps}
    legs = [("default", None, precision)] + [(f"f32_{n}", f, 32) for n, f in
                                              (("default", None), ("list_step", 3), ("rebuild_step", 2),
                                               ("unfused_tile_step", 0))]
    for name, fused, prec in legs:
        e = make_engine(d, cfg, local, 0, precision=prec)
        if fused is not None:
            e.set_option(A.OPT_FUSED_STEP, fused)
        e.run(64, first_step=0, **bd)
        e.synchronize()
        t0 = time.perf_counter()
        e.run(steps, first_step=64, **bd)
        e.synchronize()
        out[name] = d.n * steps / (time.perf_counter() - t0)
        if name == "default":
            # the same trajectory over the next 8 x `steps` steps: past the synthetic start's densest stretch (the
            # particles spread, the core scale grows), closer to what a production run sees on average
            t0 = time.perf_counter()
            e.run(8 * steps, first_step=64 + steps, **bd)
            e.synchronize()
            out["default_long"] = d.n * 8 * steps / (time.perf_counter() - t0)
            out["default_long_window"] = f"steps {64 + steps}..{64 + 9 * steps}"
        if name.endswith("default"):
            # the engine's density verdict (fp32, GCS_OPT_DENSE_NEIGHBORS): list step, or the unfused tile step when
            # dense; the fp64 engine runs the list step
            out[name + "_step"] = "list" if e.list_stats()["active"] else "unfused tile (dense start)"
        e.close()
        print(f"bench: C5 {name} {out[name]:.3e} bead-updates/s", file=log, flush=True)
    return out


def cycle_leg(local, scale, log=sys.stderr):
    """C3 (BASELINE configs[2]): one interphase -> mitosis -> interphase cell cycle of the synthetic C2 genome
    through the stage entry points and the HDF5 store (gcs.cli, as scripts/simulate:44-47 runs the reference's
    executables): prepare -> anatelophase (anaphase + telophase, 586 particles) -> transition interphase ->
    interphase (relaxation + simulation with the contact map, 60,662) -> transition prometaphase -> prometaphase
    (1,172) -> transition cycle into the daughter's file.  Step counts are the reference defaults
    (common/simulation_config.hpp:15-115) divided by `scale`; the sampling/logging/contact cadence is the
    reference's.  Each stage's wall time includes its engine setup and host work (HDF5 frames, energies, contacts)."""
    import tempfile
    from gcs import cli, mitotic, synthetic
    from gcs.config import SimulationConfig
    cfg = SimulationConfig()
    m, ip = cfg.mitotic_phase, cfg.interphase
    steps = {"anaphase": m.anaphase_steps // scale, "telophase": m.telophase_steps // scale,
             "relaxation": ip.relaxation_steps // scale, "interphase": ip.steps // scale,
             "prometaphase": m.prometaphase_steps // scale}
    d = synthetic.make_c2(master_seed=1)
    a = mitotic.anatelophase_design(d, m)
    pm = mitotic.prometaphase_design(a, m, 1)
    dev = ["--device", str(local), "--quiet"]
    out = {"scale": f"reference step counts / {scale}", "steps": steps,
           "particles": {"anatelophase": a.n, "interphase": d.n, "prometaphase": pm.n}, "stages": {}}
    with tempfile.TemporaryDirectory() as td:
        p, q = str(Path(td) / "mother.h5"), str(Path(td) / "daughter.h5")
        calls = [
            ("prepare", ["prepare-synthetic", p, "--config", "c2", "--master-seed", "1"], 0, 0),
            ("anatelophase", ["anatelophase", p, "--anaphase-steps", str(steps["anaphase"]), "--telophase-steps",
                              str(steps["telophase"])] + dev, steps["anaphase"] + steps["telophase"], a.n),
            ("transition_interphase", ["transition", "interphase", p], 0, 0),
            ("interphase", ["interphase", p, "--relaxation-steps", str(steps["relaxation"]), "--steps",
                            str(steps["interphase"])] + dev, steps["relaxation"] + steps["interphase"], d.n),
            ("transition_prometaphase", ["transition", "prometaphase", p], 0, 0),
            ("prometaphase", ["prometaphase", p, "--steps", str(steps["prometaphase"])] + dev,
             steps["prometaphase"], pm.n),
            ("prepare_daughter", ["prepare-synthetic", q, "--config", "c2", "--master-seed", "2"], 0, 0),
            ("transition_cycle", ["transition", "cycle", p, q], 0, 0),
        ]
        total = 0.0
        for name, argv, nsteps, n in calls:
            t0 = time.perf_counter()
            cli.main(argv)
            el = time.perf_counter() - t0
            total += el
            rec = {"wall_s": el}
            if nsteps:
                rec.update(steps=nsteps, particles=n, steps_per_s=nsteps / el, bead_updates_per_s=n * nsteps / el)
            out["stages"][name] = rec
            print(f"bench: cycle {name} {el:.2f} s", file=log, flush=True)
    out["cycle_wall_s"] = total
    return out


# ---------------------------------------------------------------------------------------------------------------
# decomposed single trajectory (C5)


def decomp_main(args):
    """One trajectory split into recursive-bisection boxes (gcs.domain.plan_boxes, 2 x 2 x 2 at 8; --slabs: z-slabs;
    C5 of SURVEY 8e).  value = N x steps / max-over-ranks time of the whole decomposed step loop (the decomposed list
    step: forces, update, reaction allreduce, band exchange, list rebuilds).  Under torchrun: one
    domain per GPU, the engine issues the RCCL collectives itself (gcs.domain.RcclRun); one process: K domains on
    this GPU, bands moved device-to-device (LocalTransport)."""
    from gcs import _abi as A
    from gcs import domain as D
    world, rank, local, dist = dist_setup()
    A.load()
    cfg = bench_config(args.config)
    state = load_state() if args.config == "c2" else None
    design = design_maker(args.config)(master_seed=1)
    ndom = world if world > 1 else args.decomp
    halo = D.domain_halo(cfg)
    x0 = state[0] if state is not None else design.positions
    boxes = D.plan_slabs(x0[:, 2], ndom) if args.slabs else D.plan_boxes(x0, ndom)
    mine = [rank] if world > 1 else list(range(ndom))
    doms = []
    window = window_start(args.config)
    cap = max(D.band_capacity(x0, boxes, halo, d) for d in range(ndom))  # one size: bands move between domains
    for d in mine:
        e = make_engine(design, cfg, local, window, state, precision=args.precision)
        if args.fused is not None:
            e.set_option(A.OPT_FUSED_STEP, args.fused)  # e.g. 0: the decomposed tile step (fp32)
        doms.append(D.EngineDomain(e, d, boxes, halo, cap=cap, shared=D.shared_particles(design)))
    rccl = world > 1 or (args.rccl and ndom == 1)
    run = D.RcclRun(doms[0], dist) if rccl else D.DecomposedRun(doms, D.LocalTransport(doms))
    seed = replica_noise_seed(0)
    run.run(args.warmup, first_step=window, seed=seed, timestep=cfg.timestep)
    for d in doms:
        d.synchronize()
    barrier(dist)
    t0 = time.perf_counter()
    run.run(args.steps, first_step=window + args.warmup, seed=seed, timestep=cfg.timestep)
    for d in doms:
        d.synchronize()
    el = time.perf_counter() - t0
    barrier(dist)
    el_max = max_over_ranks(dist, el)
    run.check()
    n = design.n
    ref = None
    if world == 1:
        # the same trajectory undecomposed (one engine, same window, steps and shape): what the decomposition costs
        e = make_engine(design, cfg, local, window, state, precision=args.precision)
        if args.fused is not None:
            e.set_option(A.OPT_FUSED_STEP, args.fused)
        e.run(args.warmup, first_step=window, seed=seed, timestep=cfg.timestep)
        e.synchronize()
        t0 = time.perf_counter()
        e.run(args.steps, first_step=window + args.warmup, seed=seed, timestep=cfg.timestep)
        e.synchronize()
        ref = n * args.steps / (time.perf_counter() - t0)
        e.close()
    if rank == 0:
        line = {
            "metric": "bead-updates/sec (whole node), decomposed single trajectory",
            "value": n * args.steps / el_max, "unit": "bead-updates/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el_max * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64" if args.precision == 64 else "f32",
            "data": "synthetic",
            "config": {"workload": f"{args.config.upper()} interphase BD step, {n} particles, one trajectory in "
                                   f"{ndom} {'z-slab' if args.slabs else 'box'} domains "
                                   f"({'RCCL from the engine' if rccl else 'in-process, one GPU'})",
                       "particles": n, "domains": ndom, "halo": halo, "parallelism": f"domains{ndom}",
                       "band_capacity_rank0": doms[0].cap, "peers_rank0": doms[0].peers,
                       "bytes_per_peer_per_step": (32 if args.precision == 64 else 16) * (doms[0].cap + 1),
                       "step_shape": "list" if doms[0].e.list_stats()["builds"] > 0 else "tile",
                       "undecomposed_value": ref,
                       "decomposed_over_undecomposed": (n * args.steps / el_max / ref) if ref else None},
        }
        print(json.dumps(line), flush=True)
    for d in doms:
        d.e.close()  # RCCL communicators go with their engines
    if dist is not None:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------------------------------------
# replicas (C2 / C4): the headline


def f32_leg(args, maker, cfg, bd, local, state, window, R, K, G, list_waves, rank, log=sys.stderr):
    """The fp32 engine on the headline's workload (same window, replicas, options), timed the same way for about half
    the headline's window: the rate the fp32 arithmetic buys (a secondary line item, not the headline)."""
    from gcs import _abi as A
    engines, seeds, nxt = [], [], []
    for k in range(R):
        rid = rank * R + k
        d = maker(master_seed=1 if state is not None else replica_master_seed(rid))
        e = make_engine(d, cfg, local, window, state, precision=32)
        e.set_option(A.OPT_GRAPH_STEPS, G)
        e.set_option(A.OPT_LIST_WAVES, list_waves)
        engines.append(e)
        seeds.append(replica_noise_seed(rid))
        nxt.append(window)
    n = engines[0].n

    def enqueue_all(steps):
        chunk = G if G > 0 else 64
        for s0 in range(0, steps, chunk):
            c = min(chunk, steps - s0)
            for k, (e, sd) in enumerate(zip(engines, seeds)):
                e.run(c, first_step=nxt[k], seed=sd, **bd)
                nxt[k] += c

    def sync_all():
        for e in engines:
            e.synchronize()

    for _ in range(3):
        enqueue_all(K)
    sync_all()
    t0 = time.perf_counter()
    enqueue_all(K)
    sync_all()
    per_pass = time.perf_counter() - t0
    passes = max(1, math.ceil(0.5 * args.min_window_s / max(per_pass, 1e-9)))
    t0 = time.perf_counter()
    for _ in range(passes):
        enqueue_all(K)
    sync_all()
    value = n * R * passes * K / (time.perf_counter() - t0)
    prof = engines[0].profile(args.profile_steps, first_step=nxt[0], seed=seeds[0], **bd)
    for e in engines:
        e.close()
    print(f"bench: f32 engine {value:.3e} bead-updates/s ({R} trajectories)", file=log, flush=True)
    return {"value": value, "replicas_per_gpu": R, "steps": passes * K, "k_lstep_ms": prof["force_ms"],
            "roofline_frac": n * BYTES_PER_UPDATE[32] / (prof["force_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS}


def replica_main(args):
    world, rank, local, dist = dist_setup()
    if os.environ.get("GCS_BENCH_FAIL_RANK") == str(rank):  # launcher tests: this rank dies before the first barrier
        print(f"bench: rank {rank} failing on purpose (GCS_BENCH_FAIL_RANK)", file=sys.stderr, flush=True)
        os._exit(3)
    if not args.stub_engine:
        from gcs import _abi as A
        A.load()  # this rank's engine runtime (no torch HIP runtime in replica runs)
    cfg = bench_config(args.config)
    bd = {"temperature": cfg.temperature, "timestep": cfg.timestep}  # md::brownian_dynamics_config of the stage
    maker = design_maker(args.config)
    R = max(1, args.replicas_per_gpu)
    K = max(1, args.steps)
    # list step: 2 waves per tile when trajectories share the GPU (twice the tiles resident; the other replicas'
    # launches fill the latency), 4 for a trajectory alone (the lowest step latency)
    list_waves = args.list_waves or (2 if R > 1 else 4)
    # graph chunk: a pass of K steps per replica is replayed in G-step hipGraphs (G <= K, so short passes replay
    # graphs too); warm-up captures and instantiates every engine's graph before the timed region
    G = min(args.graph_steps, K) if args.graph_steps > 0 else 0
    warm = max(args.warmup, 2 * G, 1)

    # R independent trajectories per GPU (own noise seed, own engine and HIP stream each).  Rank r owns
    # replicas r*R .. r*R + R - 1, so every trajectory of the job has its own seeds.  C2: every replica continues
    # the committed step-300,000 state of the master-seed-1 system with its own noise seed
    # (tools/make_bench_state.py); other configs start from their synthetic state at the window's context
    state = load_state() if args.config == "c2" and not args.stub_engine else None
    window = window_start(args.config)
    # the fp32 leg first, before this process has created any other stream: HIP hands streams the hardware queues
    # (4 per process here) in creation order, and measured after the headline's engines and the secondary legs its
    # 4 trajectories shared queues (4.2e9 against 6.44e9 for the same workload as the headline of its own process)
    f32 = None
    if world == 1 and not args.stub_engine and args.precision == 64 and args.f32_leg:
        f32 = f32_leg(args, maker, cfg, bd, local, state, window, R, K, G, list_waves, rank)
    designs, engines, seeds = [], [], []
    for k in range(R):
        rid = rank * R + k
        d = maker(master_seed=1 if state is not None else replica_master_seed(rid))
        if args.stub_engine:
            e = StubEngine(d.n)
        else:
            from gcs import _abi as A
            e = make_engine(d, cfg, local, window, state, precision=args.precision)
            opts = [(A.OPT_GRAPH_STEPS, G), (A.OPT_SCAN_BLOCKS, args.scan_mb), (A.OPT_LIST_WAVES, list_waves)]
            if args.stagger and R > 1:
                # the replicas' list rebuilds staggered over the period (C2: every 8 steps -> phases 0, 2, 4, 6 at
                # R = 4), so one replica's short cell kernels and list build overlap the others' step kernels
                opts.append((A.OPT_LIST_PHASE, (8 * k) // R))
            if args.precision == 32:  # the fp32 engine's tile-step shapes and their options
                opts += [(A.OPT_WAVES_PER_TILE, args.waves), (A.OPT_CHUNK_ORDER, args.chunk_order),
                         (A.OPT_FUSED_STEP, args.fused), (A.OPT_SPLIT_TILES, args.split),
                         (A.OPT_TILE_PRIORITY, args.prio), (A.OPT_SUBTILES, args.subtiles)]
            for opt, v in opts:
                e.set_option(opt, v)
            apply_engine_opts(e, args)
            if args.cu_split and R > 1:
                # replica k on CUs c with (c mod R) == k ("interleave") or a contiguous R-th of them ("block")
                ncu = args.cu_count
                cus = ([c for c in range(ncu) if c % R == k] if args.cu_split == "interleave"
                       else list(range(k * ncu // R, (k + 1) * ncu // R)))
                e.set_cu_mask(cus)
        designs.append(d)
        engines.append(e)
        seeds.append(replica_noise_seed(rid))
    design, eng, seed = designs[0], engines[0], seeds[0]
    n = design.n
    nxt = [window] * R  # next step of every replica (host-side: no device round trip in the timed loop)

    def enqueue_all(steps):
        """`steps` steps of every replica, enqueued interleaved chunk by chunk so their graphs run side by side
        (no host synchronisation: the engines' run calls only enqueue)"""
        chunk = G if G > 0 else 64
        for s0 in range(0, steps, chunk):
            c = min(chunk, steps - s0)
            for k, (e, sd) in enumerate(zip(engines, seeds)):
                e.run(c, first_step=nxt[k], seed=sd, **bd)
                nxt[k] += c

    def sync_all():
        for e in engines:
            e.synchronize()

    def run_stats():
        if not hasattr(eng, "run_stats"):
            return {}
        tot = {}
        for e in engines:
            for k, v in e.run_stats().items():
                tot[k] = tot.get(k, 0) + v
        return tot

    # warm-up: passes of exactly the timed region's shape, so every graph the timed passes replay (one per rebuild
    # phase, starting parity and length, gcs_engine_get_run_stats) is captured and instantiated before timing
    # (3 passes at least: the first pass of a run starts with an eager forced rebuild, which shifts its graphs by a
    # step, so the timed passes' first shape appears in the warm-up's second pass at the earliest)
    warm_passes = max(3, math.ceil(warm / K))
    if os.environ.get("GCS_MAPS_OUT"):  # (diagnostics) this process's mappings before its first graph launch
        with open("/proc/self/maps") as src, open(os.environ["GCS_MAPS_OUT"], "w") as dst:
            dst.write(src.read())
    enqueue_all(K)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(warm_passes - 1):
        enqueue_all(K)
    sync_all()
    per_pass = (time.perf_counter() - t0) / (warm_passes - 1)

    # one trajectory alone on the GPU (replica 0; the others are independent and idle meanwhile), its own window
    single_rate = None
    if R > 1 and rank == 0:
        k1 = G if G > 0 else 64
        eng.run(k1, first_step=nxt[0], seed=seed, **bd)  # (graph already instantiated by the warm-up)
        eng.synchronize()
        nxt[0] += k1
        reps = 0
        t1 = time.perf_counter()
        while True:  # >= half the headline window, in blocks of 8 graph replays
            eng.run(k1, first_step=nxt[0], seed=seed, **bd)
            nxt[0] += k1
            reps += 1
            if reps % 8 == 0:
                eng.synchronize()
                el1 = time.perf_counter() - t1
                if el1 >= 0.5 * args.min_window_s:
                    break
        single_rate = n * k1 * reps / el1

    # passes of K steps so the timed window lasts >= min_window_s (estimated from the warm-up, agreed by all ranks)
    # (x 1.25: the warm-up's pass estimate runs a little slow, so the window still lasts min_window_s)
    passes = max(1, math.ceil(1.25 * args.min_window_s / max(per_pass, 1e-9)))
    passes = int(max_over_ranks(dist, float(passes)))
    barrier(dist)
    sync_all()
    rs0 = run_stats()
    t0 = time.perf_counter()
    for _ in range(passes):
        enqueue_all(K)
    sync_all()
    el = time.perf_counter() - t0
    rs1 = run_stats()
    timed_runs = {k: rs1[k] - rs0.get(k, 0) for k in rs1 if k != "graphs_cached"}
    barrier(dist)
    steps = passes * K
    el_max = max_over_ranks(dist, el)
    rank_values = gather_over_ranks(dist, n * R * steps / el)
    rank_seeds = gather_over_ranks(dist, float(seed))  # every rank's first trajectory's noise seed (all distinct)
    after = nxt[0]

    # per-kernel durations with HIP events on the engine's stream (replica 0 alone, after the timed region)
    prof = eng.profile(args.profile_steps, first_step=after, seed=seed, **bd)
    force_ms = prof["force_ms"]
    bpu = BYTES_PER_UPDATE[args.precision]
    achieved = n * bpu / (force_ms * 1e-3) / 1e9
    tr = read_traffic(args.fused, args.precision)
    ctx = eng.get_context()
    lst = eng.list_stats() if hasattr(eng, "list_stats") else None
    if lst is not None:  # the list step's rebuild cadence and exact-search fallbacks (DESIGN.md "The list step")
        lst = {k: lst[k] for k in ("active", "rebuild_every", "skin", "builds", "fallback_particle_steps",
                                   "pair_classes", "capacity")}
    finite = all(bool(np.isfinite(e.get_positions()).all()) for e in engines)
    # every rank's trajectories: all finite, and a position checksum of its first one (distinct seeds: distinct sums)
    rank_finite = gather_over_ranks(dist, 1.0 if finite else 0.0)
    rank_sums = gather_over_ranks(dist, float(np.asarray(engines[0].get_positions(), dtype=np.float64).sum()))
    at = after + args.profile_steps
    rank_steps = gather_over_ranks(dist, float(at))  # the step each rank's checksum was taken at

    contacts_ms, contacts_distinct = None, None
    start_rate = None
    if not args.stub_engine:
        # secondary (off the step metric): the contact-map update (contact_map.cpp:33-63) that
        # production runs every 20 steps, measured as the extra time of 20-step chunks with an update after each
        # (the update then reads the engine's own cell list, as in production)
        dcon = cfg.contactmap_distance * ctx["core_scale"]

        def chunks(k, with_update):
            nonlocal at
            eng.synchronize()
            t1 = time.perf_counter()
            for _ in range(k):
                eng.run(20, first_step=at, seed=seed, **bd)
                at += 20
                if with_update:
                    eng.contacts_update(dcon)
            eng.synchronize()
            return time.perf_counter() - t1

        chunks(2, True)
        base = chunks(20, False)
        withc = chunks(20, True)
        contacts_ms = max(0.0, (withc - base) * 1e3 / 20)
        contacts_distinct = int(eng.contacts_accumulate().shape[0])
        eng.contacts_clear()

        # secondary: the production start window (step 0, core_scale 0.5, ~7x fewer neighbours), one replica
        if rank == 0 and not args.no_start_window:
            e0 = make_engine(design, cfg, local, 0, precision=args.precision)
            e0.set_option(A.OPT_GRAPH_STEPS, G)
            apply_engine_opts(e0, args)
            e0.run(max(64, 2 * G), first_step=0, seed=seed, **bd)
            e0.synchronize()
            k0 = max(256, K // 4)
            t1 = time.perf_counter()
            e0.run(k0, first_step=max(64, 2 * G), seed=seed, **bd)
            e0.synchronize()
            start_rate = n * k0 / (time.perf_counter() - t1)
            e0.close()

    if rank != 0:
        for e in engines:
            e.close()
        if dist is not None:
            dist.destroy_process_group()
        return
    for e in engines[1:]:
        e.close()  # (replica 0 stays for the line's context)

    c5 = cycle = None
    if world == 1 and not args.stub_engine:
        if args.c5_steps > 0:
            c5 = c5_leg(local, seed, args.c5_steps, args.precision)
        if args.cycle_scale > 0:
            cycle = cycle_leg(local, args.cycle_scale)

    cpu = None  # (rank 0 at any world size: the line of an 8-GPU run carries its CPU leg too)
    if args.cpu_budget > 0 and state is not None and args.config == "c2":
        cpu = cpu_baseline(args.cpu_budget, args.cpu_procs)

    value = whole_job_value(n * R, steps, world, el_max)
    line = {
        "metric": "bead-updates/sec (whole node), 60k-bead diploid interphase",
        "value": value,
        "unit": "bead-updates/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": el_max * 1e3 / steps,  # one step of every replica
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == 64 else "f32",
        "data": "synthetic" if not args.stub_engine else "stub",
        "steps_requested": K,
        "passes": passes,
        "warmup_steps_run": warm_passes * K,
        "graph_replays": timed_runs.get("graph_launches"),
        "timed_runs": timed_runs,
        "timed_s": el_max,
        "per_rank_values": rank_values,
        "per_rank_seeds": rank_seeds,
        "per_rank_finite": rank_finite,
        "per_rank_checksums": rank_sums,
        "per_rank_checksum_steps": rank_steps,
        "window_start": window,
        "config": {"workload": f"{args.config.upper()} interphase BD step, {n} particles, {R} independent "
                               f"trajectories per GPU, window from step {window} "
                               f"(core_scale {ctx['core_scale']:.4f})",
                   "particles": n, "replicas": world * R, "replicas_per_gpu": R,
                   "parallelism": f"replicas{world}x{R}",
                   "single_trajectory_value": single_rate if R > 1 else value,
                   "mean_neighbors": prof["mean_neighbors"], "graph_steps": G,
                   "waves_per_tile": args.waves, "chunk_order": args.chunk_order, "fused": args.fused,
                   "split_tiles": args.split, "tile_priority": args.prio, "subtiles": args.subtiles,
                   "scan_mb": args.scan_mb, "start_window_value": start_rate, "finite": finite,
                   "contacts_update_ms": contacts_ms, "contacts_distinct_pairs_22_updates": contacts_distinct,
                   "list_step": lst, "list_waves_per_tile": list_waves,
                   "c5_value": c5["default"] if c5 else None, "c5": c5,
                   "c3_cycle_wall_s": cycle["cycle_wall_s"] if cycle else None, "c3_cycle": cycle,
                   "precision": args.precision, "f32_value": f32["value"] if f32 else None, "f32": f32},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": tr.get("bytes_per_launch") if tr else None,
                     "kernel": STEP_KERNEL.get((args.fused, args.precision), ("?",))[0], "force_ms": force_ms,
                     "cell_ms": prof["cell_ms"], "tail_ms": prof["tail_ms"], "bytes_per_launch": n * bpu,
                     "bytes_per_update": bpu,
                     # the same accounting on the committed rocprofv3 kernel trace (profiles/, R = 1 bench)
                     "rocprof_avg_us": tr.get("avg_us") if tr else None,
                     "frac_rocprof": (n * bpu / (tr["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS)
                     if tr and tr.get("avg_us") else None,
                     "traffic_source": tr.get("source") if tr else None},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000, help="steps per replica per timed pass")
    ap.add_argument("--warmup", type=int, default=200, help="untimed steps per replica (at least 2 graph chunks)")
    ap.add_argument("--min-window-s", type=float, default=0.5,
                    help="the timed region repeats passes of --steps until it lasts this long")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c5"])
    ap.add_argument("--precision", type=int, default=64, choices=[32, 64],
                    help="engine arithmetic: 64 (default; the reference's double) or 32")
    ap.add_argument("--no-f32-leg", dest="f32_leg", action="store_false",
                    help="skip the secondary fp32-engine window of an fp64 run")
    ap.add_argument("--graph-steps", type=int, default=32)
    ap.add_argument("--waves", type=int, default=4)
    ap.add_argument("--chunk-order", type=int, default=1)
    ap.add_argument("--split", type=int, default=0, help="0 off, 1 split every tile over two workgroups, 2 the heavy tiles")
    ap.add_argument("--prio", type=int, default=700, help="n > 0: wave priority min(3, tile candidates / n)")
    ap.add_argument("--subtiles", type=int, default=2, help="pair-loop stencils per 64-particle tile: 1, 2, 4")
    ap.add_argument("--scan-mb", type=int, default=1, help="1: multi-block look-back cell scan, 0: one workgroup")
    ap.add_argument("--cu-split", default="", choices=["", "interleave", "block"],
                    help="several replicas per GPU: give each its own share of the compute units")
    ap.add_argument("--cu-count", type=int, default=256)
    ap.add_argument("--engine-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="extra engine option (gcs._abi OPT_<NAME>), repeatable; for experiments")
    ap.add_argument("--stagger", action="store_true",
                    help="several replicas per GPU: stagger their list rebuilds over the period (GCS_OPT_LIST_PHASE; "
                         "measured no faster, profiles/r06_stagger_ab.txt)")
    ap.add_argument("--list-waves", type=int, default=0,
                    help="list step waves per tile: 2 or 4 (0: 2 with several replicas per GPU, else 4)")
    ap.add_argument("--fused", type=int, default=3,
                    help="3: list step (default); fp32 engines only: 2 the 2-launch rebuild step, 0 unfused")
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--replicas-per-gpu", type=int, default=4,
                    help="independent trajectories per GPU, each its own engine + stream (1 = single trajectory)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="independent single-threaded CPU trajectories for the multi-core leg (the box's CPU share)")
    ap.add_argument("--cpu-worker", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--stub-engine", action="store_true", help=argparse.SUPPRESS)  # CPU tests of the launcher
    ap.add_argument("--no-start-window", action="store_true", help="skip the secondary step-0 window")
    ap.add_argument("--c5-steps", type=int, default=256, help="secondary C5 window per step shape (0 = skip)")
    ap.add_argument("--cycle-scale", type=int, default=1,
                    help="secondary C3 cell cycle at the reference step counts / this (1: as configured; 0 = skip)")
    ap.add_argument("--decomp", type=int, default=0,
                    help="spatial domain decomposition of ONE trajectory: K domains (torchrun: one per rank over "
                         "RCCL; single process: K domains on this GPU, in-process exchange)")
    ap.add_argument("--slabs", action="store_true", help="--decomp: z-slabs instead of recursive-bisection boxes")
    ap.add_argument("--rccl", action="store_true",
                    help="--decomp 1 in one process: the engine-issued RCCL sequence with one rank (graph-captured)")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.cpu_worker is not None:
        cpu_worker(args.cpu_worker)
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv)  # launcher only: no device call in this process
    if args.decomp:
        decomp_main(args)
        return 0
    replica_main(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
