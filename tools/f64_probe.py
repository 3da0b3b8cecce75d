"""fp64 engine vs the fp64 oracle, quick numbers (forces, energy, trajectories, spacestep, C2 list step, timing).
usage: python tools/f64_probe.py"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "3d-genome-cycle_amd"), str(ROOT / "oracle"), str(ROOT)]
import numpy as np  # noqa: E402

from gcs import _abi as A, interphase, synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402
import oracle  # noqa: E402

cfg = InterphaseConfig()
c1 = synthetic.make_c1()


def both(design, prec=64):
    e, _ = interphase.build_interphase(Engine, design, cfg, precision=prec)
    o, _ = interphase.build_interphase(oracle.OracleSystem, design, cfg, precision=prec)
    return e, o


for prec in (64, 32):
    e, o = both(c1, prec)
    fe, fo = e.compute_forces(), o.compute_forces()
    print(f"[{prec}] C1 forces max|dF| {np.abs(fe - fo).max():.3e} (max|F| {np.abs(fo).max():.3e})", flush=True)
    te, pe = e.compute_energy()
    to, po = o.compute_energy()
    print(f"[{prec}] C1 energy rel {abs(te - to) / abs(to):.3e} per-kind max {np.abs(pe - po).max():.3e}", flush=True)
    ce, co = e.get_context(), o.get_context()
    print(f"[{prec}] reactions d {np.abs(np.array(ce['inward_reaction']) - co['inward_reaction']).max():.3e}", flush=True)
    steps = 50
    xi = oracle.reference_normals(123, steps * c1.n * 3).reshape(steps, c1.n, 3)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
        s.set_noise(xi)
        s.run(steps, temperature=cfg.temperature, timestep=cfg.timestep, noise=A.NOISE_INJECTED)
    print(f"[{prec}] C1 injected 50 steps max|dx| {np.abs(e.get_positions() - o.get_positions()).max():.3e} "
          f"wall d {np.abs(np.array(e.get_context()['wall_semiaxes']) - o.get_context()['wall_semiaxes']).max():.3e}",
          flush=True)
    e, o = both(c1, prec)
    for s in (e, o):
        s.set_schedule(**interphase.interphase_schedule(cfg))
        s.apply_schedule(0)
        s.run(50, temperature=cfg.temperature, timestep=cfg.timestep, seed=987654321)
    print(f"[{prec}] C1 philox 50 steps max|dx| {np.abs(e.get_positions() - o.get_positions()).max():.3e}", flush=True)
    e, o = both(c1, prec)
    xi = oracle.reference_normals(7, 10 * c1.n * 3).reshape(10, c1.n, 3)
    for s in (e, o):
        s.set_noise(xi)
        s.run(10, temperature=cfg.temperature, timestep=cfg.timestep, spacestep=cfg.relaxation_spacestep,
              noise=A.NOISE_INJECTED)
    print(f"[{prec}] C1 spacestep 10 max|dx| {np.abs(e.get_positions() - o.get_positions()).max():.3e} dt "
          f"{e.get_context()['last_timestep']:.6e} / {o.get_context()['last_timestep']:.6e}", flush=True)
    for d in (0.12, 0.3):
        got = e.search_neighbors(d)
        exp = oracle.search_neighbors(e.get_positions(), d, prec)
        print(f"[{prec}] search d={d}: {got.shape[0]} pairs, equal {np.array_equal(got, exp)}", flush=True)

# C2 from the bench state: list step, fp64, timing
z = np.load(ROOT / "benchdata" / "c2_interphase_step300000.npz", allow_pickle=False)
c2 = synthetic.make_c2(master_seed=1)
ctx = {"step": int(z["step"]), "time": float(z["time"]), "core_scale": float(z["core_scale"]),
       "bond_scale": float(z["bond_scale"]), "wall_semiaxes": [float(v) for v in z["wall_semiaxes"]]}
for prec in (64, 32):
    e, _ = interphase.build_interphase(Engine, c2, cfg, precision=prec)
    e.set_schedule(**interphase.interphase_schedule(cfg))
    e.set_positions(z["positions"])
    e.set_context(ctx)
    st = int(z["step"])
    e.run(64, first_step=st, seed=3)
    e.synchronize()
    t0 = time.perf_counter()
    e.run(640, first_step=st + 64, seed=3)
    e.synchronize()
    el = time.perf_counter() - t0
    print(f"[{prec}] C2 list step {c2.n * 640 / el:.3e} bead-updates/s, stats {e.list_stats()}", flush=True)
    p = e.profile(50, first_step=st + 704, seed=3)
    print(f"[{prec}] C2 profile {p}", flush=True)
    x = e.get_positions()
    print(f"[{prec}] finite {np.isfinite(x).all()}", flush=True)
# fp64 C2 list step vs oracle, 20 steps, injected noise
e, o = both(c2, 64)
xi = oracle.reference_normals(5, 20 * c2.n * 3).reshape(20, c2.n, 3)
for s in (e, o):
    s.set_positions(z["positions"])
    s.set_context(ctx)
    s.set_schedule(**interphase.interphase_schedule(cfg))
    s.set_noise(xi)
    s.run(20, first_step=int(z["step"]), temperature=cfg.temperature, timestep=cfg.timestep, noise=A.NOISE_INJECTED)
print(f"[64] C2 injected 20 steps max|dx| {np.abs(e.get_positions() - o.get_positions()).max():.3e}", flush=True)
