"""The persistent small-system step (k_pstep) against the list step on the C3 mitotic systems, one GPU: steps/s of
the engine alone (run() of `chunk` steps, synchronized) and through the anatelophase / prometaphase drivers.
usage: python tools/small_probe.py [steps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import _abi as A, mitotic, synthetic  # noqa: E402
from gcs.config import MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
cfg = MitoticPhaseConfig()
d = synthetic.make_c2()
a = mitotic.anatelophase_design(d, cfg)
p = mitotic.prometaphase_design(a, cfg, d.master_seed)
for stage, design, build in (("anatelophase", a, mitotic.build_anatelophase),
                             ("prometaphase", p, mitotic.build_prometaphase)):
    for small in (1, 0):
        for prec in (64, 32):
            s, h = build(Engine, design, cfg, precision=prec)
            s.set_option(A.OPT_SMALL_STEP, small)
            if stage == "anatelophase":
                mitotic.AnatelophaseDriver(s, h, design, cfg, log=None).run_initialization()
            else:
                import numpy as np
                s.set_positions(np.random.default_rng(1).normal(scale=2.0, size=(design.n, 3)))
            bd = dict(temperature=cfg.temperature, timestep=cfg.timestep, seed=3)
            s.run(2000, **bd)
            s.synchronize()
            for chunk in (1000, steps):
                t0 = time.perf_counter()
                done = 0
                while done < steps:
                    s.run(chunk, first_step=2000 + done, **bd)
                    done += chunk
                s.synchronize()
                el = time.perf_counter() - t0
                print(f"{stage:13s} n {design.n:5d} fp{prec} small {small} chunk {chunk:6d}: {steps / el:10.0f} steps/s "
                      f"({1e6 * el / steps:6.2f} us/step)", flush=True)
            s.close()
# the anatelophase driver (sampling every 1000 steps, energy log every 1000) as the C3 cycle runs it, minus the store
for small in (1, 0):
    s, h = mitotic.build_anatelophase(Engine, a, cfg, precision=64)
    s.set_option(A.OPT_SMALL_STEP, small)
    drv = mitotic.AnatelophaseDriver(s, h, a, cfg, log=open("/dev/null", "w"))
    drv.run_initialization()
    t0 = time.perf_counter()
    drv.run_dragging_stage(steps)
    s.synchronize()
    el = time.perf_counter() - t0
    print(f"anaphase driver small {small}: {steps / el:10.0f} steps/s", flush=True)
# phase stamps of workgroup 0 (GCS_DEBUG_PSTEP): us from the step start, medians over 63 steps
import os
import numpy as np
dbg = str(ROOT / "gpurun_out" / "pstep_times.bin")
os.environ["GCS_DEBUG_PSTEP"] = dbg
for stage, design, build in (("anatelophase", a, mitotic.build_anatelophase), ("prometaphase", p, mitotic.build_prometaphase)):
    s, h = build(Engine, design, cfg, precision=64)
    if stage == "anatelophase":
        mitotic.AnatelophaseDriver(s, h, design, cfg, log=None).run_initialization()
    else:
        s.set_positions(np.random.default_rng(1).normal(scale=2.0, size=(design.n, 3)))
    s.run(64, temperature=cfg.temperature, timestep=cfg.timestep, seed=3)
    s.synchronize()
    raw = np.fromfile(dbg, dtype=np.uint64).astype(np.int64)
    S = 32
    t = raw[:16 * S].reshape(S, 16)
    us = lambda j: np.median((t[1:S - 1, j] - t[1:S - 1, 0]) / 100.0)
    step = np.median((t[2:S, 0] - t[1:S - 1, 0]) / 100.0)
    print(f"{stage}: step {step:.2f} us; local terms done {us(1):.2f}, wave 0 prefilter {us(8):.2f}, pairs done "
          f"{us(2):.2f}/{us(9):.2f}/{us(10):.2f}/{us(11):.2f} (waves 0-3), sums {us(13):.2f}, stored "
          f"{us(14):.2f}, handed off {us(3):.2f}, first poll back {us(4):.2f} (retries {np.median(t[1:S - 1, 5]):.0f}), image in {us(12):.2f}, totals {us(7):.2f}, tail done {us(6):.2f}", flush=True)
    g = (design.n + 15) // 16
    w = raw[1024:1024 + 128 * S].reshape(S, 128)[1:S - 1, :g]
    late = np.median((w - t[1:S - 1, 0:1]) / 100.0, axis=0)
    print(f"  hand-off by workgroup (median us from wg 0's step start): min {late.min():.2f} max {late.max():.2f} "
          f"slowest wg {int(late.argmax())}; " + " ".join(f"{v:.1f}" for v in late), flush=True)
    s.close()
