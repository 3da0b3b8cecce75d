"""Host-side costs of the C3 anatelophase stage in a process whose HIP runtime and library are already warm (as in
bench.py's cycle leg): engine + driver calls alone, then the CLI stage (store, design load, frames) under cProfile.
usage: python tools/stage_overhead_probe.py   (writes gpurun_out/stage_overhead.txt)"""
import cProfile
import io
import pstats
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
from gcs import cli, mitotic, synthetic  # noqa: E402
from gcs.config import MitoticPhaseConfig  # noqa: E402
from gcs.engine import Engine  # noqa: E402

cfg = MitoticPhaseConfig()
a = mitotic.anatelophase_design(synthetic.make_c2(), cfg)
warm, _ = mitotic.build_anatelophase(Engine, a, cfg, precision=64)
warm.run(10, temperature=cfg.temperature, timestep=cfg.timestep, seed=1)
warm.synchronize()
warm.close()
T = {}


def t(name, f):
    t0 = time.perf_counter()
    r = f()
    T[name] = T.get(name, 0) + time.perf_counter() - t0
    return r


s, h = t("build", lambda: mitotic.build_anatelophase(Engine, a, cfg, precision=64))
drv = mitotic.AnatelophaseDriver(s, h, a, cfg, log=None)
t("init", drv.run_initialization)
for k in range(25):
    t("run_calls", lambda: s.run(1000, first_step=1000 * k, temperature=cfg.temperature, timestep=cfg.timestep, seed=3))
    t("samples (incl. the steps)", lambda: s.sample_positions(16))
t("close", s.close)
out = [f"engine + driver alone: {({k: round(v * 1e3, 2) for k, v in T.items()})} ms"]
with tempfile.TemporaryDirectory() as td:
    p = str(Path(td) / "m.h5")
    cli.main(["prepare-synthetic", p, "--config", "c2", "--master-seed", "1"])
    argv = ["anatelophase", p, "--anaphase-steps", "10000", "--telophase-steps", "15000", "--quiet"]
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.runcall(cli.main, argv)
    out.append(f"first CLI stage in this process: {time.perf_counter() - t0:.4f} s")
    t0 = time.perf_counter()
    cli.main(argv)
    out.append(f"second CLI stage: {time.perf_counter() - t0:.4f} s")
    buf = io.StringIO()
    pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(18)
    out.append(buf.getvalue())
text = "\n".join(out)
(ROOT / "gpurun_out").mkdir(exist_ok=True)
(ROOT / "gpurun_out" / "stage_overhead.txt").write_text(text)
print(text[:3000])
