"""GPU: the replica path of bench.py with the REAL engine in more than one process (independent
trajectories one per GPU; the reference's ensemble is `scripts/simulate -s <seed>` runs, scripts/simulate:15-17).

`bench.py --gpus 2` without WORLD_SIZE starts two ranks (gloo on 127.0.0.1 for the barrier and the max-over-ranks
time); GCS_BENCH_SAME_DEVICE=1 puts both on device 0 of this one-GPU box (each rank its own process, HIP runtime,
engine and stream).  Checked: one JSON line from rank 0, every rank's rate present and positive, distinct noise seeds,
every rank's trajectories finite with distinct position checksums, the whole-job value = all ranks' bead-updates over
the slowest rank's time, fp64 arithmetic.  2 ranks, and 8 (C4's 8-trajectory ensemble shape)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ranks", [2, 8])
def test_bench_real_engine_ranks_on_one_device(ranks):
    """2 ranks, and C4's ensemble shape: 8 independent trajectories, one per rank (here all on device 0)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["GCS_BENCH_SAME_DEVICE"] = "1"
    args = ["--gpus", str(ranks), "--config", "c2", "--steps", "64", "--warmup", "8", "--replicas-per-gpu", "1",
            "--cpu-budget", "0", "--profile-steps", "4", "--min-window-s", "0.3", "--no-start-window",
            "--c5-steps", "0", "--cycle-scale", "0", "--no-f32-leg"]
    p = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True, env=env,
                       timeout=240, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    print({k: line[k] for k in ("value", "per_rank_values", "per_rank_seeds", "timed_s", "dtype")})
    assert line["n_gpus"] == ranks and line["dtype"] == "f64" and line["data"] == "synthetic"
    assert len(line["per_rank_values"]) == ranks and min(line["per_rank_values"]) > 1e7
    assert len(set(line["per_rank_seeds"])) == ranks
    assert line["per_rank_finite"] == [1.0] * ranks  # every rank's trajectories, not only rank 0's
    assert len(set(line["per_rank_checksums"])) == ranks  # distinct seeds: distinct trajectories
    n = line["config"]["particles"]
    assert line["value"] == pytest.approx(n * ranks * line["steps"] / line["timed_s"], rel=1e-9)
    assert line["config"]["finite"]
