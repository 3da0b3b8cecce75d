"""GPU: the replica path of bench.py with the REAL engine in more than one process (independent
trajectories one per GPU; the reference's ensemble is `scripts/simulate -s <seed>` runs, scripts/simulate:15-17).

`bench.py --gpus 2` without WORLD_SIZE starts two ranks (gloo on 127.0.0.1 for the barrier and the max-over-ranks
time); GCS_BENCH_SAME_DEVICE=1 puts both on device 0 of this one-GPU box (each rank its own process, HIP runtime,
engine and stream).  Checked: one JSON line from rank 0, every rank's rate present and positive, distinct noise seeds,
every rank's trajectories finite with distinct position checksums, the whole-job value = all ranks' bead-updates over
the slowest rank's time, fp64 arithmetic -- and, bit for bit, that rank r's trajectory is the one a single process
computes for replica r's noise seed from the same state (the launcher and the seed plumbing change nothing; VERDICT
r5 item 7).  2 ranks, and 8 (C4's 8-trajectory ensemble shape)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

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

    # every rank's trajectory again in this process: the same state, options and noise seed, run to the step its
    # checksum was taken at (chunking and graph replays do not change bits) -- the same float64 sum, exactly
    import bench
    from gcs import _abi as A
    cfg = bench.bench_config("c2")
    state = bench.load_state()
    w0 = line["window_start"]
    for r in range(ranks):
        e = bench.make_engine(bench.design_maker("c2")(master_seed=1), cfg, 0, w0, state, precision=64)
        for opt, v in ((A.OPT_GRAPH_STEPS, 32), (A.OPT_SCAN_BLOCKS, 1), (A.OPT_LIST_WAVES, 4)):
            e.set_option(opt, v)
        steps = int(line["per_rank_checksum_steps"][r]) - w0
        e.run(steps, first_step=w0, seed=bench.replica_noise_seed(r), temperature=cfg.temperature,
              timestep=cfg.timestep)
        s = float(np.asarray(e.get_positions(), dtype=np.float64).sum())
        e.close()
        assert s == line["per_rank_checksums"][r], (r, steps, s, line["per_rank_checksums"][r])
