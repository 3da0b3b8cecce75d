"""The N>1 path of bench.py (independent replicas, no data-path collective) on CPU with gloo,
world_size 2: rendezvous, barrier, max-over-ranks time, distinct replica seeds, whole-job value -- and the
`bench.py --gpus 2` launcher itself (no WORLD_SIZE: the parent starts two ranks) with a stub engine."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _rank_main(rank, world, port, out_dir):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, str(ROOT))
    import bench
    w, r, local, dist = bench.dist_setup()
    bench.barrier(dist)
    el = 1.0 + 0.5 * r  # rank 1 is the slowest
    el_max = bench.max_over_ranks(dist, el)
    res = {"world": w, "rank": r, "local": local, "el_max": el_max,
           "master_seed": bench.replica_master_seed(r), "noise_seed": bench.replica_noise_seed(r),
           "value": bench.whole_job_value(60662, 100, w, el_max),
           "gathered": bench.gather_over_ranks(dist, 10.0 * (r + 1))}
    Path(out_dir, f"rank{r}.json").write_text(json.dumps(res))
    dist.destroy_process_group()


def test_two_replicas_gloo(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, bench._free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(world)]
    assert [x["rank"] for x in res] == [0, 1]
    assert all(x["world"] == world for x in res)
    assert all(x["el_max"] == pytest.approx(1.5) for x in res)  # max over ranks, seen by every rank
    assert res[0]["master_seed"] != res[1]["master_seed"]
    assert res[0]["noise_seed"] != res[1]["noise_seed"]
    assert res[0]["value"] == pytest.approx(60662 * 100 * 2 / 1.5)
    assert all(x["gathered"] == [10.0, 20.0] for x in res)


def _bench_line(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True, env=env,
                       timeout=240, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only prints
    return json.loads(lines[0])


def test_gpus_flag_launches_ranks_stub_engine():
    """`bench.py --gpus 2` with no WORLD_SIZE: two child ranks (gloo on 127.0.0.1), n_gpus 2, aggregate value = the
    updates of both ranks over the slower rank's time, per-rank rates reported."""
    line = _bench_line(["--gpus", "2", "--stub-engine", "--config", "c1", "--steps", "64", "--warmup", "8",
                        "--graph-steps", "32", "--replicas-per-gpu", "2", "--cpu-budget", "0", "--profile-steps", "2",
                        "--min-window-s", "0.2"])
    assert line["n_gpus"] == 2 and line["config"]["replicas"] == 4
    assert line["steps"] % 64 == 0 and line["steps"] >= 64 and line["steps_requested"] == 64
    assert line["warmup_steps_run"] >= 64  # at least two graph chunks
    assert line["timed_s"] >= 0.2
    assert len(line["per_rank_values"]) == 2
    n = line["config"]["particles"]
    assert line["value"] == pytest.approx(n * 2 * 2 * line["steps"] / line["timed_s"], rel=1e-9)
    assert line["value"] <= sum(line["per_rank_values"]) * (1 + 1e-9)


def test_single_gpu_stub_engine_defaults_to_one_rank():
    line = _bench_line(["--stub-engine", "--config", "c1", "--steps", "16", "--warmup", "2", "--cpu-budget", "0",
                        "--replicas-per-gpu", "1", "--profile-steps", "2", "--min-window-s", "0.05"])
    assert line["n_gpus"] == 1 and line["steps_requested"] == 16 and line["steps"] % 16 == 0
    assert line["warmup_steps_run"] >= 32  # G = min(graph_steps, steps) = 16, two chunks


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_launcher_ends_when_a_rank_fails(fail_rank):
    """`bench.py --gpus 2` when one rank dies (GCS_BENCH_FAIL_RANK: exit 3 right after the rendezvous, before the
    first barrier): the launcher polls every child, so it returns that exit code within seconds -- it does not sit
    in rank 0's wait while the survivor blocks in its barrier until the gloo timeout -- and no child is left
    running."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["GCS_BENCH_FAIL_RANK"] = str(fail_rank)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--stub-engine", "--config", "c1",
                        "--steps", "16", "--warmup", "2", "--cpu-budget", "0", "--replicas-per-gpu", "1",
                        "--profile-steps", "2", "--min-window-s", "0.05"],
                       capture_output=True, text=True, env=env, timeout=120, cwd=str(ROOT))
    elapsed = time.monotonic() - t0
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "failing on purpose" in p.stderr
    assert elapsed < 60, elapsed  # (gloo's own timeout is 30 min)
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]  # no bench line
