"""The N>1 path of bench.py (independent replicas, no data-path collective) on CPU with gloo,
world_size 2: rendezvous, barrier, max-over-ranks time, distinct replica seeds, whole-job value."""
import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
           "value": bench.whole_job_value(60662, 100, w, el_max)}
    Path(out_dir, f"rank{r}.json").write_text(json.dumps(res))
    dist.destroy_process_group()


def test_two_replicas_gloo(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(world)]
    assert [x["rank"] for x in res] == [0, 1]
    assert all(x["world"] == world for x in res)
    assert all(x["el_max"] == pytest.approx(1.5) for x in res)  # max over ranks, seen by every rank
    assert res[0]["master_seed"] != res[1]["master_seed"]
    assert res[0]["noise_seed"] != res[1]["noise_seed"]
    assert res[0]["value"] == pytest.approx(60662 * 100 * 2 / 1.5)
