#!/usr/bin/env python3
"""Throughput of R independent C2 replicas sharing one GPU (one engine + HIP stream each).

    python tools/replicas_probe.py [--replicas 1 2 4] [--steps 1000]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))

import bench  # noqa: E402
from gcs import synthetic  # noqa: E402
from gcs.config import InterphaseConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    args = ap.parse_args()
    cfg = InterphaseConfig()
    for r in args.replicas:
        engines = []
        for k in range(r):
            d = synthetic.make_c2(master_seed=1 + k)
            engines.append(bench.make_engine(d, cfg, 0, bench.WINDOW_START))
        for k, e in enumerate(engines):
            e.run(args.warmup, first_step=bench.WINDOW_START, seed=bench.replica_noise_seed(k))
        for e in engines:
            e.synchronize()
        t0 = time.perf_counter()
        first = bench.WINDOW_START + args.warmup
        chunk = 64
        for s0 in range(0, args.steps, chunk):
            for k, e in enumerate(engines):
                e.run(min(chunk, args.steps - s0), first_step=first + s0, seed=bench.replica_noise_seed(k))
        for e in engines:
            e.synchronize()
        el = time.perf_counter() - t0
        n = engines[0].n
        print(json.dumps({"replicas": r, "steps": args.steps, "bead_updates_per_s": n * r * args.steps / el,
                          "us_per_step_per_replica": el / args.steps * 1e6}), flush=True)
        for e in engines:
            e.close()


if __name__ == "__main__":
    main()
