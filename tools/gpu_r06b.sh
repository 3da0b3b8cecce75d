#!/bin/bash
# round 6: the new small-step tests (stall, droplet, long horizon), the repeated decomposed run, the variant bench
# (prefilter shapes, slot-indexed bonds) and the full default bench line (C3 at the reference step counts)
set -u
o=gpurun_out/r06b
mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_small.py \
  tests/test_gpu_small_long.py tests/test_gpu_domain.py -k "small or twice" > $o/tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash tools/bench_variants.sh --steps 20 --warmup 5 && cp gpurun_out/bench_variants.log $o/bench_variants.log || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { echo "bench failed"; exit 1; }
