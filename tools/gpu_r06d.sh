#!/bin/bash
# round 6: the decomposed tests first (the unbinned-slot fix, poisoned buffers), then the whole GPU suite, smoke,
# the slot-bonds A/B and the default bench line
set -u
o=gpurun_out/r06d
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -v --timeout 300 --timeout-method thread > $o/domain_tests.log 2>&1 || { echo "domain tests failed"; tail -30 $o/domain_tests.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_gpu_domain.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/bench_variants.sh --steps 20 --warmup 5 && cp gpurun_out/bench_variants.log $o/bench_variants.log || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { echo "bench failed"; exit 1; }
