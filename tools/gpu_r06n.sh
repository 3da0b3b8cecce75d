#!/bin/bash
# round 6: the decomposed tests with every allocation poisoned (and a sync after each decomposed launch), then the
# whole GPU suite in its own order (the order in which the fault came), smoke, the default bench line
set -u
o=gpurun_out/r06n
mkdir -p $o
GCS_DEBUG_POISON=2 GCS_DEBUG_SYNC=1 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_domain.py -k "capacity or motion or twice or poison" > $o/poisoned_domain.log 2>&1 || { echo "poisoned domain tests failed"; grep -E "GCS_DEBUG_SYNC|Error" $o/poisoned_domain.log | head; exit 1; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { echo "bench failed"; exit 1; }
# the interphase stage with the per-workgroup contact compaction (contacts_accumulate host ms per call)
timeout -k 10 300 python -u tools/interphase_probe.py 300000 10000 > $o/interphase_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
