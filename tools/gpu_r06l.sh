#!/bin/bash
# round 6 at HEAD: the whole GPU suite, smoke, the default bench line
set -u
o=gpurun_out/r06l
mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { echo "bench failed"; exit 1; }
