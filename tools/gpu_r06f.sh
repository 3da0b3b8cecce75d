#!/bin/bash
# round 6, final state: the GPU suite, smoke, the default bench line, and the C2 profiles (R = 1, R = 4) at HEAD
set -u
o=gpurun_out/r06f
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; cat $o/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail $o/bench.err; exit 1; }
bash tools/profile_round.sh r06f || { echo "profile failed"; exit 1; }
tail -1 $o/tests.log; tail -1 $o/smoke.log; tail -c 600 $o/bench.json
