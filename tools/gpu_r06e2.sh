#!/bin/bash
# round 6, closing check: the whole GPU suite (with the skin-base tests) and smoke at HEAD
set -u
o=gpurun_out/r06e2
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $o/tests.log | head; tail -30 $o/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; cat $o/smoke.log; exit 1; }
tail -1 $o/tests.log; grep skin_base $o/tests.log; tail -1 $o/smoke.log
