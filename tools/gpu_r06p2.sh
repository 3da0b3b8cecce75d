#!/bin/bash
# round 6: the whole GPU suite (the long-horizon tests aside) with EVERY device allocation poisoned at birth
# (GCS_DEBUG_POISON=2) -- any kernel that reads memory nothing wrote sees hashed garbage instead of zeros
set -u
o=gpurun_out/r06p2
mkdir -p $o
GCS_DEBUG_POISON=2 GCS_DEBUG_SYNC=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -k "not long" -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "poisoned suite failed"; grep -E "FAILED|Error|GCS_DEBUG_SYNC" $o/tests.log | head -20; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
