#!/bin/bash
# round 6: GCS_OPT_LIST_SKIN_BASE -- its test, the whole GPU suite, then the default bench line (the C3 leg's
# interphase stage now runs its one trajectory at s1 = 400)
set -u
o=gpurun_out/r06h3
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $o/tests.log | head; tail -30 $o/tests.log; exit 1; }
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || { echo "bench failed"; tail $o/bench.err; exit 1; }
tail -1 $o/tests.log; grep skin_base $o/tests.log
python3 -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); c=d['config']
print(d['value'], c['c3_cycle_wall_s'], c['c3_cycle']['stages']['interphase'])"
