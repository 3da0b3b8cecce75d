#!/bin/bash
# round 6: staggered replica rebuild phases A/B (alternating), the phase test, the interphase stage's breakdown at the
# reference step count
set -u
o=gpurun_out/r06g
mkdir -p $o
: > $o/stagger_ab.txt
for rep in 1 2; do
  for s in "" "--no-stagger"; do
    timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 20 --warmup 5 $s 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('stagger=${s:-on} value %.3e single %.3e' % (d['value'], c['single_trajectory_value']))" >> $o/stagger_ab.txt || { echo "bench failed"; exit 1; }
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_list.py -k "phase" > $o/tests.log 2>&1 || { echo "tests failed"; tail -20 $o/tests.log; exit 1; }
timeout -k 10 400 python -u tools/interphase_probe.py 700000 10000 > $o/interphase_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
