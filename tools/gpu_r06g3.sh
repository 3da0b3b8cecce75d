#!/bin/bash
# round 6: waves per tile with several trajectories (the bench picks 2 for R > 1)
set -u
o=gpurun_out/r06g3
mkdir -p $o
: > $o/waves.txt
for R in 4 8; do
  for w in 2 4; do
    timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 20 --warmup 5 --replicas-per-gpu $R --engine-opt list_waves=$w 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('R=$R list_waves=$w value %.3e ms_per_step %.4f' % (d['value'], d['ms_per_step']))" >> $o/waves.txt || { echo "failed"; exit 1; }
  done
done
cat $o/waves.txt
