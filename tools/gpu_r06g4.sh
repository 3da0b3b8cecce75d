#!/bin/bash
# round 6: the fp64 list skin (per mille of the cutoff) at HEAD, the bench line (R = 4) and single
set -u
o=gpurun_out/r06g4
mkdir -p $o
: > $o/skin.txt
for rep in 1 2; do
for sk in 300 350 400 450; do
  timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 20 --warmup 5 --engine-opt list_skin=$sk 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('skin=$sk value %.3e single %.3e every %s' % (d['value'], c['single_trajectory_value'], c['list_step'].get('rebuild_every')))" >> $o/skin.txt || { echo "failed"; exit 1; }
done
done
cat $o/skin.txt
