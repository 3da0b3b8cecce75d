#!/bin/bash
# round 6: the list rebuild period at the default fp64 skin (auto = 8 at the C2 window), the bench line and single
set -u
o=gpurun_out/r06g5
mkdir -p $o
: > $o/every.txt
for rep in 1 2; do
for m in 0 7 9 10 12; do
  timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 20 --warmup 5 --engine-opt list_every=$m 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']; l=c['list_step']
print('every=$m value %.3e single %.3e rebuild_every %s fallback %s builds %s' % (d['value'], c['single_trajectory_value'], l.get('rebuild_every'), l.get('fallback_particle_steps'), l.get('builds')))" >> $o/every.txt || { echo "failed"; exit 1; }
done
done
cat $o/every.txt
