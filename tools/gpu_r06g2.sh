#!/bin/bash
# round 6: trajectories per GPU (the replica count) at HEAD, fp64 C2 bench window
set -u
o=gpurun_out/r06g2
mkdir -p $o
: > $o/replicas.txt
for R in 2 3 4 5 6 8; do
  timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 20 --warmup 5 --replicas-per-gpu $R 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('R=$R value %.3e ms_per_step %.4f waves %s' % (d['value'], d['ms_per_step'], c.get('list_waves_per_tile')))" >> $o/replicas.txt || { echo "R=$R failed"; exit 1; }
done
cat $o/replicas.txt
