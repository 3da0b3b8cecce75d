#!/bin/bash
# the bench line at several replicas per GPU (no CPU leg, no start window)
set -u
out=gpurun_out/replica_sweep.log
: > $out
for r in "$@"; do
  echo "== replicas $r" >> $out
  timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --replicas-per-gpu $r 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('value %.3e single %.3e waves %s' % (d['value'], c['single_trajectory_value'], c.get('list_waves_per_tile')))" >> $out || { echo "failed" >> $out; exit 1; }
done
