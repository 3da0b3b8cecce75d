#!/bin/bash
# round 6: C5 fp64 one trajectory with the single-trajectory skin base (GCS_OPT_LIST_SKIN_BASE 400, 450) vs the default
set -u
o=gpurun_out/r06c2
mkdir -p $o
: > $o/c5.txt
for rep in 1 2; do
for b in 0 400 450; do
  timeout -k 10 200 python -u bench.py --config c5 --replicas-per-gpu 1 --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 300 --warmup 50 --engine-opt list_skin_base=$b 2>/dev/null | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); l=d['config']['list_step']
print('base=$b value %.3e force_us %.2f every %s skin %.4f' % (d['value'], 1e3*d['roofline']['force_ms'], l.get('rebuild_every'), l.get('skin')))" >> $o/c5.txt || { echo "failed"; exit 1; }
done
done
cat $o/c5.txt
