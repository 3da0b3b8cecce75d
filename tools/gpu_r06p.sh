#!/bin/bash
# round 6: C5 fp64 A/B -- the default against the fp32 prefilter (8 + 2, 8 + 4 hits per round), then 2 waves per tile
set -u
STEPS=300 bash tools/c5_variants.sh || { echo "c5 variants failed"; cat gpurun_out/c5_variants.log; exit 1; }
for w in 2 4; do
  timeout -k 10 200 python -u bench.py --config c5 --replicas-per-gpu 1 --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 300 --warmup 50 --engine-opt list_waves=$w 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('list_waves=$w', 'value %.3e force_us %.2f' % (d['value'], 1e3*d['roofline']['force_ms']))" >> gpurun_out/c5_variants.log || { echo "waves $w failed"; exit 1; }
done
cat gpurun_out/c5_variants.log
