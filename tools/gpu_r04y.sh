#!/bin/bash
# headline shape sweep: replicas per GPU x hardware queues (GPU_MAX_HW_QUEUES, read at HIP init) x waves per tile
set -u
mkdir -p gpurun_out
out=gpurun_out/r04y_shapes.log
: > $out
run() {
  local label=$1; shift
  timeout -k 10 200 "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e single %.3e force_us %.2f' % (d['value'], c['single_trajectory_value'], 1e3*d['roofline']['force_ms']))" >> $out
}
b="python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg --no-start-window --steps 300 --warmup 50"
run "R4 q4 (default)" $b || exit 1
run "R4 q4 waves4" $b --list-waves 4 || exit 1
run "R8 q8" env GPU_MAX_HW_QUEUES=8 $b --replicas-per-gpu 8 || exit 1
run "R6 q8" env GPU_MAX_HW_QUEUES=8 $b --replicas-per-gpu 6 || exit 1
run "R4 q8" env GPU_MAX_HW_QUEUES=8 $b || exit 1
run "R12 q16" env GPU_MAX_HW_QUEUES=16 $b --replicas-per-gpu 12 || exit 1
run "R16 q16" env GPU_MAX_HW_QUEUES=16 $b --replicas-per-gpu 16 || exit 1
cat $out
