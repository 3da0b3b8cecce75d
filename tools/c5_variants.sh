#!/bin/bash
# C5 (606,248 beads, fp64, one trajectory) rate: the default library and every build/variants/*.so, alternating twice
set -u
shopt -s nullglob
out=gpurun_out/c5_variants.log
: > $out
for i in 1 2; do
  for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
    GCS_LIB=$lib timeout -k 10 200 python -u bench.py --config c5 --replicas-per-gpu 1 --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps ${STEPS:-300} --warmup 50 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$lib', 'value %.3e force_us %.2f' % (d['value'], 1e3*d['roofline']['force_ms']))" >> $out || { echo "failed $lib" >> $out; exit 1; }
  done
done
