#!/bin/bash
# the bench line (no CPU leg, no start window) with the default library and every build/variants/*.so
set -u
shopt -s nullglob
out=gpurun_out/bench_variants.log
: > $out
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
  echo "== $lib $*" >> $out
  GCS_LIB=$lib timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('value %.3e single %.3e force_us %.2f' % (d['value'], c['single_trajectory_value'], 1e3*d['roofline']['force_ms']))" >> $out || { echo "failed" >> $out; exit 1; }
done
