#!/bin/bash
# C5 decomposed (1 domain) rate, default library vs build/variants/all5.so, alternating 3 times on one box
set -u
out=gpurun_out/c5_ab.log
: > $out
for i in 1 2 3; do
  for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/all5.so; do
    GCS_LIB=$lib timeout -k 10 150 python -u bench.py --cpu-budget 0 --config c5 --decomp 1 --steps 300 --warmup 50 2>&1 | tail -n 1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$lib', '%.3e' % d['value'])" >> $out || { echo "failed" >> $out; exit 1; }
  done
done
