#!/bin/bash
# tile-kernel (k_force) variants: the rebuild step on C2 (--fused 2) and the decomposed C5 path with one domain,
# for the default library and every build/variants/*.so on one box
set -u
shopt -s nullglob
out=gpurun_out/force_variants.log
: > $out
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
  for args in "--fused 2" "--config c5 --decomp 1 --steps 300 --warmup 50 --replicas-per-gpu 1"; do
    echo "== $lib $args" >> $out
    GCS_LIB=$lib timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window $args 2>&1 | tail -n 1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value %.3e' % d['value'])" >> $out || { echo "failed" >> $out; exit 1; }
  done
done
