#!/bin/bash
# contact-map update cost (bench config.contacts_update_ms) for the default library vs build/variants/*.so, alternating
set -u
shopt -s nullglob
out=gpurun_out/contact_ab.log
: > $out
for i in 1 2 3; do
  for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
    GCS_LIB=$lib timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --replicas-per-gpu 1 2>&1 | tail -n 1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$lib value %.3e contacts_ms %.4f' % (d['value'], c['contacts_update_ms']))" >> $out || { echo "failed" >> $out; exit 1; }
  done
done
