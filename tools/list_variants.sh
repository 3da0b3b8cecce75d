#!/bin/bash
# time the list step of every library under build/variants (and the default build) on the bench workload
set -u
shopt -s nullglob
out=gpurun_out/variants.log
: > $out
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
  echo "== $lib" >> $out
  GCS_LIB=$lib timeout -k 10 120 python -u tools/list_probe.py "$@" >> $out 2>&1 || { echo "failed rc=$?" >> $out; exit 1; }
done
