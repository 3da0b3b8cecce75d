#!/bin/bash
# list step: skin (per mille of the cutoff) x rebuild period on the bench workload (profile() per-step times)
set -u
out=gpurun_out/sweep.log
: > $out
for cfg in "list_skin=400 list_every=5" "list_skin=400 list_every=8" "list_skin=500 list_every=8" "list_skin=500 list_every=10" "list_skin=600 list_every=12" "list_skin=300 list_every=4"; do
  echo "== $cfg" >> $out
  timeout -k 10 120 python -u tools/list_probe.py $cfg 2>&1 | head -2 >> $out || { echo "failed rc=$?" >> $out; exit 1; }
done
