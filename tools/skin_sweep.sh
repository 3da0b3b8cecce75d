#!/bin/bash
# list step: skin (per mille of the cutoff) x rebuild period on the full 4-replica bench (value per setting)
set -u
out=gpurun_out/skin_sweep.log
: > $out
for cfg in "400 8" "300 5" "350 6" "450 10" "500 12"; do
  set -- $cfg
  echo "== skin $1 every $2" >> $out
  timeout -k 10 150 python bench.py --cpu-budget 0 --no-start-window --engine-opt list_skin=$1 --engine-opt list_every=$2 > gpurun_out/skin_$1_$2.json 2>&1 || { echo "failed rc=$?" >> $out; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'],d['config']['single_trajectory_value'],d['config']['list_step'])" gpurun_out/skin_$1_$2.json >> $out
done
