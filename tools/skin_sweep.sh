#!/bin/bash
# list step: skin (per mille of the cutoff) x rebuild period on the 4-replica bench (value per setting)
#   tools/skin_sweep.sh [precision] ["skin every" ...]   (default: fp64, the period at each skin from the auto rule)
set -u
prec=${1:-64}; shift || true
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=("350 8" "400 10" "450 13" "500 16" "600 23")
out=gpurun_out/skin_sweep_f$prec.log
: > $out
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  echo "== f$prec skin $1 every $2" >> $out
  timeout -k 10 150 python bench.py --precision $prec --no-f32-leg --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window --steps 400 \
    --engine-opt list_skin=$1 --engine-opt list_every=$2 > gpurun_out/skin_$1_$2.json 2>&1 || { echo "failed rc=$?" >> $out; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['config'];print('%.4e single %.4e k_lstep %.2f us cells %.2f us/step' % (d['value'],c['single_trajectory_value'],1e3*d['roofline']['force_ms'],1e3*d['roofline']['cell_ms']), c['list_step'])" gpurun_out/skin_$1_$2.json >> $out
done
cat $out
