#!/bin/bash
# list skin against the core scale: C5 fp64 / fp32 (the synthetic start, core scale 0.5 -> ...) and the C2 fp64
# start window (core scale 0.5) and headline (0.99), per skin
set -u
mkdir -p gpurun_out
out=gpurun_out/r04o_skin.log
: > $out
run() {  # label, bench args...
  local label=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e force_us %.2f start_window %s' % (d['value'], 1e3*d['roofline']['force_ms'], c.get('start_window_value')))" >> $out
}
c5="--config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --no-start-window"
for sk in 150 200 250; do run "c5 f64 skin $sk" $c5 --precision 64 --engine-opt list_skin=$sk || exit 1; done
for sk in 200 250 300 350 500; do run "c5 f32 skin $sk" $c5 --precision 32 --engine-opt list_skin=$sk || exit 1; done
for sk in 175 250 350; do run "c2 f64 skin $sk" --config c2 --steps 300 --warmup 50 --engine-opt list_skin=$sk || exit 1; done
