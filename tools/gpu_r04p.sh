#!/bin/bash
# skin levels (engine.hip skin_level): list + parity GPU tests, then the C5 fp64 rate and the C2 headline / start
# window at fp64 and fp32 with the default (core-scale) skin against the fixed skin
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_list.py tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r04p_tests.log 2>&1 || { tail -30 gpurun_out/r04p_tests.log; exit 1; }
tail -2 gpurun_out/r04p_tests.log
out=gpurun_out/r04p_bench.log
: > $out
run() {
  local label=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e force_us %.2f start_window %s' % (d['value'], 1e3*d['roofline']['force_ms'], c.get('start_window_value')))" >> $out
}
c5="--config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --no-start-window --precision 64"
run "c5 f64 default" $c5 || exit 1
run "c5 f64 skin 350" $c5 --engine-opt list_skin=350 || exit 1
run "c2 f64 default" --config c2 --steps 300 --warmup 50 || exit 1
run "c2 f64 skin 350" --config c2 --steps 300 --warmup 50 --engine-opt list_skin=350 || exit 1
run "c2 f32 default" --config c2 --steps 300 --warmup 50 --precision 32 || exit 1
run "c2 f32 skin 500" --config c2 --steps 300 --warmup 50 --precision 32 --engine-opt list_skin=500 || exit 1
