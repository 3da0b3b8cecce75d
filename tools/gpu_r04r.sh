#!/bin/bash
# fp32 skin x cs and the dense threshold 96: list GPU tests, C5 fp32 / fp64 defaults, C2 fp32 headline + start window
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04r_tests.log 2>&1 || { tail -30 gpurun_out/r04r_tests.log; exit 1; }
tail -1 gpurun_out/r04r_tests.log
out=gpurun_out/r04r_bench.log
: > $out
run() {
  local label=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e force_us %.2f start_window %s' % (d['value'], 1e3*d['roofline']['force_ms'], c.get('start_window_value')))" >> $out
}
c5="--config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --no-start-window"
run "c5 f32 default" $c5 --precision 32 || exit 1
run "c5 f32 list, skin 200" $c5 --precision 32 --engine-opt list_skin=200 || exit 1
run "c5 f64 default" $c5 --precision 64 || exit 1
run "c2 f32 default + start window" --config c2 --steps 300 --warmup 50 --precision 32 || exit 1
