#!/bin/bash
# C5 fp32: the list step (GCS_OPT_DENSE_NEIGHBORS 0) against the tile step the density switch picks; then a C5 fp64
# kernel trace at the default (core-scale) skin
set -u
mkdir -p gpurun_out
out=gpurun_out/r04q_bench.log
: > $out
run() {
  local label=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e force_us %.2f start_window %s' % (d['value'], 1e3*d['roofline']['force_ms'], c.get('start_window_value')))" >> $out
}
c5="--config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --no-start-window"
run "c5 f32 default (tile step)" $c5 --precision 32 || exit 1
run "c5 f32 list step, default skin" $c5 --precision 32 --engine-opt dense_neighbors=0 || exit 1
run "c5 f32 list step, skin 250" $c5 --precision 32 --engine-opt dense_neighbors=0 --engine-opt list_skin=250 || exit 1
run "c5 f32 list step, skin 300" $c5 --precision 32 --engine-opt dense_neighbors=0 --engine-opt list_skin=300 || exit 1
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04q -o run --output-format csv -- python3 bench.py \
  --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg $c5 --precision 64 --profile-steps 10 > gpurun_out/r04q_trace.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py -x -v --timeout 300 --timeout-method thread -k "skin" \
  > gpurun_out/r04q_tests.log 2>&1 || { tail -30 gpurun_out/r04q_tests.log; exit 1; }
run "c5 f64 default (sqrt rule)" $c5 --precision 64 || exit 1
run "c2 f64 default (sqrt rule) + start window" --config c2 --steps 300 --warmup 50 || exit 1
