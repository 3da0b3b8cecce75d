#!/bin/bash
# C5 fp64 at slot order with plane-relative 16-bit entries: the default (non-temporal list words) against
# build/variants nt0 / u8 (8 entries per batch), 32-bit entries, and the list skin
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py -x -v --timeout 300 --timeout-method thread \
  -k "list_formats or relative_entries" > gpurun_out/r04n_tests.log 2>&1 || { tail -30 gpurun_out/r04n_tests.log; exit 1; }
common="--c5-steps 0 --cycle-scale 0 --no-f32-leg --replicas-per-gpu 1 --steps 200 --warmup 30 --config c5 --precision 64"
for rep in 1 2; do
  bash tools/bench_variants.sh $common || exit 1
  cp gpurun_out/bench_variants.log gpurun_out/bw_c5_64_$rep.log
done
for opt in list_format=2 list_skin=250 list_skin=300 list_skin=450; do
  GCS_LIB=3d-genome-cycle_amd/gcs/libgcs.so timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window $common \
    --engine-opt $opt 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$opt value %.3e force_us %.2f' % (d['value'], 1e3*d['roofline']['force_ms']))" >> gpurun_out/bw_c5_opts.log || exit 1
done
