#!/bin/bash
# list formats + tile dispatch order: the new GPU tests, then C5 rates of the default library (plane-relative 16-bit
# entries, tile order Bz = 4) against build/variants (Bz = 0 / 2 / 8, non-temporal list words) and 32-bit entries;
# C2 fp64 (variants must not matter there)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py -x -v --timeout 300 --timeout-method thread \
  -k "list_formats or relative_entries or ragged" > gpurun_out/r04m_tests.log 2>&1 || { tail -30 gpurun_out/r04m_tests.log; exit 1; }
tail -3 gpurun_out/r04m_tests.log
common="--c5-steps 0 --cycle-scale 0 --no-f32-leg --replicas-per-gpu 1 --steps 200 --warmup 30"
for rep in 1 2; do
  bash tools/bench_variants.sh --config c5 --precision 64 $common || exit 1
  cp gpurun_out/bench_variants.log gpurun_out/bv_c5_64_$rep.log
done
bash tools/bench_variants.sh --config c5 --precision 32 $common || exit 1
cp gpurun_out/bench_variants.log gpurun_out/bv_c5_32.log
for prec in 64 32; do
  GCS_LIB=3d-genome-cycle_amd/gcs/libgcs.so timeout -k 10 150 python -u bench.py --cpu-budget 0 --no-start-window --config c5 \
    --precision $prec $common --engine-opt list_format=2 2>&1 | tail -1 > gpurun_out/bv_c5_${prec}_int.json || exit 1
done
bash tools/bench_variants.sh --config c2 --steps 300 --warmup 50 --c5-steps 0 --cycle-scale 0 --no-f32-leg || exit 1
cp gpurun_out/bench_variants.log gpurun_out/bv_c2_64.log
