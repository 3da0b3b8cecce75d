#!/bin/bash
# A/B: non-temporal list word loads (build/variants/nt.so) vs the default library, C5 fp64 / fp32 and C2 fp64
set -u
mkdir -p gpurun_out
common="--c5-steps 0 --cycle-scale 0 --no-f32-leg"
for rep in 1 2; do
  bash tools/bench_variants.sh --config c5 --precision 64 --replicas-per-gpu 1 --steps 200 --warmup 30 $common || exit 1
  cp gpurun_out/bench_variants.log gpurun_out/bv_c5_64_$rep.log
done
bash tools/bench_variants.sh --config c5 --precision 32 --replicas-per-gpu 1 --steps 200 --warmup 30 $common || exit 1
cp gpurun_out/bench_variants.log gpurun_out/bv_c5_32.log
bash tools/bench_variants.sh --config c2 --steps 300 --warmup 50 $common || exit 1
cp gpurun_out/bench_variants.log gpurun_out/bv_c2_64.log
