#!/bin/bash
# bond-batch (GCS_LIST_BOND_BATCH 2 / 8 vs 4) alternating A/B
export TMPDIR=/tmp
: > gpurun_out/r03k_ab.txt
for rep in 1 2; do
  bash tools/bench_variants.sh --steps 200 --warmup 50 --c5-steps 0 --cycle-scale 0 --replicas-per-gpu 1 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03k_ab.txt
  bash tools/bench_variants.sh --steps 20 --warmup 5 --c5-steps 0 --cycle-scale 0 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03k_ab.txt
done
cat gpurun_out/r03k_ab.txt
