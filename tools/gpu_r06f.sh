#!/bin/bash
# round 6 A/B: fp64 list entries per batch 8 vs 4 (the default)
set -u
mkdir -p gpurun_out/r06f
bash tools/bench_variants.sh --steps 20 --warmup 5 && cp gpurun_out/bench_variants.log gpurun_out/r06f/u8_ab1.txt || exit 1
bash tools/bench_variants.sh --steps 20 --warmup 5 && cp gpurun_out/bench_variants.log gpurun_out/r06f/u8_ab2.txt || exit 1
bash tools/bench_variants.sh --steps 20 --warmup 5 --config c5 --replicas-per-gpu 1 && cp gpurun_out/bench_variants.log gpurun_out/r06f/u8_c5.txt || exit 1
