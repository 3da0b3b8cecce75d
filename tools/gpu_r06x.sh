#!/bin/bash
# round 6: the fp64 list step at 5 waves per SIMD (96 VGPRs, 80 B/lane of spills outside the pair loop) vs 4
set -u
o=gpurun_out/r06x
mkdir -p $o
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/c2_1.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/c2_2.txt
STEPS=300 bash tools/c5_variants.sh || exit 1
cp gpurun_out/c5_variants.log $o/c5.txt
cat $o/c2_1.txt $o/c2_2.txt $o/c5.txt
