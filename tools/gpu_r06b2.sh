#!/bin/bash
# round 6: the list build's compile-time shape at HEAD -- candidate groups per tile (4 vs 2) and occupancy target
# (6 / 4 vs 8 waves per SIMD) -- the bench line (C2, 4 trajectories + single), alternating twice, then C5
set -u
o=gpurun_out/r06b2
mkdir -p $o
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/c2_1.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/c2_2.txt
STEPS=300 bash tools/c5_variants.sh || exit 1
cp gpurun_out/c5_variants.log $o/c5.txt
cat $o/c2_1.txt $o/c2_2.txt $o/c5.txt
