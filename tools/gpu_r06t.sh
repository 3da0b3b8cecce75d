#!/bin/bash
# round 6: the XCD remap off at C2 (the bench line: 4 trajectories + single), alternating, twice
set -u
o=gpurun_out/r06t
mkdir -p $o
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab1.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab2.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 --precision 32 || exit 1
cp gpurun_out/bench_variants.log $o/ab_f32.txt
cat $o/ab1.txt $o/ab2.txt $o/ab_f32.txt
