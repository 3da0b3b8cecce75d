#!/bin/bash
# round 4: the fp64 rebuild period at the new default skin (350 per mille) and its neighbour 300
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/skin_sweep.sh 64 "350 8" "350 10" "350 12" "300 6" "300 8" "350 8" || exit 1
cp gpurun_out/skin_sweep_f64.log gpurun_out/skin_sweep_f64_period.log
