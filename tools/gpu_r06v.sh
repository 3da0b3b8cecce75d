#!/bin/bash
# round 6: k_lbuild's slabs at C5 (variant) against the default, then the C5 fp64 profile at HEAD
set -u
o=gpurun_out/r06v
mkdir -p $o
STEPS=300 bash tools/c5_variants.sh || { cat gpurun_out/c5_variants.log; exit 1; }
cp gpurun_out/c5_variants.log $o/c5.txt
CONFIG=c5 STEPS=200 PROFILE_REPLICAS=1 KERNEL="k_lstep<ListRel16, 4" bash tools/profile_round.sh r06v_c5 || { echo "c5 profile failed"; exit 1; }
cat $o/c5.txt
