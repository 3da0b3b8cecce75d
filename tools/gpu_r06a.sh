#!/bin/bash
# round 6: the fp64 list step's fp32 prefilter -- bitwise vs the gather-every-entry step, the new small-step tests,
# then the bench line of every variant library (tools/build_variant.sh)
set -u
mkdir -p gpurun_out/r06a
o=gpurun_out/r06a
for cfg in "c2 64 60" "c5 64 12"; do
  set -- $cfg
  for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/pf0.so; do
    tag=$(basename $lib .so)
    GCS_LIB=$lib timeout -k 10 240 python -u tools/lib_bitwise.py $1 $2 $3 $o/$1_$tag.npy >> $o/bitwise.log 2>&1 || { echo "bitwise run failed: $cfg $lib" >> $o/bitwise.log; exit 1; }
  done
  python3 -c "
import numpy as np,sys
a=np.load('$o/$1_libgcs.npy'); b=np.load('$o/$1_pf0.npy')
print('$1 bitwise', np.array_equal(a,b), float(np.abs(a-b).max()))" >> $o/bitwise.log
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_small.py \
  tests/test_gpu_list.py -k "small or formats or relative or c1 or c2_" > $o/tests.log 2>&1 || { echo "tests failed"; exit 1; }
bash tools/bench_variants.sh --steps 20 --warmup 5 && cp gpurun_out/bench_variants.log $o/bench_variants.log
