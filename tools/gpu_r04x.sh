#!/bin/bash
# the blocked list build (GCS_LBUILD_BLOCK 4) against the previous HEAD (build/variants/prev.so): bitwise equal
# trajectories (C2 fp64 / fp32, C5 fp64), the list GPU tests, then the rates (bench_variants: C2 headline, C5)
set -u
mkdir -p gpurun_out
out=gpurun_out/r04x_bitwise.log
: > $out
for spec in "c2 64 200" "c2 32 200" "c5 64 40"; do
  set -- $spec
  for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/prev.so; do
    tag=$(basename $lib .so)
    GCS_LIB=$lib timeout -k 10 200 python -u tools/lib_bitwise.py $1 $2 $3 gpurun_out/bw_$1_$2_$tag.npy >> $out 2>&1 || exit 1
  done
  python3 -c "
import numpy as np
a=np.load('gpurun_out/bw_$1_$2_libgcs.npy'); b=np.load('gpurun_out/bw_$1_$2_prev.npy')
print('$1 $2', 'bitwise equal' if np.array_equal(a,b) else 'DIFFERENT max %g' % abs(a-b).max())" >> $out
done
rm -f gpurun_out/bw_*.npy
cat $out | grep -E "bitwise|DIFF"
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04x_tests.log 2>&1 || { tail -30 gpurun_out/r04x_tests.log; exit 1; }
tail -1 gpurun_out/r04x_tests.log
bash tools/bench_variants.sh --config c2 --steps 300 --warmup 50 --c5-steps 0 --cycle-scale 0 --no-f32-leg || exit 1
cp gpurun_out/bench_variants.log gpurun_out/r04x_bv_c2.log
bash tools/bench_variants.sh --config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --c5-steps 0 --cycle-scale 0 --no-f32-leg || exit 1
cp gpurun_out/bench_variants.log gpurun_out/r04x_bv_c5.log
