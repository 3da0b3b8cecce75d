#!/bin/bash
# round 4: fp64 bond batch x occupancy variants (A/B on one box, twice), then the R = 4 rocprofv3 passes (last)
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  bash tools/bench_variants.sh --no-f32-leg --c5-steps 0 --cycle-scale 0 --steps 400 || { cat gpurun_out/bench_variants.log; exit 1; }
  cat gpurun_out/bench_variants.log >> gpurun_out/r04_variants_bb.log
done
cat gpurun_out/r04_variants_bb.log
PROFILE_REPLICAS=4 bash tools/profile_round.sh ${TAG:-r04} > gpurun_out/${TAG:-r04}_profile_r4.log 2>&1 || { tail -20 gpurun_out/${TAG:-r04}_profile_r4.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04}_profile_r4.log
