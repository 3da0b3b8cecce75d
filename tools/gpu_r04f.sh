#!/bin/bash
# round 4: fp64 bond batch x occupancy variants (A/B on one box, twice), then the R = 4 rocprofv3 passes (last)
export TMPDIR=/tmp
mkdir -p gpurun_out
# the fp64 skin below the round's first sweep (400 per mille / 10 steps was the best of 400..600)
bash tools/skin_sweep.sh 64 "250 4" "300 6" "350 8" "400 10" || exit 1
cp gpurun_out/skin_sweep_f64.log gpurun_out/skin_sweep_f64_low.log
for rep in 1 2; do
  bash tools/bench_variants.sh --no-f32-leg --c5-steps 0 --cycle-scale 0 --steps 400 || { cat gpurun_out/bench_variants.log; exit 1; }
  cat gpurun_out/bench_variants.log >> gpurun_out/r04_variants_bb.log
done
cat gpurun_out/r04_variants_bb.log
# the interphase stage at fp64 (contact map, energy, frames at the reference cadence; relaxation on the lists)
timeout -k 10 300 python tools/interphase_probe.py 20000 1000 > gpurun_out/r04_interphase_probe.txt 2>&1 || { tail -20 gpurun_out/r04_interphase_probe.txt; exit 1; }
tail -12 gpurun_out/r04_interphase_probe.txt
PROFILE_REPLICAS=4 bash tools/profile_round.sh ${TAG:-r04} > gpurun_out/${TAG:-r04}_profile_r4.log 2>&1 || { tail -20 gpurun_out/${TAG:-r04}_profile_r4.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04}_profile_r4.log
