#!/bin/bash
# One GPU call: the full suite + driver bench + interphase probe (tools/gpu_full.sh), then the k_lstep occupancy
# variants A/B (build/variants/*.so, tools/build_variant.sh), then the rocprofv3 passes (tools/profile_round.sh r03c)
set -u
bash tools/gpu_full.sh || exit $?
for rep in 1 2; do
  bash tools/bench_variants.sh --steps 20 --warmup 5 --c5-steps 0 --cycle-scale 0 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03c_variants.txt
  bash tools/bench_variants.sh --steps 200 --warmup 50 --c5-steps 0 --cycle-scale 0 --replicas-per-gpu 1 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03c_variants.txt
done
cat gpurun_out/r03c_variants.txt
bash tools/profile_round.sh r03c > gpurun_out/r03c_profile.log 2>&1 || { tail -20 gpurun_out/r03c_profile.log; exit 1; }
tail -3 gpurun_out/r03c_profile.log
