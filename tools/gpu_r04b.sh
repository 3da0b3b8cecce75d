#!/bin/bash
# round 4: fp64 step variants (A/B on one box), then the rocprofv3 passes of the fp64 bench at R = 1 and R = 4 (last:
# an R = 4 kernel-trace crash ends the call with its trace and memory map kept for tools/symbolize_trace.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
# the fp32 engine as the headline (does the f32 leg of the fp64 line read the same rate?)
timeout -k 10 300 python bench.py --precision 32 --no-f32-leg --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window > gpurun_out/r04_bench_f32.log 2>&1 || { tail -20 gpurun_out/r04_bench_f32.log; exit 1; }
tail -1 gpurun_out/r04_bench_f32.log | cut -c1-300
bash tools/bench_variants.sh --no-f32-leg --c5-steps 0 --cycle-scale 0 --steps 400 || { cat gpurun_out/bench_variants.log; exit 1; }
cat gpurun_out/bench_variants.log
bash tools/profile_round.sh ${TAG:-r04} > gpurun_out/${TAG:-r04}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG:-r04}_profile.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04}_profile.log
