#!/bin/bash
# round 4: PMC passes of the default C5 step (fp64 list step at the dense synthetic start; 64-step window)
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIG=c5 STEPS=64 REPLICAS=1 bash tools/profile.sh r04_c5 > gpurun_out/r04_c5_profile.log 2>&1 || { tail -20 gpurun_out/r04_c5_profile.log; exit 1; }
d=gpurun_out/prof_r04_c5
python tools/summarize_pmc.py $d --traffic-out gpurun_out/r04_c5_lstep_traffic.json --kernel "k_lstep<int, 4, false, false, double, false>" > gpurun_out/r04_c5_pmc_summary.json || exit 1
cp "$(find $d/trace -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r04_c5_kernel_stats.csv
rm -rf $d
cat gpurun_out/r04_c5_lstep_traffic.json
