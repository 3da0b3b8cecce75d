#!/bin/bash
# Reproduce the rocprofv3 --kernel-trace SIGSEGV of round 3 (first hipGraphLaunch after the density probe, fp32 engine,
# 4 replicas) with the process's /proc/self/maps captured just before the first graph launch (bench.py GCS_MAPS_OUT),
# so the crash trace's PCs can be symbolised against the loaded libraries.  Run LAST in a GPU call (it may abort).
set -u
export TMPDIR=/tmp
out=gpurun_out/crash_${TAG:-r04}
mkdir -p $out
bench=(python3 "$(pwd)/bench.py" --precision ${PREC:-32} --steps 300 --warmup 50 --cpu-budget 0 --profile-steps 10
       --no-start-window --replicas-per-gpu ${REPLICAS:-4} --c5-steps 0 --cycle-scale 0 --no-f32-leg)
GCS_MAPS_OUT=$out/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv \
  -- "${bench[@]}" > $out/trace.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc" | tee -a $out/trace.log
tail -3 $out/trace.log
find $out/trace -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \; 2>/dev/null
rm -rf $out/trace
exit 0
