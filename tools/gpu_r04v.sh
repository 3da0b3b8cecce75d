#!/bin/bash
# decomposed one-rank RCCL runs at the round-4 arguments (400 steps, 64 warm-up), then the C2 R = 4 profile at HEAD
set -u
mkdir -p gpurun_out
for cfgn in c5 c2; do
  timeout -k 10 300 python -u bench.py --config $cfgn --decomp 1 --rccl --precision 64 --steps 400 --warmup 64 \
    > gpurun_out/r04v_decomp_$cfgn.log 2>&1 || { tail -20 gpurun_out/r04v_decomp_$cfgn.log; exit 1; }
  tail -1 gpurun_out/r04v_decomp_$cfgn.log
done
PROFILE_REPLICAS=4 bash tools/profile_round.sh r04v > gpurun_out/r04v_profile.log 2>&1 || { tail -20 gpurun_out/r04v_profile.log; exit 1; }
tail -2 gpurun_out/r04v_profile.log
