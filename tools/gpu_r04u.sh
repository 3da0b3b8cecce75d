#!/bin/bash
# decomposed runs at the new defaults (one rank RCCL vs undecomposed, C5 / C2 fp64), then the C2 R = 1 profile at HEAD
set -u
mkdir -p gpurun_out
for cfgn in c5 c2; do
  timeout -k 10 300 python -u bench.py --config $cfgn --decomp 1 --rccl --precision 64 --steps 200 --warmup 30 \
    > gpurun_out/r04u_decomp_$cfgn.log 2>&1 || { tail -20 gpurun_out/r04u_decomp_$cfgn.log; exit 1; }
  tail -1 gpurun_out/r04u_decomp_$cfgn.log
done
PROFILE_REPLICAS=1 bash tools/profile_round.sh r04u > gpurun_out/r04u_profile.log 2>&1 || { tail -20 gpurun_out/r04u_profile.log; exit 1; }
tail -2 gpurun_out/r04u_profile.log
