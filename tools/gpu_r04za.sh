#!/bin/bash
# decomposed runs follow the core-scale skin: the domain GPU tests (+ the list skin test), then the one-rank RCCL
# runs against undecomposed at the round-4 arguments
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_domain.py tests/test_gpu_list.py -k "domain or skin" -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04za_tests.log 2>&1 || { tail -40 gpurun_out/r04za_tests.log; exit 1; }
tail -1 gpurun_out/r04za_tests.log
for cfgn in c5 c2; do
  timeout -k 10 300 python -u bench.py --config $cfgn --decomp 1 --rccl --precision 64 --steps 400 --warmup 64 \
    > gpurun_out/r04za_decomp_$cfgn.log 2>&1 || { tail -20 gpurun_out/r04za_decomp_$cfgn.log; exit 1; }
  tail -1 gpurun_out/r04za_decomp_$cfgn.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$cfgn decomp %.3e undecomposed %.3e ratio %.3f' % (d['value'], c['undecomposed_value'], c['decomposed_over_undecomposed']))"
done
