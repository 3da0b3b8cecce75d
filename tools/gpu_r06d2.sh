#!/bin/bash
# round 6: the decomposed single trajectory at HEAD -- one domain, the engine-issued RCCL sequence with one rank,
# beside the same trajectory undecomposed (bench.py --decomp 1 --rccl), C2 and C5, fp64
set -u
o=gpurun_out/r06d2
mkdir -p $o
timeout -k 10 300 python -u bench.py --decomp 1 --rccl --steps 400 --warmup 100 > $o/c2.json 2> $o/c2.err || { echo "c2 failed"; tail $o/c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --decomp 1 --rccl --config c5 --steps 200 --warmup 50 > $o/c5.json 2> $o/c5.err || { echo "c5 failed"; tail $o/c5.err; exit 1; }
for f in c2 c5; do python3 -c "
import json; d=json.loads([l for l in open('$o/$f.json').read().splitlines() if l.startswith('{')][-1]); c=d['config']
print('$f', d['value'], c.get('undecomposed_value'), c.get('decomposed_over_undecomposed'))"; done
