#!/bin/bash
# round 6: the list step's tail with the wave-parallel combine (kernels.hip list_totals) -- bitwise against HEAD's
# build, a same-box A/B (alternating), the per-workgroup timeline, then the GPU suite
set -u
o=gpurun_out/r06q
mkdir -p $o
for c in "c2 64 200" "c1 64 300" "c2 32 200"; do
  set -- $c
  GCS_LIB=build/variants/head.so timeout -k 10 120 python -u tools/lib_bitwise.py $1 $2 $3 $o/a.npy > /dev/null 2>&1 || { echo "head run failed $c"; exit 1; }
  timeout -k 10 120 python -u tools/lib_bitwise.py $1 $2 $3 $o/b.npy > /dev/null 2>&1 || { echo "new run failed $c"; exit 1; }
  python3 -c "
import numpy as np; a=np.load('$o/a.npy'); b=np.load('$o/b.npy')
print('$c', 'bitwise' if np.array_equal(a, b) else 'DIFFER max %g' % abs(a-b).max())" >> $o/bitwise.txt
done
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab1.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab2.txt
timeout -k 10 120 python -u tools/list_probe.py > $o/list_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log; cat $o/bitwise.txt $o/ab1.txt $o/ab2.txt
