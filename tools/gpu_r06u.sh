#!/bin/bash
# round 6: the XCD slab remap only for the 16-bit absolute lists -- C5 and C2 against HEAD's build, then the suite
set -u
o=gpurun_out/r06u
mkdir -p $o
STEPS=300 bash tools/c5_variants.sh || { cat gpurun_out/c5_variants.log; exit 1; }
cp gpurun_out/c5_variants.log $o/c5.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/c2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log; cat $o/c5.txt $o/c2.txt
