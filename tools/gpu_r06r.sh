#!/bin/bash
# round 6: the list step's tail variants (GCS_TAIL_PAR x GCS_TAIL_OVERLAP) against HEAD's build: bench A/B twice and
# each build's final-workgroup timeline
set -u
o=gpurun_out/r06r
mkdir -p $o
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab1.txt
bash tools/bench_variants.sh --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench_variants.log $o/ab2.txt
for lib in build/variants/*.so; do
  GCS_LIB=$lib timeout -k 10 120 python -u tools/list_probe.py > $o/probe.txt 2>&1 || { echo "probe failed"; exit 1; }
  echo "$lib $(grep -E 'final workgroup|^ticket' $o/probe.txt | tr '\n' ' ')" >> $o/tails.txt
done
cat $o/ab1.txt $o/ab2.txt $o/tails.txt
