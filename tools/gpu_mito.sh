#!/bin/bash
export TMPDIR=/tmp
for sp in 0 1; do
  timeout -k 10 200 python tools/mitotic_probe.py 20000 $sp > gpurun_out/r03g_mitotic_small$sp.txt 2>&1 || { tail -20 gpurun_out/r03g_mitotic_small$sp.txt; exit 1; }
  echo "small path $sp:"; cat gpurun_out/r03g_mitotic_small$sp.txt
done
