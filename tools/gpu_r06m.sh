#!/bin/bash
# round 6 diagnosis: the decomposed capacity test with every allocation poisoned (GCS_DEBUG_POISON=2) and a
# synchronisation after each decomposed launch (GCS_DEBUG_SYNC): which kernel reads memory nothing wrote
set -u
o=gpurun_out/r06m
mkdir -p $o
GCS_DEBUG_POISON=2 GCS_DEBUG_SYNC=1 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_domain.py -k "capacity" > $o/capacity.log 2>&1
echo "rc=$?" >> $o/capacity.log
