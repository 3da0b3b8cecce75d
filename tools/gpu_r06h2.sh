#!/bin/bash
# round 6: the interphase stage (700k steps, contact map on) with the fp64 default skin's s1 at 350 (default), 400,
# 450, 500 per mille (GCS_OPT_LIST_SKIN_BASE); one trajectory alone on the GPU
set -u
o=gpurun_out/r06h2
mkdir -p $o
timeout -k 10 600 python -u tools/interphase_probe.py 700000 10000 0 0,400,450,500 > $o/probe.txt 2>&1 || { echo "probe failed"; tail $o/probe.txt; exit 1; }
grep -E "skin base|sha1|^contacts=" $o/probe.txt
