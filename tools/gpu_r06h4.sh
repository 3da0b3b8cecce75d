#!/bin/bash
# round 6 (experiment): the fp64 default skin's core-scale exponent (s1 cs^x, x = 0.5 default) for the stage
# driver's one trajectory (s1 = 400), interphase stage 300k steps (the core-scale ramp) with contacts
set -u
o=gpurun_out/r06h4
mkdir -p $o
: > $o/exp.txt
for x in 0.5 0.25 0.0; do
  GCS_SKIN_EXP=$x timeout -k 10 300 python -u tools/interphase_probe.py 300000 10000 > $o/probe.txt 2>&1 || { echo "probe failed"; tail $o/probe.txt; exit 1; }
  echo "x=$x $(grep -E '^contacts=True' $o/probe.txt)" >> $o/exp.txt
done
cat $o/exp.txt
