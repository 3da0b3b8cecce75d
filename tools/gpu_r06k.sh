#!/bin/bash
# round 6: the contact table's size (GCS_OPT_CONTACT_BITS 25 = default at C2, 24, 23) in the interphase stage
set -u
mkdir -p gpurun_out/r06k
timeout -k 10 500 python -u tools/interphase_probe.py 300000 10000 25,24,23 > gpurun_out/r06k/contact_bits.txt 2>&1 || { echo "probe failed"; exit 1; }
