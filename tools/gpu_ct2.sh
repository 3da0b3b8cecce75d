#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python tools/interphase_probe.py 20000 1000 0,25,27 > gpurun_out/r03d_interphase_bits.txt 2>&1 || { tail -20 gpurun_out/r03d_interphase_bits.txt; exit 1; }
grep -E "contacts=|bits|run stats" gpurun_out/r03d_interphase_bits.txt
