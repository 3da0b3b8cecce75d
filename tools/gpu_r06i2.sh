#!/bin/bash
# round 6: kernel trace of the interphase stage (C2 from step 0 through InterphaseDriver: 100k steps with the contact
# map, 10k relaxation), for the stage's kernel mix
set -u
o=gpurun_out/r06i2
mkdir -p $o
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0  # (tools/profile.sh: the profiler's graph-packet overread)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 tools/interphase_probe.py 100000 10000 > $o/trace.log 2>&1 || { echo "trace failed"; tail -20 $o/trace.log; exit 1; }
cp "$(find $o/trace -name '*kernel_stats.csv' | head -n 1)" $o/kernel_stats.csv && rm -rf $o/trace
head -12 $o/kernel_stats.csv | cut -c1-200
