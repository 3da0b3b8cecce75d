#!/bin/bash
# round 6 profiles at HEAD: rocprofv3 kernel trace + PMC passes of the bench (R = 1 and R = 4), the production-start
# and bench-window list-step timelines, and the rocprofv3 exit crash of the small-step run with its memory map
set -u
mkdir -p gpurun_out/r06e
bash tools/profile_round.sh r06 || { echo "profile failed"; exit 1; }
timeout -k 10 240 python -u tools/list_probe.py start=1 > gpurun_out/r06e/list_probe_start.txt 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 240 python -u tools/list_probe.py > gpurun_out/r06e/list_probe_window.txt 2>&1 || { echo "probe failed"; exit 1; }
export TMPDIR=/tmp
GCS_MAPS_OUT=gpurun_out/r06e/pstep_maps.txt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e/pstep -o run --output-format csv -- python3 tools/pstep_run.py 8192 > gpurun_out/r06e/pstep_prof.log 2>&1
echo "pstep profile rc=$?" >> gpurun_out/r06e/pstep_prof.log
exit 0
