#!/bin/bash
# round 4: per-workgroup timeline of one k_lstep (GCS_DEBUG_TIMES), fp64 default and fp32
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/list_probe.py > gpurun_out/r04_list_probe_f64.txt 2>&1 || { tail -20 gpurun_out/r04_list_probe_f64.txt; exit 1; }
cat gpurun_out/r04_list_probe_f64.txt
GCS_PROBE_PRECISION=32 timeout -k 10 200 python tools/list_probe.py > gpurun_out/r04_list_probe_f32.txt 2>&1 || { tail -20 gpurun_out/r04_list_probe_f32.txt; exit 1; }
cat gpurun_out/r04_list_probe_f32.txt
