#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
#   pass 0: kernel trace + stats (durations)
#   pass 1..: PMC counters, one pass each (no tracing domains combined with --pmc)
# Outputs under gpurun_out/prof_<tag>/ ; summarise with tools/summarize_pmc.py.
set -u
tag=${1:-r01}
steps=${STEPS:-300}
root=$(pwd)
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
bench=(python3 "$root/bench.py" --steps "$steps" --warmup 50 --cpu-budget 0 --profile-steps 10 --no-start-window --replicas-per-gpu "${REPLICAS:-1}" --c5-steps 0 --cycle-scale 0 --precision "${PREC:-64}" --no-f32-leg --config "${CONFIG:-c2}")
# rocprofv3 --kernel-trace segfaults inside hipGraphLaunch when HIP dispatches a graph's pre-captured AQL packets
# (the default graph packet capture): the fault is in librocprofiler-sdk's queue-write interceptor, which reads a
# packet header one page past the array it is handed (profiles/r04_rocprof_crash.txt).  Profiling runs
# turn the capture off (every graph node dispatched on its own); GCS_PROFILE_PACKET_CAPTURE=1 keeps it.
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=${GCS_PROFILE_PACKET_CAPTURE:-0}
# (GCS_MAPS_OUT: the process's memory map before the first warm-up step, to symbolise a crash trace's PCs)
GCS_MAPS_OUT=$out/maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- "${bench[@]}" > "$out/trace.log" 2>&1 || exit $?
i=0
for ctrs in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d "$out/pmc$i" -o run --output-format csv -- "${bench[@]}" > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo "profile done: $out"
