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
bench=(python3 "$root/bench.py" --steps "$steps" --warmup 50 --cpu-budget 0 --profile-steps 10 --no-start-window --replicas-per-gpu "${REPLICAS:-1}" --c5-steps 0 --cycle-scale 0 --precision "${PREC:-64}" --no-f32-leg)
# the engines' density probe (GCS_OPT_DENSE_NEIGHBORS) makes rocprofv3 --kernel-trace segfault in the first graph
# launch (engine.hip probe_density); the C2 window is list-step territory either way (25 neighbours)
export GCS_BENCH_DENSE=0
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
