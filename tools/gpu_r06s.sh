#!/bin/bash
# round 6: C5 fp64 L2 experiments -- write-through (sc1) slot-order position stores, the XCD remap off -- rate
# (alternating) and FETCH / WRITE / TCC hits per k_lstep launch for each build
set -u
o=gpurun_out/r06s
mkdir -p $o
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0  # (as tools/profile.sh)
STEPS=300 bash tools/c5_variants.sh || { cat gpurun_out/c5_variants.log; exit 1; }
cp gpurun_out/c5_variants.log $o/rates.txt
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
  t=$(basename $lib .so)
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    p=$o/pmc_${t}_${ctr%% *}
    GCS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr -d $p -o run --output-format csv -- python3 bench.py --config c5 --replicas-per-gpu 1 --cpu-budget 0 --no-start-window --c5-steps 0 --cycle-scale 0 --no-f32-leg --steps 100 --warmup 20 > $p.log 2>&1 || { echo "pmc $t $ctr failed"; tail -5 $p.log; exit 1; }
  done
  echo "$t $(python3 tools/pmc_fetch.py 'k_lstep<ListRel16, 4, false' $o/pmc_${t}_*)" >> $o/fetch.txt
  rm -rf $o/pmc_${t}_*
done
cat $o/rates.txt $o/fetch.txt
