#!/bin/bash
# tools/profile.sh for R = 1 and R = 4, summarised on the box (raw rocprofv3 output exceeds what gpurun copies back)
set -u
tag=${1:?tag}
for R in ${PROFILE_REPLICAS:-1 4}; do
  t=$tag; [ $R -gt 1 ] && t=${tag}_r$R
  REPLICAS=$R bash tools/profile.sh $t || { d=gpurun_out/prof_$t; cp $d/trace.log gpurun_out/${t}_trace.log; cp $d/maps.txt gpurun_out/${t}_maps.txt; rm -rf $d/trace $d/pmc*; exit 1; }
  d=gpurun_out/prof_$t
  # the step kernel of the bench's shape: 4 waves per tile for one trajectory, 2 with replicas (bench.py list_waves)
  W=4; [ $R -gt 1 ] && W=2
  [ "${PREC:-64}" = 64 ] && k="k_lstep<unsigned short, $W, false, false, double, false>" || k="k_lstep<unsigned short, $W, false, false, float, false>"
  k=${KERNEL:-$k}
  python tools/summarize_pmc.py $d --traffic-out gpurun_out/${t}_lstep_traffic.json --kernel "$k" > gpurun_out/${t}_pmc_summary.json || { cp $d/trace.log $d/maps.txt gpurun_out/ 2>/dev/null; exit 1; }
  cp "$(find $d/trace -name '*kernel_stats.csv' | head -n 1)" gpurun_out/${t}_kernel_stats.csv || exit 1
  rm -rf $d
done
