#!/bin/bash
# C5 at the new defaults: 2 waves per tile vs 4 (fp64 / fp32), then the fp64 PMC passes (tools/profile.sh, CONFIG=c5)
set -u
mkdir -p gpurun_out
out=gpurun_out/r04s_bench.log
: > $out
run() {
  local label=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-f32-leg "$@" 2>&1 | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$label value %.3e force_us %.2f' % (d['value'], 1e3*d['roofline']['force_ms']))" >> $out
}
c5="--config c5 --replicas-per-gpu 1 --steps 200 --warmup 30 --no-start-window"
run "c5 f64 list waves 2" $c5 --precision 64 --list-waves 2 || exit 1
run "c5 f64 list waves 4" $c5 --precision 64 --list-waves 4 || exit 1
run "c5 f32 list waves 2" $c5 --precision 32 --list-waves 2 || exit 1
run "c5 f32 list waves 4" $c5 --precision 32 --list-waves 4 || exit 1
STEPS=100 CONFIG=c5 PREC=64 bash tools/profile.sh r04s_c5 > gpurun_out/r04s_prof.log 2>&1 || { tail -20 gpurun_out/r04s_prof.log; exit 1; }
d=gpurun_out/prof_r04s_c5
python tools/summarize_pmc.py $d --traffic-out gpurun_out/r04s_c5_lstep_traffic.json \
  --kernel "k_lstep<ListRel16, 4, false, false, double, false>" > gpurun_out/r04s_c5_pmc_summary.json || exit 1
cp "$(find $d/trace -name '*kernel_stats.csv' | head -n 1)" gpurun_out/r04s_c5_kernel_stats.csv || exit 1
rm -rf $d
