#!/bin/bash
# round 4: fp64 skin x period sweep (4 replicas), the headline with and without the fp32 leg (stream order check),
# the list-deal rows with periods 9 and 10, then the R = 4 rocprofv3 passes (last)
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/skin_sweep.sh 64 "400 10" "450 13" "500 16" "550 19" "600 23" || exit 1
# waves per tile with 4 replicas at fp64 (2: the fp32-tuned default, 4: the single-trajectory shape)
for lw in 2 4 2 4; do
  timeout -k 10 200 python bench.py --no-f32-leg --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window --steps 400 --list-waves $lw > gpurun_out/r04_lw_tmp.json 2>&1 || { tail -20 gpurun_out/r04_lw_tmp.json; exit 1; }
  tail -1 gpurun_out/r04_lw_tmp.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('list_waves $lw: %.4e single %.4e' % (d['value'],c['single_trajectory_value']))" >> gpurun_out/r04_list_waves.log
done
cat gpurun_out/r04_list_waves.log
out=gpurun_out/r04_f32leg_order.log
: > $out
for leg in "" "--no-f32-leg"; do
  timeout -k 10 300 python bench.py --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window --steps 20 --warmup 5 $leg > gpurun_out/r04_leg_tmp.json 2>&1 || { tail -20 gpurun_out/r04_leg_tmp.json; exit 1; }
  tail -1 gpurun_out/r04_leg_tmp.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('leg=[$leg] headline %.4e single %.4e f32 %s' % (d['value'],c['single_trajectory_value'],c.get('f32_value')))" >> $out
done
cat $out
timeout -k 10 900 bash tools/deal_sweep.sh r04_deal "rr 001" "0120123 012012013 0120120123" > gpurun_out/r04_deal.log 2>&1 || { tail -5 gpurun_out/r04_deal.log; exit 1; }
cat gpurun_out/r04_deal.log
