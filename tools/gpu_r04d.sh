#!/bin/bash
# round 4: (1) graph packet capture on / off on the fp64 bench (does the profiling setting change the step?),
# (2) the rocprofv3 passes at R = 1 and R = 4 with the capture off (tools/profile.sh), last
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r04_capture_ab.log
: > $out
for c in 1 0 1 0; do
  echo "== DEBUG_CLR_GRAPH_PACKET_CAPTURE=$c" >> $out
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$c timeout -k 10 200 python bench.py --no-f32-leg --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window --steps 400 > gpurun_out/r04_cap_tmp.json 2>&1 || { tail -20 gpurun_out/r04_cap_tmp.json; exit 1; }
  tail -1 gpurun_out/r04_cap_tmp.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('value %.4e single %.4e k_lstep %.2f us' % (d['value'],c['single_trajectory_value'],1e3*d['roofline']['force_ms']))" >> $out
done
cat $out
bash tools/profile_round.sh ${TAG:-r04} > gpurun_out/${TAG:-r04}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG:-r04}_profile.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04}_profile.log
