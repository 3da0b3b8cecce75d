#!/bin/bash
# round 4: 16-bit relative list entries beyond 65,536 particles (C5): the list tests, the C5 leg, the C5 PMC passes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_list.py tests/test_gpu_contacts.py tests/test_gpu_domain.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c5 or relative or ragged or c2 or relaxation or decomposed_c5 or bitwise" > gpurun_out/r04k_tests.log 2>&1 || { tail -30 gpurun_out/r04k_tests.log; exit 1; }
tail -2 gpurun_out/r04k_tests.log
timeout -k 10 400 python bench.py --no-f32-leg --cycle-scale 0 --cpu-budget 0 --no-start-window --steps 20 --warmup 5 > gpurun_out/r04k_bench.log 2>&1 || { tail -20 gpurun_out/r04k_bench.log; exit 1; }
tail -1 gpurun_out/r04k_bench.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('headline %.4e single %.4e' % (d['value'],c['single_trajectory_value'])); print('c5', c['c5'])"
bash tools/gpu_r04j.sh
