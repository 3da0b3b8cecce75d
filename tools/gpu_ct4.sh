#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "contact or cli" > gpurun_out/r03l_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03l_tests.log
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/interphase_probe.py 20000 1000 > gpurun_out/r03l_interphase_probe.txt 2>&1 || exit 1
grep -E "contacts=|contacts_accumulate" gpurun_out/r03l_interphase_probe.txt
for k in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --c5-steps 0 --cycle-scale 0 > gpurun_out/r03l_bench$k.log 2>&1 || exit 1
tail -1 gpurun_out/r03l_bench$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4e contacts_update_ms %.4f' % (d['value'], d['config']['contacts_update_ms']))"
done
