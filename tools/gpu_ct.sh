#!/bin/bash
# contact-step graph change: the contact / list / CLI tests, the interphase-stage probe, the driver bench
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "contact or list or cli or small or golden" > gpurun_out/r03d_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03d_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/interphase_probe.py 20000 1000 > gpurun_out/r03d_interphase_probe.txt 2>&1 || { tail -20 gpurun_out/r03d_interphase_probe.txt; exit 1; }
cat gpurun_out/r03d_interphase_probe.txt
exit $rc
grep "^bench:" gpurun_out/r03d_bench.log
tail -1 gpurun_out/r03d_bench.log
exit $rc
