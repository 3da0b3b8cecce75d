#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "contact or cli or store or golden" > gpurun_out/r03i_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03i_tests.log
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/interphase_probe.py 20000 1000 > gpurun_out/r03i_interphase_probe.txt 2>&1 || exit 1
grep -E "contacts=|contacts_accumulate" gpurun_out/r03i_interphase_probe.txt
