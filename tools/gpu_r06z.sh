#!/bin/bash
# round 6: the contact step's batched first probes -- the interphase stage (300k steps) with the default (batched),
# HEAD's build (one probe chain per contact) and the batched build at 3 waves per SIMD for the contact step; the
# last window's table must be identical (sha1); then the contact tests
set -u
o=gpurun_out/r06z
mkdir -p $o
: > $o/stage.txt
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/head.so build/variants/ct3.so; do
  GCS_LIB=$lib timeout -k 10 200 python -u tools/interphase_probe.py 300000 10000 > $o/probe.txt 2>&1 || { echo "probe failed $lib"; tail $o/probe.txt; exit 1; }
  echo "$lib: $(grep -E 'sha1|^contacts=' $o/probe.txt | tr '\n' ' ')" >> $o/stage.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_contacts.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log; cat $o/stage.txt
