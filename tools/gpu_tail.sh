#!/bin/bash
# the parallel accumulator combine in the list step's final workgroup: parity subset + alternating A/B against the
# HEAD build (build/variants/base_head.so)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "list or contact or domain or golden or ensemble" > gpurun_out/r03h_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03h_tests.log
case $rc in 0) ;; *) exit $rc ;; esac
: > gpurun_out/r03h_ab.txt
for rep in 1 2; do
  bash tools/bench_variants.sh --steps 200 --warmup 50 --c5-steps 0 --cycle-scale 0 --replicas-per-gpu 1 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03h_ab.txt
  bash tools/bench_variants.sh --steps 20 --warmup 5 --c5-steps 0 --cycle-scale 0 || exit 1
  cat gpurun_out/bench_variants.log >> gpurun_out/r03h_ab.txt
done
cat gpurun_out/r03h_ab.txt
