#!/bin/bash
# round 4: the decomposition tests (fused band pack) and the decomposed bench legs (C2: 1 domain over RCCL,
# 2 / 4 / 8 boxes in process; C5: 1 domain over RCCL)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04_domain_tests.log 2>&1 || { tail -30 gpurun_out/r04_domain_tests.log; exit 1; }
tail -2 gpurun_out/r04_domain_tests.log
out=gpurun_out/r04_decomp.log
: > $out
for a in "--decomp 1 --rccl" "--decomp 2" "--decomp 4" "--decomp 8" "--decomp 1 --rccl --config c5"; do
  echo "== $a" >> $out
  timeout -k 10 300 python bench.py $a --steps 400 --warmup 64 > gpurun_out/r04_decomp_tmp.json 2>&1 || { tail -20 gpurun_out/r04_decomp_tmp.json; exit 1; }
  tail -1 gpurun_out/r04_decomp_tmp.json >> $out
done
cut -c1-300 $out
