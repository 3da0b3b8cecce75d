#!/bin/bash
# round 4: the decomposition tests (fused band pack) and the decomposed bench legs (C2: 1 domain over RCCL,
# 2 / 4 / 8 boxes in process; C5: 1 domain over RCCL)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04_domain_tests.log 2>&1 || { tail -30 gpurun_out/r04_domain_tests.log; exit 1; }
tail -2 gpurun_out/r04_domain_tests.log
out=gpurun_out/r04_decomp.log
: > $out
for a in "--decomp 1 --rccl" "--decomp 1 --rccl --precision 32" "--decomp 8" "--decomp 8 --precision 32" "--decomp 1 --rccl --config c5 --precision 32" "--decomp 1 --rccl --config c5"; do
  echo "== $a" >> $out
  timeout -k 10 300 python bench.py $a --steps 400 --warmup 64 > gpurun_out/r04_decomp_tmp.json 2>&1 || { tail -20 gpurun_out/r04_decomp_tmp.json; exit 1; }
  tail -1 gpurun_out/r04_decomp_tmp.json >> $out
done
cut -c1-300 $out
# C5 fp64 (the engine default) vs fp32 list step: kernel durations (rocprofv3 kernel trace, last: may abort)
for p in 64 32; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_$p -o run --output-format csv -- python3 bench.py --config c5 --precision $p --replicas-per-gpu 1 --steps 64 --warmup 64 --no-f32-leg --c5-steps 0 --cycle-scale 0 --cpu-budget 0 --no-start-window --fused 3 --engine-opt dense_neighbors=0 > gpurun_out/r04_c5prof_$p.log 2>&1 || { tail -20 gpurun_out/r04_c5prof_$p.log; exit 1; }
  f=$(find gpurun_out/c5prof_$p -name '*kernel_stats.csv' | head -n 1); cp "$f" gpurun_out/r04_c5_f${p}_kernel_stats.csv; rm -rf gpurun_out/c5prof_$p
  head -8 gpurun_out/r04_c5_f${p}_kernel_stats.csv | cut -c1-200
done
