#!/bin/bash
# k_lbuild / k_lstep average durations (rocprofv3 kernel stats, 4 replicas) for the default library and each
# build/variants/*.so
set -u
shopt -s nullglob
out=gpurun_out/lbuild_times.log
: > $out
export TMPDIR=/tmp
i=0
for lib in 3d-genome-cycle_amd/gcs/libgcs.so build/variants/*.so; do
  i=$((i+1))
  echo "== $lib" >> $out
  GCS_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lbt$i -o run --output-format csv -- python3 bench.py --steps 300 --warmup 50 --cpu-budget 0 --no-start-window > gpurun_out/lbt$i.log 2>&1 || { echo failed >> $out; exit 1; }
  python3 - gpurun_out/lbt$i >> $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_lbuild" in r["Name"] or "k_lstep" in r["Name"]:
        print(r["Name"].replace("void gcs::(anonymous namespace)::", "").split("(")[0], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  grep '^{"metric"' gpurun_out/lbt$i.log | tail -1 | python3 -c "import json,sys; print('value %.3e' % json.loads(sys.stdin.read())['value'])" >> $out
  rm -f gpurun_out/lbt$i/*/*kernel_trace.csv
done
