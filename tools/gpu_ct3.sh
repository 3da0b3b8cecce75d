#!/bin/bash
# kernel durations of the interphase stage's step loop with the contact map (rocprofv3 kernel trace)
export TMPDIR=/tmp
out=gpurun_out/prof_r03e_ip
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 tools/interphase_probe.py 6000 200 > gpurun_out/r03e_ip_prof.log 2>&1 || { tail -20 gpurun_out/r03e_ip_prof.log; exit 1; }
f=$(find $out -name '*kernel_stats.csv' | head -n 1)
cp "$f" gpurun_out/r03e_interphase_kernel_stats.csv
rm -rf $out
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r03e_interphase_kernel_stats.csv")):
    print(r["Name"].split("(")[0][-70:], r["Calls"], "%.1f us avg" % (float(r["AverageNs"]) / 1e3), "%.1f%%" % float(r["Percentage"]))
PY
