#!/bin/bash
# One GPU call: a parity subset, the driver-shaped bench (R = 4 and R = 1), and rocprofv3 kernel stats (R = 1, R = 4).
#   bash tools/gpu_quick.sh <tag> [pytest -k expression]
set -u
tag=${1:?tag}
sel=${2:-"list or contact or parity_long"}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$sel" \
  > $out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 $out/${tag}_tests.log; exit 1; }
tail -2 $out/${tag}_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --c5-steps 0 --cycle-scale 0 > $out/${tag}_bench.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 50 --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --replicas-per-gpu 1 --no-start-window > $out/${tag}_bench_r1.log 2>&1 || exit 1
for R in 1 4; do
  GCS_BENCH_DENSE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_${tag}_r$R -o run --output-format csv -- \
    python3 bench.py --steps 300 --warmup 50 --cpu-budget 0 --c5-steps 0 --cycle-scale 0 --profile-steps 10 \
    --no-start-window --replicas-per-gpu $R > $out/${tag}_prof_r$R.log 2>&1 || exit 1
  cp "$(find $out/prof_${tag}_r$R -name '*kernel_stats.csv' | head -n 1)" $out/${tag}_r${R}_kernel_stats.csv
  rm -rf $out/prof_${tag}_r$R
done
python3 - "$tag" <<'PY'
import json, sys, csv
tag = sys.argv[1]
for f in (f"gpurun_out/{tag}_bench.log", f"gpurun_out/{tag}_bench_r1.log"):
    l = [x for x in open(f) if x.startswith("{")][-1]
    d = json.loads(l)
    print(f, "value %.3e single %.3e replays %s force_ms %.4f" % (d["value"], d["config"]["single_trajectory_value"],
          d.get("graph_replays"), d["roofline"]["force_ms"]))
for R in (1, 4):
    for row in csv.DictReader(open(f"gpurun_out/{tag}_r{R}_kernel_stats.csv")):
        if float(row["Percentage"]) > 1:
            print(R, row["Name"].split("(")[0][-60:], row["Calls"], "%.2f us" % (float(row["AverageNs"]) / 1e3))
PY
