#!/bin/bash
# List-build chunk deal (GCS_OPT_LIST_DEAL) A/B on one box, alternating: the 4-replica bench (2 waves per tile) and the
# single trajectory (4 waves per tile).   bash tools/deal_sweep.sh <tag> "<R=4 patterns>" "<R=1 patterns>"
set -u
tag=${1:?tag}; p4=${2:-"rr 001 00101"}; p1=${3:-"rr 0120123 012012013"}
out=gpurun_out/$tag; mkdir -p $out
common="--cpu-budget 0 --c5-steps 0 --cycle-scale 0 --no-start-window"
for rep in 1 2; do
  for p in $p4; do
    o=""; [ "$p" != rr ] && o="--engine-opt list_deal=d:$p"; [ "$p" = rr ] && o="--engine-opt list_deal=0"
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 $common $o > $out/r4_${p}_$rep.log 2>&1 || exit 1
  done
  for p in $p1; do
    o=""; [ "$p" != rr ] && o="--engine-opt list_deal=d:$p"; [ "$p" = rr ] && o="--engine-opt list_deal=0"
    timeout -k 10 120 python bench.py --steps 200 --warmup 50 --replicas-per-gpu 1 $common $o > $out/r1_${p}_$rep.log 2>&1 || exit 1
  done
done
python3 - $out <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(os.path.basename(f), "no line"); continue
    d = json.loads(l[-1])
    print("%-28s %.4e  force_ms %.4f" % (os.path.basename(f), d["value"], d["roofline"]["force_ms"]))
PY
