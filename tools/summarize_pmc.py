#!/usr/bin/env python3
"""Average per-dispatch counters / durations per kernel from a tools/profile.sh output directory."""
import csv
import glob
import json
import sys
from collections import defaultdict


def short(name):
    return name.replace("void ", "").replace("gcs::(anonymous namespace)::", "").split("(")[0]


def main(d):
    out = {"kernels": {}}
    stats = glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True)
    for row in csv.DictReader(open(stats[0])) if stats else []:
        out["kernels"].setdefault(short(row["Name"]), {}).update(
            {"calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3, "pct": float(row["Percentage"])})
    for f in sorted(glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True)):
        acc = defaultdict(lambda: defaultdict(list))
        for row in csv.DictReader(open(f)):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, ctrs in acc.items():
            for c, v in ctrs.items():
                out["kernels"].setdefault(k, {})[c] = sum(v) / len(v)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
