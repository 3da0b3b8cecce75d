#!/usr/bin/env python3
"""Average per-dispatch counters / durations per kernel from a tools/profile.sh output directory.

    python tools/summarize_pmc.py gpurun_out/prof_r01 [--traffic-out profiles/pmc_force_traffic.json] [--kernel k_lstep]

HBM traffic per force launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads (MI355X_MICROARCH.md "HBM"); both counters are fabric-side (L2 misses, Infinity Cache hits
included).
"""
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
    return out


def force_traffic(out, kernel_prefix="k_force<0"):
    for k, v in out["kernels"].items():
        if k.startswith(kernel_prefix) and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            fetch = 2.0 * v["FETCH_SIZE"] * 1024.0
            write = v["WRITE_SIZE"] * 1024.0
            return {"kernel": k, "bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch,
                    "write_bytes": write, "FETCH_SIZE_KiB": v["FETCH_SIZE"], "WRITE_SIZE_KiB": v["WRITE_SIZE"],
                    "avg_us": v.get("avg_us"), "correction": "2 x FETCH_SIZE (gfx950) + WRITE_SIZE"}
    return None


if __name__ == "__main__":
    res = main(sys.argv[1])
    if "--traffic-out" in sys.argv:
        prefix = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_force<0"
        t = force_traffic(res, prefix)
        if t is None:
            sys.exit(f"no {prefix} FETCH_SIZE/WRITE_SIZE in the profile")
        t["source"] = sys.argv[1]
        with open(sys.argv[sys.argv.index("--traffic-out") + 1], "w") as f:
            json.dump(t, f, indent=1)
            f.write("\n")
