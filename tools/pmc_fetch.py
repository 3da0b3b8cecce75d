"""Average FETCH_SIZE / WRITE_SIZE / TCC hit counters per dispatch of the kernels whose names start with a prefix, from
rocprofv3 --pmc output directories.  usage: python tools/pmc_fetch.py <kernel prefix> <dir> [<dir> ...]"""
import csv
import glob
import sys
from collections import defaultdict

from summarize_pmc import short

prefix = sys.argv[1]
acc = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if short(row["Kernel_Name"]).startswith(prefix):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {c: sum(v) / len(v) for c, v in acc.items()}
if "FETCH_SIZE" in out:
    out["fetch_MB_corrected"] = 2 * out["FETCH_SIZE"] * 1024 / 1e6
if "WRITE_SIZE" in out:
    out["write_MB"] = out["WRITE_SIZE"] * 1024 / 1e6
print({k: round(v, 3) for k, v in out.items()})
