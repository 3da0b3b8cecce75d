"""Per calibration kernel (tools/calib/fetch_calib.hip): the counters per dispatch against the bytes it requests.
usage: python tools/calib/summarize.py gpurun_out/calib"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
GiB = 1 << 30
count = 32 << 20
want = {  # kernel name fragment -> (bytes requested, what)
    "k_stream<HIP_vector_type<unsigned int, 4u>": (GiB, "stream 16 B/lane"),
    "k_stream<HIP_vector_type<unsigned int, 2u>": (GiB, "stream 8 B/lane"),
    "k_stream<unsigned short>": (GiB, "stream 2 B/lane"),
    "k_gather<Rec32>": (32 * count, "gather 32-B records"),
    "k_gather<HIP_vector_type<unsigned int, 4u>": (16 * count, "gather 16-B records"),
    "k_gather<unsigned short>": (2 * count, "gather 2-B records"),
    "k_write16": (GiB, "write 16 B/lane"),
}
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
dur = {}
for f in glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        dur[row["Name"]] = float(row["AverageNs"]) / 1e3
print("%-22s %10s %12s %12s %9s %9s %12s %8s" % ("kernel", "req MB", "FETCH MB", "WRITE MB", "FETCH/req", "2F/req",
                                                 "RDREQ(x64)MB", "avg us"))
for frag, (req, what) in want.items():
    k = next((n for n in vals if frag in n), None)
    if k is None:
        print(what, "missing")
        continue
    c = {n: sum(v) / len(v) for n, v in vals[k].items()}
    fetch = c.get("FETCH_SIZE", float("nan")) * 1024
    write = c.get("WRITE_SIZE", float("nan")) * 1024
    rd = c.get("TCC_EA0_RDREQ_sum", float("nan")) * 64
    us = next((v for n, v in dur.items() if frag in n), float("nan"))
    print("%-22s %10.1f %12.1f %12.1f %9.3f %9.3f %12.1f %8.1f" % (what, req / 1e6, fetch / 1e6, write / 1e6, fetch / req,
                                                                   2 * fetch / req, rd / 1e6, us))
