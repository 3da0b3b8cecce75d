"""Kernel register / scratch / occupancy table from `make -C 3d-genome-cycle_amd/csrc resource-usage` output (stdin).
usage: make -s -C 3d-genome-cycle_amd/csrc resource-usage | python tools/resource_table.py [name-filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].replace("\\", "")] = int(m.group(1))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    d = d.replace("gcs::(anonymous namespace)::", "")
    if flt in d:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>4} B scratch occ {r.get('Occupancy', '?'):>2} "
              f"lds {r.get('LDS', '?'):>6}  {d[:150]}")
