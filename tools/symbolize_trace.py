"""Symbolise the PCs of a crash stack trace ("@ 0x7f.. (unknown)" lines, e.g. rocprofv3's SIGSEGV report) against
the process's /proc/self/maps captured before the crash (bench.py GCS_MAPS_OUT).  The libraries are the image's
own, so this runs in the build container as well as on the GPU box.
usage: python tools/symbolize_trace.py trace.log maps.txt"""
import re
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    maps = []
    for line in open(path):
        p = line.split()
        if len(p) < 6 or not p[5].startswith("/"):
            continue
        lo, hi = (int(x, 16) for x in p[0].split("-"))
        maps.append((lo, hi, int(p[2], 16), p[5]))
    base = {}
    for lo, hi, off, f in maps:  # load base: start of the mapping at file offset 0
        if off == 0 and f not in base:
            base[f] = lo
    return maps, base


def main(trace, maps_path):
    maps, base = load_maps(maps_path)
    pcs = []
    for line in open(trace):
        m = re.search(r"(PC: )?@\s+(0x[0-9a-f]+)", line)
        if m:
            pcs.append((line.rstrip(), int(m.group(2), 16)))
    for line, pc in pcs:
        hit = next(((lo, hi, off, f) for lo, hi, off, f in maps if lo <= pc < hi), None)
        if hit is None:
            print(f"{line}\n    -> not in a file mapping")
            continue
        f = hit[3]
        rel = pc - base.get(f, hit[0] - hit[2])
        try:
            out = subprocess.run([SYM, f"--obj={f}", "--demangle", "--functions=linkage", hex(rel)],
                                 capture_output=True, text=True, timeout=60).stdout.strip().split("\n")
        except (OSError, subprocess.TimeoutExpired):
            out = ["?"]
        print(f"{line}\n    -> {f} +{rel:#x}: {out[0][:160]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
