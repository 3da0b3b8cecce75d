#!/bin/bash
# round 6: C5, chunks of 4 / 16 / 64 tiles dealt round-robin to the XCDs (plane-relative lists) vs interleaved tiles
set -u
STEPS=300 bash tools/c5_variants.sh || { cat gpurun_out/c5_variants.log; exit 1; }
mkdir -p gpurun_out/r06y && cp gpurun_out/c5_variants.log gpurun_out/r06y/c5.txt && cat gpurun_out/r06y/c5.txt
