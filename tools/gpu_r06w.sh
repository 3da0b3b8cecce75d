#!/bin/bash
# round 6: does the tile order matter at C5? reversed, both-ends-inwards against slot order (plane-relative lists)
set -u
STEPS=300 bash tools/c5_variants.sh || { cat gpurun_out/c5_variants.log; exit 1; }
mkdir -p gpurun_out/r06w && cp gpurun_out/c5_variants.log gpurun_out/r06w/c5.txt && cat gpurun_out/r06w/c5.txt
