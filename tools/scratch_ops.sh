#!/bin/bash
# per kernel: scratch instructions actually in the code object vs the reserved private-segment frame
# (Makefile resource-usage reports the frame; a frame with no scratch_load/store in the body costs nothing)
set -eu
src=$(cd "$(dirname "$0")/../3d-genome-cycle_amd/csrc" && pwd)
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-result "$@" \
  --cuda-device-only -S -o /tmp/gcs_kernels_scratch.s "$src/kernels.hip"
awk '
/^_ZN3gcs12_GLOBAL__N_1[0-9]+k_(force|lstep|lbuild|lupdate|eval64)[^:]*:/ {name=$1; n=0; next}
name!="" && /scratch_(load|store)/ {n++}
name!="" && /^\.Lfunc_end/ {cnt[name]=n; name=""}
/\.amdhsa_kernel / {k=$2}
/\.amdhsa_private_segment_fixed_size/ {ps[k]=$2}
END {for (x in cnt) {y=x; sub(":","",y); printf "%-60s scratch_ops=%-3d frame_B=%s\n", substr(y,20,60), cnt[x], ps[y]}}' \
  /tmp/gcs_kernels_scratch.s | sort
