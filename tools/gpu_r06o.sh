#!/bin/bash
# round 6: the C5 fp64 list-step profile (kernel trace + PMC passes, one domain, the bench's
# single-trajectory shape at C5), summarised on the box
set -u
CONFIG=c5 STEPS=${STEPS:-200} PROFILE_REPLICAS=1 KERNEL="k_lstep<ListRel16, 4" bash tools/profile_round.sh r06_c5 || { echo "c5 profile failed"; exit 1; }
