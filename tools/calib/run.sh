#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over build/fetch_calib (tools/calib/fetch_calib.hip); summary:
# python tools/calib/summarize.py gpurun_out/calib
set -u
out=$(pwd)/gpurun_out/calib
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $GRAFT_REPO_ROOT/build/fetch_calib > $out/trace.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $out/pmc1 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/fetch_calib > $out/pmc1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $out/pmc2 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/fetch_calib > $out/pmc2.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $out/pmc3 -o run --output-format csv -- $GRAFT_REPO_ROOT/build/fetch_calib > $out/pmc3.log 2>&1 || echo "pass 3 failed"
echo calib done
