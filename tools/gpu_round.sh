#!/bin/bash
# one GPU call: the -m gpu suite, then the default bench line (and optionally a rocprofv3 pass: `prof`)
TAG=${TAG:-r04}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
# a failed assertion (rc 1) still lets the bench run; a crash, abort or time limit ends the call
case $rc in 0|1) ;; *) echo "tests ended with rc=$rc"; exit $rc ;; esac
if [ "${NOBENCH:-0}" = 0 ]; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log
fi
if [ "${1:-}" = prof ]; then
  bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
  tail -3 gpurun_out/${TAG}_profile.log
fi
