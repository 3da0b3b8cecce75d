#!/bin/bash
# retry a gpurun call only while the pool reports no box (the command never ran); stop at any other outcome
out=$1; shift
for i in $(seq 1 ${RETRIES:-15}); do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  if grep -q "status=transient" $out; then sleep 200; continue; fi
  break
done
tail -4 $out
