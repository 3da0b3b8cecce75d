#!/bin/bash
# retry a gpurun call only while the pool reports no box (the command never ran); stop at any other outcome
out=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  if grep -q "status=transient" $out; then sleep 200; continue; fi
  break
done
tail -4 $out
