#!/bin/bash
# run a gpurun command, retrying only while no GPU slot is free (exit 3 / transient queue)
out=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "GPU slot(s) on this pod are busy\|no box\|status=transient" $out && [ $rc -ne 0 ]; then sleep 90; continue; fi
  echo "RC=$rc" >> $out
  exit $rc
done
