#!/bin/bash
# r04wl: final build, the other workloads' writer lines (C3, C4, C5) and resident C3 / C4
OUT=gpurun_out/r04wl
mkdir -p $OUT
for wl in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --per-record-records 0 --secondary-steps 0 > $OUT/w_$wl.log 2>&1 || exit $?
done
