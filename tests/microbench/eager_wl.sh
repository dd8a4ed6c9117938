#!/bin/bash
# Test infrastructure: writer-path bench of C3/C4/C5 with and without eager jobs (KPW_EAGER_MB).
set -e
mkdir -p gpurun_out
for wl in c3 c4 c5; do
  for e in -1 512; do
    KPW_EAGER_MB=$e timeout -k 10 300 python bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 > gpurun_out/eagerwl_${wl}_$e.log 2>&1
  done
done
