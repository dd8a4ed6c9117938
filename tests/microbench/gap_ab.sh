#!/bin/bash
# Test infrastructure: A/B of the adaptive carry gap (KPW_GAP_ADAPT=0 = fixed 2 x blockSize gap)
# on the C3 / C2 writer benches, alternating, with the writer trace on for the rebuild counts.
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for g in 0 1; do
    KPW_GAP_ADAPT=$g KPW_TRACE=1 timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline --no-resident --per-record-records 0 --steps 3 --warmup 1 > gpurun_out/gap_c3_${g}_$r.log 2>&1
  done
done
KPW_GAP_ADAPT=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-resident --per-record-records 0 > gpurun_out/gap_c2_1.log 2>&1
