#!/bin/bash
# r04eg3: eager job size 384 vs 512 MiB on the C3 / C4 / C5 writer lines (alternating)
OUT=gpurun_out/r04eg3
mkdir -p $OUT
for wl in c3 c4 c5; do
  for r in 1 2; do
    for mb in 512 384; do
      KPW_EAGER_MB=$mb timeout -k 10 300 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_${wl}_${mb}_$r.log 2>&1 || exit $?
    done
  done
done
