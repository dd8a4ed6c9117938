#!/bin/bash
# r04eg: eager job size A/B on the c2 writer line (alternating, 2 reps)
OUT=gpurun_out/r04eg2
mkdir -p $OUT
for r in 1 2 3; do
  for mb in 512 384; do
    KPW_EAGER_MB=$mb timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_${mb}_$r.log 2>&1 || exit $?
  done
done
