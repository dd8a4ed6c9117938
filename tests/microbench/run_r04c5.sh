#!/bin/bash
# r04c5: C5 writer line, final build vs the round's starting build (libkpw_r04pre), alternating
OUT=gpurun_out/r04c5
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/cur_$r.log 2>&1 || exit $?
  KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_r04pre.so timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/pre_$r.log 2>&1 || exit $?
done
