#!/bin/bash
# r05m: C5 / C2 writer lines, the r05a library (KPW_GPU_LIB) against the current tree, alternating
OUT=gpurun_out/r05m
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0"
OLD=tests/microbench/build/libvar/libkpw_r05a.so
for r in 1 2; do
  for w in c5 c2; do
    KPW_GPU_LIB=$OLD timeout -k 10 300 $B --workload $w --steps 3 --warmup 1 > $OUT/${w}_old$r.json 2> $OUT/${w}_old$r.err || exit $?
    timeout -k 10 300 $B --workload $w --steps 3 --warmup 1 > $OUT/${w}_new$r.json 2> $OUT/${w}_new$r.err || exit $?
  done
done
