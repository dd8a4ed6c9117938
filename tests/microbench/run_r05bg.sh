#!/bin/bash
# r05bg: the bench line's c5 key with the c5 leg before / after the c4 and bulk_multipage legs
# (KPW_BENCH_C5_FIRST, a temporary bench knob removed after this measurement), alternated twice
OUT=gpurun_out/r05bg
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --steps 2 --warmup 1"
for r in 1 2; do
  for f in 0 1; do
    KPW_BENCH_C5_FIRST=$f timeout -k 10 400 $B > $OUT/first${f}_$r.json 2> $OUT/first${f}_$r.err || exit $?
  done
done
