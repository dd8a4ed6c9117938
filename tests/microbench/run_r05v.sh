#!/bin/bash
# r05v: a smaller first job per file (KPW_FIRST_EAGER_MB) — C2 / C3 / C5 A/B, alternating
OUT=gpurun_out/r05v
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for r in 1 2; do
  for w in c2 c3; do
    for f in 0 160 256; do
      KPW_FIRST_EAGER_MB=$f timeout -k 10 300 $B --workload $w --steps 4 --warmup 1 > $OUT/${w}_f${f}_$r.json 2> $OUT/${w}_f${f}_$r.err || exit $?
    done
  done
done
