#!/bin/bash
# r05be: K7 routing budgets above the defaults (VBUDGET / SBUDGET 256/128 default, 512/128, 1024/128, 256/256), C2 and C4, alternated twice
OUT=gpurun_out/r05be
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1"
for r in 1 2; do
  for cfg in 256_128 512_128 1024_128 256_256; do
    vb=${cfg%_*}; sb=${cfg#*_}
    for w in c2 c4; do
      KPW_SNAPPY_VBUDGET=$vb KPW_SNAPPY_SBUDGET=$sb timeout -k 10 300 $B --workload $w > $OUT/${w}_${cfg}_$r.json 2> $OUT/${w}_${cfg}_$r.err || exit $?
    done
  done
done
