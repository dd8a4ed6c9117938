#!/bin/bash
# r06q: bulk multi-page leg, speculative horizon 12 vs 25 %, three alternations, 3 timed steps each
OUT=gpurun_out/r06q
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --steps 2 --warmup 1 --secondary-steps 3"
for r in 1 2 3; do
  for p in 12 25; do
    KPW_BENCH_LEGS=bulk_multipage KPW_MP_HORIZON_PCT=$p timeout -k 10 300 python3 bench.py $A > $OUT/bulk_p${p}_$r.json 2> $OUT/bulk_p${p}_$r.err || exit 1
  done
done
echo done
