#!/bin/bash
# r05bb: the final C2 profile set (profiles/profile_round.sh r05az c2), then eager-job size at
# eight hardware queues (KPW_EAGER_MB 384 / 512 / 768, alternated twice) on C2
set -e
bash profiles/profile_round.sh r05az c2
OUT=gpurun_out/r05bb
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 4 --warmup 1"
for r in 1 2; do
  for e in 384 512 768; do
    KPW_EAGER_MB=$e timeout -k 10 300 $B > $OUT/c2_e${e}_$r.json 2> $OUT/c2_e${e}_$r.err
  done
done
