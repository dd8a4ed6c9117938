#!/bin/bash
# r05aw: C5 and C4 with GPU_MAX_HW_QUEUES 4 vs 8, alternated (paired A/B on one box)
OUT=gpurun_out/r05aw
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1"
for r in 1 2 3; do
  for q in 4 8; do
    for w in c5 c4; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B --workload $w > $OUT/${w}_q${q}_$r.json 2> $OUT/${w}_q${q}_$r.err || exit $?
    done
  done
done
