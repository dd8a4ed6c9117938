#!/bin/bash
# r05ar: C4 line A/B: stream pool and length preparation on / off
OUT=gpurun_out/r05ar
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload c4 --steps 3 --warmup 1"
for r in 1 2; do
  timeout -k 10 300 $B > $OUT/c4_base_$r.json 2> $OUT/c4_base_$r.err || exit $?
  KPW_STREAM_POOL=0 timeout -k 10 300 $B > $OUT/c4_nopool_$r.json 2> $OUT/c4_nopool_$r.err || exit $?
  KPW_PREP_LENGTHS=0 timeout -k 10 300 $B > $OUT/c4_noprep_$r.json 2> $OUT/c4_noprep_$r.err || exit $?
done
KPW_TRACE=1 timeout -k 10 300 $B > $OUT/c4_trace.json 2> $OUT/c4_trace.log || exit $?
