#!/bin/bash
# r05af: job timeline of the bulk multi-page leg (decode + inputs, hand-over); C5 with the boundary
# copy on 4 threads / on one (KPW_PAR_BOUNDS), alternating
OUT=gpurun_out/r05af
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace_bmp.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload c5 --steps 2 --warmup 1"
for r in 1 2; do
  KPW_PAR_BOUNDS=0 timeout -k 10 300 $B > $OUT/c5_p0_$r.json 2> $OUT/c5_p0_$r.err || exit $?
  timeout -k 10 300 $B > $OUT/c5_p1_$r.json 2> $OUT/c5_p1_$r.err || exit $?
done
