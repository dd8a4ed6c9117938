#!/bin/bash
# r05an: C2 writer job timeline (KPW_TRACE) of the current build
OUT=gpurun_out/r05an
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload c2 --steps 2 --warmup 1 > $OUT/c2.json 2> $OUT/c2_trace.log || exit $?
