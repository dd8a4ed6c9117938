#!/bin/bash
# r04tl: the c2 writer line with the writer's per-job trace (KPW_TRACE=1)
OUT=gpurun_out/r04tl
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w.log 2>&1
