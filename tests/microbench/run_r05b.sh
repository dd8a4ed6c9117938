#!/bin/bash
# r05b: where the C2 step's close() tail comes from.  KPW_TRACE=1 bench steps (job submit /
# start / encode / append times, close timings) under the default pipeline and variants:
# one encode worker, smaller eager jobs, smaller full jobs.
OUT=gpurun_out/r05b
mkdir -p $OUT
A="--no-resident --no-cpu-baseline --per-record-records 0 --secondary-steps 0 --steps 3 --warmup 1"
KPW_TRACE=1 timeout -k 10 120 python bench.py $A > $OUT/base.log 2>&1 || exit $?
KPW_TRACE=1 KPW_ENCODERS=1 timeout -k 10 120 python bench.py $A > $OUT/enc1.log 2>&1 || exit $?
KPW_TRACE=1 KPW_EAGER_MB=192 timeout -k 10 120 python bench.py $A > $OUT/eager192.log 2>&1 || exit $?
KPW_TRACE=1 KPW_STAGE_FLUSH_MB=512 timeout -k 10 120 python bench.py $A > $OUT/flush512.log 2>&1 || exit $?
timeout -k 10 120 python bench.py $A > $OUT/base_notrace.log 2>&1 || exit $?
