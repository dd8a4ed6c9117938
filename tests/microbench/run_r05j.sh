#!/bin/bash
# r05j: where the bulk multi-page writer path (C2 Rec8, 1 MiB pages, 128 MiB row groups) spends
# its time: the leg alone (20 M records), a kernel trace of it, and a writer trace
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 2 > $OUT/leg.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bmp -- python3 \
    tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/prof.log 2>&1 || exit $?
