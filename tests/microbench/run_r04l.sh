#!/bin/bash
# r04l: the per-record loop with page cuts (C2 Rec8, 1 MiB and 64 KiB pages in 128 MiB row
# groups) under KPW_TRACE (probe count / time) and under rocprofv3 (kernels per probe).
OUT=gpurun_out/r04l
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 3000000 1048576 > $OUT/pr_1m.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 300000 65536 > $OUT/pr_64k.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_1m -o run -- python tests/microbench/pr_leg.py 1000000 1048576 > $OUT/prof_1m.log 2>&1
