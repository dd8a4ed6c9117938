#!/bin/bash
# r04bm: kernel trace of the bulk multi-page leg (1 MiB pages)
OUT=gpurun_out/r04bm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
KPW_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/bm.log 2>&1
