#!/bin/bash
# r04pr: kernel trace of the per-record loop with 1 MiB pages (page-size probes).
OUT=gpurun_out/r04pr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
KPW_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tests/microbench/pr_leg.py 1000000 1048576 > $OUT/pr.log 2>&1
