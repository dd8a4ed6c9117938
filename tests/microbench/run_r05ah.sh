#!/bin/bash
# r05ah: kernel trace of the bulk multi-page leg (20 M records, 1 timed step)
OUT=gpurun_out/r05ah
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bmp -- python3 tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/prof.log 2>&1 || exit $?
