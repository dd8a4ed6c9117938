#!/bin/bash
# r05t: where the GZIP writer's time goes (kernel trace of the 10 M-record gzip leg)
OUT=gpurun_out/r05t
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o gz -- python3 \
    tests/microbench/gzip_leg.py 10000000 > $OUT/gz_prof.log 2>&1 || exit $?
