#!/bin/bash
OUT=gpurun_out/r04g
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/mp_leg.py 10000000 1048576 3 > $OUT/mp_trace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mp_prof -o run -- python tests/microbench/mp_leg.py 10000000 1048576 2 > $OUT/mp_prof.log 2>&1
