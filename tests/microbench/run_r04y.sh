#!/bin/bash
# r04y: the planner changes in the writer: c2 / c3 writer lines, the per-record multi-page loop,
# and a kernel trace of the c2 writer (dispatches per job).
OUT=gpurun_out/r04y
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_c3.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 3000000 1048576 > $OUT/pr_1m.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/w_prof -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/w_prof.log 2>&1
