#!/bin/bash
# r04f: full GPU suite, traced C2 writer (async writes), default bench line.  From the repo root.
OUT=gpurun_out/r04f
mkdir -p $OUT
timeout -k 10 1800 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/trace_c2.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/mp_leg.py 10000000 1048576 2 > $OUT/mp_trace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mp_prof -o run -- python tests/microbench/mp_leg.py 10000000 1048576 1 > $OUT/mp_prof.log 2>&1
