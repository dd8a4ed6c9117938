#!/bin/bash
# r04pp: probe path (dictionary rounds of >= 1024 tiles over the dictionary chunks, few-fragment
# K7 launches straight to the segment kernel): GPU suite, the per-record loop, the full bench line.
OUT=gpurun_out/r04pp
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 3000000 1048576 > $OUT/pr_1m.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench.log 2>&1 || exit $?
