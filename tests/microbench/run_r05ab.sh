#!/bin/bash
# r05ab: multi-page jobs sized to the last row group; tail rule "fewer records than the row group"
OUT=gpurun_out/r05ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/leg_$r.log 2>&1 || exit $?
done
