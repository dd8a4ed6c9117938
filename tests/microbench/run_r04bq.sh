#!/bin/bash
# r04bq: multi-page planners with per-column inputs loaded once: GPU suite, planner profile, bulk leg
OUT=gpurun_out/r04bq
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
true
timeout -k 10 300 python3 tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/bm.log 2>&1 || exit $?
