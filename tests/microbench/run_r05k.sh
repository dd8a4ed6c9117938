#!/bin/bash
# r05k: multi-page batches planned as a whole before their exact passes (the next job starts
# after the cuts, not after every exact pass) — multi-page / rotation / async suites, the bulk
# multi-page leg (20 M and 100 M records) and its writer trace
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_multipage.py tests/test_gpu_rotation.py tests/test_gpu_async_write.py \
    tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 2 > $OUT/leg20.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 600 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/leg100.log 2>&1 || exit $?
