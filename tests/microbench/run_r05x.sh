#!/bin/bash
# r05x: multi-page splice + lazy open row groups — parity suites, full-size 1 MiB-page C2, then
# per-phase traces and the bulk multi-page leg (lazy on / off)
OUT=gpurun_out/r05x
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py \
  tests/test_gpu_rotation.py tests/test_gpu_async_write.py > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py \
  -k multipage > $OUT/pytest_full.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/on.log 2>&1 || exit $?
KPW_TRACE=1 KPW_MP_LAZY=0 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/off.log 2>&1 || exit $?
for r in 1 2; do
  KPW_MP_LAZY=0 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/lazy0_$r.log 2>&1 || exit $?
  timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/lazy1_$r.log 2>&1 || exit $?
done
