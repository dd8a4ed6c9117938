#!/bin/bash
# r05w: multi-page splice (exact pass = each column's last page + dictionary page) — parity
# suites, then the bulk multi-page leg with the splice on / off
OUT=gpurun_out/r05w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py \
  tests/test_gpu_rotation.py tests/test_gpu_async_write.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace20.log 2>&1 || exit $?
for r in 1 2; do
  KPW_MP_SPLICE=0 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/off_$r.log 2>&1 || exit $?
  timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/on_$r.log 2>&1 || exit $?
done
