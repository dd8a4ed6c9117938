#!/bin/bash
# r05am: every v1 column's page checks in speculative batches (KPW_PAGE_CUT_SPEC 1 / 0) — multi-page
# and rotation suites, then the bulk multi-page leg alternating
OUT=gpurun_out/r05am
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py \
  tests/test_gpu_rotation.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace.log 2>&1 || exit $?
for r in 1 2; do
  for p in 0 1; do
    KPW_PAGE_CUT_SPEC=$p timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/bmp_p${p}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k multipage > $OUT/pytest_full.log 2>&1 || exit $?
