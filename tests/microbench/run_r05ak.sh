#!/bin/bash
# r05ak: multi-page dictionary rounds doubling up to 4x (KPW_MP_ROUND_GROW 4 / 1) — multi-page and
# rotation suites, the bulk multi-page leg and the 64 KiB-page per-record loop, alternating
OUT=gpurun_out/r05ak
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py \
  tests/test_gpu_rotation.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace.log 2>&1 || exit $?
for r in 1 2; do
  for g in 1 4; do
    KPW_MP_ROUND_GROW=$g timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/bmp_g${g}_$r.log 2>&1 || exit $?
    KPW_MP_ROUND_GROW=$g timeout -k 10 300 python tests/microbench/pr_leg.py 600000 65536 > $OUT/pr64k_g${g}_$r.log 2>&1 || exit $?
  done
done
