#!/bin/bash
# r04w: folded planner evaluation (Q): GPU suite, planner profile, resident A/B against
# KPW_PLAN_FOLD=0 (same build).
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
for wl in c3 c2; do
  KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_pfold.so timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/pfold_${wl}.log 2>&1 || exit $?
done
for wl in c3 c2; do
  timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/res_${wl}.log 2>&1 || exit $?
  KPW_PLAN_FOLD=0 timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/nofold_${wl}.log 2>&1 || exit $?
done
