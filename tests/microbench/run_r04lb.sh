#!/bin/bash
# r04lb: k_plan walker long runs per load round, 8 vs 16 (KPW_PLAN_PROF builds), resident C3
OUT=gpurun_out/r04lb
mkdir -p $OUT
for r in 1 2; do
  for v in pb8 pb16; do
    KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_$v.so timeout -k 10 200 python3 tests/microbench/resident_only.py c3 > $OUT/${v}_$r.log 2>&1 || exit $?
  done
done
