#!/bin/bash
# r04v: planner profile (wall-clock per evaluation kind) before / after the LDS stream tables,
# then the GPU suite on the in-tree build (LDS tables).
OUT=gpurun_out/r04v
mkdir -p $OUT
for v in pprof pprof_lds; do
  for wl in c3 c2; do
    KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_$v.so timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > $OUT/${v}_${wl}.log 2>&1 || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
