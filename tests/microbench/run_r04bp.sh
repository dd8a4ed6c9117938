#!/bin/bash
# r04bp: the multi-page planners' checks and walks (KPW_PLAN_PROF build, device printf)
OUT=gpurun_out/r04bp
mkdir -p $OUT
KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_pmp.so timeout -k 10 300 python3 tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/bp.log 2>&1
