#!/bin/bash
# r05al: k_page_cuts per column (checks, walker steps, ticks) on the bulk multi-page leg (KPW_PLAN_PROF build)
OUT=gpurun_out/r05al
mkdir -p $OUT
KPW_GPU_LIB=tests/microbench/build/libvar/libkpw_pprof.so timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/pprof.log 2>&1 || exit $?
