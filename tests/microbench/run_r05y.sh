#!/bin/bash
# r05y: bulk multi-page leg at 100 M records, traced (job timeline + multi-page phases)
OUT=gpurun_out/r05y
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace100.log 2>&1 || exit $?
