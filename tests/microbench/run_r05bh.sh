#!/bin/bash
# r05bh: the whole GPU suite with eight hardware queues (bench.py's setting), then again with
# KPW_LB_SPIN=16 (look-backs fall back after 16 polls: the decoupled fallback under every test)
OUT=gpurun_out/r05bh
mkdir -p $OUT
GPU_MAX_HW_QUEUES=8 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/q8.log 2>&1 || exit $?
KPW_LB_SPIN=16 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/spin16.log 2>&1 || exit $?
