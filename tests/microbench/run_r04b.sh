#!/bin/bash
# r04b: the GPU suite, a traced C2 writer run, the default bench line.  From the repo root.
set -e
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/trace_c2.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
