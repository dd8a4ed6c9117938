#!/bin/bash
# r05e: K7 GZIP (k_deflate.hip) parity on the GPU: the page parity suites over codec GZIP (v1 and
# v2), byte patterns, writer files
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "gzip" -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || exit $?
# C3 blit attribution: the engine's host <-> device table copies and the carried open row groups
KPW_TRACE=1 KPW_COPY_TRACE=1 timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --no-resident \
    --per-record-records 0 --secondary-steps 0 --steps 1 --warmup 1 > $OUT/c3_copies.log 2>&1 || exit $?
