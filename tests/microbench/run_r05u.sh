#!/bin/bash
# r05u: the full-size C2 file with GZIP, row group by row group against the oracle
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "c2_gzip" -x -v --timeout 800 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || exit $?
