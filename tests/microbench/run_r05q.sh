#!/bin/bash
# r05q: K7' GZIP with the segment-parallel parse and block-parallel bit streams: the GZIP parity
# tests, then writer timing at page sizes the tests do not reach, checked against the oracle
OUT=gpurun_out/r05q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "gzip" -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 120 python tests/microbench/gzip_leg.py 100000 > $OUT/gz100k.log 2>&1 || exit $?
timeout -k 10 300 python tests/microbench/gzip_leg.py 1000000 > $OUT/gz1m.log 2>&1 || exit $?
