#!/bin/bash
# r05r: GZIP writer at 10 M records (multi-row-group file, 10-80 MB pages), checked against the oracle
OUT=gpurun_out/r05r
mkdir -p $OUT
timeout -k 10 600 python tests/microbench/gzip_leg.py 10000000 > $OUT/gz10m.log 2>&1 || exit $?
