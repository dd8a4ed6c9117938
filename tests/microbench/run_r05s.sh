#!/bin/bash
# r05s: the driver's default bench line (with the gzip key)
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
