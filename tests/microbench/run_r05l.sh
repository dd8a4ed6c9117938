#!/bin/bash
# r05l: the driver's default bench line on the current tree
OUT=gpurun_out/r05l
mkdir -p $OUT
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
