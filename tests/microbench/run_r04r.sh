#!/bin/bash
# r04r: the whole GPU suite (full size included) on the final round-4 engine changes, then
# the default bench line.
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
