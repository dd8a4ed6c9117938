#!/bin/bash
# r04fin: final round-4 build: the whole GPU suite (full-size C2 / C3 / C4 included) and the
# default bench line
OUT=gpurun_out/r04fin2
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
