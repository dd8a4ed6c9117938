#!/bin/bash
# r05o: the whole GPU suite, smoke, and the driver's default bench line (with per_record_64k)
OUT=gpurun_out/r05o
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
