#!/bin/bash
# r05bf: round-5 final validation after the probe metadata change and the fallback guard — the whole GPU suite, smoke, the default bench line
OUT=gpurun_out/r05bf
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
