#!/bin/bash
# r05ae: speculative page-cut batches for REQUIRED BYTE_ARRAY columns (A/B on the bulk leg), then
# the checkpoint: the whole GPU suite, smoke, the default bench line
OUT=gpurun_out/r05ae
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multipage.py > $OUT/pytest_mp.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace_on.log 2>&1 || exit $?
KPW_TRACE=1 KPW_PAGE_CUT_SPEC=0 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace_off.log 2>&1 || exit $?
for r in 1 2; do
  KPW_PAGE_CUT_SPEC=0 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/off_$r.log 2>&1 || exit $?
  timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/on_$r.log 2>&1 || exit $?
done
timeout -k 10 1500 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
