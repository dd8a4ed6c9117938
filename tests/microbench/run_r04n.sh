#!/bin/bash
# r04n: the GPU suite (minus full size) on the probe changes (model page cuts, no planner
# inputs, cached cut pages), then the per-record loops with page cuts under KPW_TRACE.
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 3000000 1048576 > $OUT/pr_1m.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 300000 65536 > $OUT/pr_64k.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "reference_defaults or every_record_multipage" > $OUT/pytest_pr.log 2>&1 || exit $?
