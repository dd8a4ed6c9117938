#!/bin/bash
# r05p: the cross-engine speculative-horizon hint (multi-page suites, bulk multi-page leg) and a
# kernel trace of the per-record loop at 64 KiB pages (where a size probe's time goes)
OUT=gpurun_out/r05p
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_multipage.py tests/test_gpu_rotation.py -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 600 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/leg100.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 20000000 1 > $OUT/trace20.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/pr_leg.py 600000 65536 > $OUT/pr64k_trace.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o pr64k -- python3 \
    tests/microbench/pr_leg.py 600000 65536 > $OUT/pr64k_prof.log 2>&1 || exit $?
