#!/bin/bash
# r05ay: the look-back fallback with its in-place guard (re-check of the predecessor word after the recompute): forced-fallback parity, the parity suites, C5/C2 at 16 hardware queues
OUT=gpurun_out/r05ay
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lookback.py > $OUT/lookback.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multipage.py > $OUT/parity.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1"
for q in 16; do
  for w in c5 c2; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B --workload $w > $OUT/${w}_q${q}.json 2> $OUT/${w}_q${q}.err || exit $?
  done
done
