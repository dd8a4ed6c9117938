#!/bin/bash
# r05av: look-back decoupled fallback: the forced-fallback parity test, the look-back users'
# parity suites, then the hardware-queue sweep that exposed the cross-kernel wait (C5 at 8 / 16)
OUT=gpurun_out/r05av
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lookback.py > $OUT/lookback.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multipage.py > $OUT/parity.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1"
for q in 16 8 4; do
  for w in c5 c2; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B --workload $w > $OUT/${w}_q${q}.json 2> $OUT/${w}_q${q}.err || exit $?
  done
done
