#!/bin/bash
# r05ao: pooled HIP streams (KPW_STREAM_POOL 1 / 0) — writer suites, then C2 / C4 / C5 lines alternating
OUT=gpurun_out/r05ao
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_concurrent.py tests/test_gpu_async_write.py tests/test_gpu_faults.py tests/test_gpu_rotation.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload c2 --steps 2 --warmup 1 > $OUT/c2_trace.json 2> $OUT/c2_trace.log || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 4 --warmup 1"
for r in 1 2; do
  for p in 0 1; do
    for w in c2 c5; do
      KPW_STREAM_POOL=$p timeout -k 10 300 $B --workload $w > $OUT/${w}_p${p}_$r.json 2> $OUT/${w}_p${p}_$r.err || exit $?
    done
  done
done
