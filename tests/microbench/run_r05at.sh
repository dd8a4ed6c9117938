#!/bin/bash
# r05at: writer stream sets pooled whole — writer suites, then the bench line's legs with the pool
# on / off
OUT=gpurun_out/r05at
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_concurrent.py tests/test_gpu_async_write.py tests/test_gpu_faults.py tests/test_gpu_rotation.py > $OUT/pytest.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --steps 3 --warmup 1"
timeout -k 10 600 $B > $OUT/on1.json 2> $OUT/on1.err || exit $?
KPW_STREAM_POOL=0 timeout -k 10 600 $B > $OUT/off1.json 2> $OUT/off1.err || exit $?
timeout -k 10 600 $B > $OUT/on2.json 2> $OUT/on2.err || exit $?
