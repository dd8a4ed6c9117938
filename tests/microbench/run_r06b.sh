#!/bin/bash
# r06b: device encode gate (KPW_DEVICE_ENCODES) on C5 standalone: 2 / 3 / 4 / unlimited, with
# 8 and 16 hardware queues; concurrency parity tests; a traced C2 line (the close tail)
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrent.py tests/test_gpu_async_write.py "tests/test_gpu_fullsize.py::test_c5_concurrent_writers_full_size" -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for g in 2 3 4 0; do
  KPW_DEVICE_ENCODES=$g timeout -k 10 300 $B --workload c5 --steps 3 --warmup 1 > $OUT/c5_g$g.json 2> $OUT/c5_g$g.err || exit $?
done
KPW_DEVICE_ENCODES=2 GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --workload c5 --steps 3 --warmup 1 > $OUT/c5_g2_q16.json 2> $OUT/c5_g2_q16.err || exit $?
KPW_DEVICE_ENCODES=3 GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --workload c5 --steps 3 --warmup 1 > $OUT/c5_g3_q16.json 2> $OUT/c5_g3_q16.err || exit $?
timeout -k 10 300 $B --steps 5 --warmup 1 > $OUT/c2.json 2> $OUT/c2.err || exit $?
KPW_TRACE=1 timeout -k 10 300 $B --steps 2 --warmup 1 > $OUT/c2_tr.json 2> $OUT/c2_tr.err || exit $?
KPW_TRACE=1 KPW_DEVICE_ENCODES=2 timeout -k 10 300 $B --workload c5 --steps 2 --warmup 1 > $OUT/c5_g2_tr.json 2> $OUT/c5_g2_tr.err || exit $?
echo done
