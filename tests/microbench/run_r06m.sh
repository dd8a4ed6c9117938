#!/bin/bash
# r06m: three encode workers per writer (KPW_ENCODERS=3) against two on C3 / C2 / C4 / C5, paired,
# plus the writer parity tests at three workers
OUT=gpurun_out/r06m
mkdir -p $OUT
KPW_ENCODERS=3 timeout -k 10 900 python -u -m pytest tests/test_gpu_async_write.py tests/test_gpu_concurrent.py tests/test_gpu_faults.py "tests/test_gpu_parity.py::test_writer_file_identical" "tests/test_gpu_parity.py::test_writer_eager_jobs" -x -q --timeout 300 --timeout-method thread > $OUT/tests_e3.log 2>&1 || { tail -30 $OUT/tests_e3.log; exit 1; }
tail -1 $OUT/tests_e3.log
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for r in 1 2; do
  for e in 2 3; do
    KPW_ENCODERS=$e timeout -k 10 300 python3 bench.py $A --workload c3 --steps 4 --warmup 1 > $OUT/c3_e${e}_$r.json 2> $OUT/c3_e${e}_$r.err || exit 1
    KPW_ENCODERS=$e timeout -k 10 300 python3 bench.py $A --workload c2 --steps 8 --warmup 2 > $OUT/c2_e${e}_$r.json 2> $OUT/c2_e${e}_$r.err || exit 1
    KPW_ENCODERS=$e timeout -k 10 300 python3 bench.py $A --workload c4 --steps 3 --warmup 1 > $OUT/c4_e${e}_$r.json 2> $OUT/c4_e${e}_$r.err || exit 1
    KPW_ENCODERS=$e timeout -k 10 300 python3 bench.py $A --workload c5 --steps 4 --warmup 2 > $OUT/c5_e${e}_$r.json 2> $OUT/c5_e${e}_$r.err || exit 1
  done
done
echo done
