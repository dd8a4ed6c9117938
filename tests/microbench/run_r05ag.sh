#!/bin/bash
# r05ag: record lengths narrowed by a waiting worker (KPW_PREP_LENGTHS) — writer suites, the bulk
# multi-page leg and C2 / C5 lines with it on / off, alternating
OUT=gpurun_out/r05ag
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_multipage.py tests/test_gpu_rotation.py tests/test_gpu_async_write.py tests/test_gpu_concurrent.py \
  tests/test_gpu_faults.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace_bmp.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 3 --warmup 1"
for r in 1 2; do
  for p in 0 1; do
    KPW_PREP_LENGTHS=$p timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/bmp_p${p}_$r.log 2>&1 || exit $?
    KPW_PREP_LENGTHS=$p timeout -k 10 300 $B --workload c2 > $OUT/c2_p${p}_$r.json 2> $OUT/c2_p${p}_$r.err || exit $?
    KPW_PREP_LENGTHS=$p timeout -k 10 300 $B --workload c5 > $OUT/c5_p${p}_$r.json 2> $OUT/c5_p${p}_$r.err || exit $?
  done
done
