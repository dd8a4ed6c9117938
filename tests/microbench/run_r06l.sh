#!/bin/bash
# r06l: bulk multi-page leg with the speculative horizon margin 25 / 12 / 6 % (KPW_MP_HORIZON_PCT),
# alternated twice, then the multi-page parity suite at 6 %
OUT=gpurun_out/r06l
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --steps 2 --warmup 1 --secondary-steps 3"
for r in 1 2; do
  for p in 25 12 6; do
    KPW_BENCH_LEGS=bulk_multipage KPW_MP_HORIZON_PCT=$p timeout -k 10 300 python3 bench.py $A > $OUT/bulk_p${p}_$r.json 2> $OUT/bulk_p${p}_$r.err || exit 1
  done
done
KPW_MP_HORIZON_PCT=6 timeout -k 10 900 python -u -m pytest tests/test_gpu_multipage.py -x -q --timeout 300 --timeout-method thread > $OUT/mp_tests.log 2>&1 || { tail -30 $OUT/mp_tests.log; exit 1; }
tail -1 $OUT/mp_tests.log
echo done
