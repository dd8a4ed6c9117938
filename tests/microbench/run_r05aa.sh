#!/bin/bash
# r05aa: parallel boundary copy; multi-page eager queue 2 / 3 on the 100 M bulk leg; C2 line
OUT=gpurun_out/r05aa
mkdir -p $OUT
KPW_TRACE=1 KPW_MP_EAGER_QUEUE=3 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace_q3.log 2>&1 || exit $?
for r in 1 2; do
  for q in 2 3; do
    KPW_MP_EAGER_QUEUE=$q timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/q${q}_$r.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload c2 --steps 4 --warmup 1 > $OUT/c2.json 2> $OUT/c2.err || exit $?
