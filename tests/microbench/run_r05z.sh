#!/bin/bash
# r05z: multi-page eager jobs while the workers are busy (KPW_MP_EAGER_QUEUE) on the 100 M bulk leg
OUT=gpurun_out/r05z
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace_q2.log 2>&1 || exit $?
for r in 1 2; do
  for q in 0 1 2; do
    KPW_MP_EAGER_QUEUE=$q timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/q${q}_$r.log 2>&1 || exit $?
  done
done
