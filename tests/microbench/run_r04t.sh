#!/bin/bash
# r04t: where the C2 writer step goes now (KPW_TRACE, one step), and the eager-job threshold
# re-swept on the round-4 build (per-job GPU time dropped since r03's sweep).
OUT=gpurun_out/r04t
mkdir -p $OUT
KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/trace.log 2>&1 || exit $?
for rep in 1 2; do
  for mb in 256 384 512 768; do
    KPW_EAGER_MB=$mb timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/eager_$mb.log 2>&1 || exit $?
    grep -h '"value"' $OUT/eager_$mb.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('eager $mb', d['value'], d['ms_per_step'], d.get('encode_jobs_per_step'))" >> $OUT/eager.txt
  done
done
