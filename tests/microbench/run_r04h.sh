#!/bin/bash
OUT=gpurun_out/r04h
mkdir -p $OUT
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > /dev/null
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin > /dev/null
for b in tests/microbench/build/seg_bench*; do
  for k in 2 4; do timeout -k 10 120 $b /tmp/p$k.bin 3 > $OUT/seg_$(basename $b)_c$k.log 2>&1 || exit $?; done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "multipage or rotation or v2 or fullsize or async" > $OUT/pytest_mp.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/mp_leg.py 10000000 1048576 3 > $OUT/mp_trace.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-resident --no-cpu-baseline --secondary-steps 0 --per-record-records 3000000 > $OUT/per_record.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mp_prof -o run -- python tests/microbench/mp_leg.py 10000000 1048576 2 > $OUT/mp_prof.log 2>&1
for v in 0 1 0 1; do
  KPW_ASM_D2H_STREAM=$v KPW_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/d2hab_$v.log 2>&1 || exit $?
  grep -h '"value"' $OUT/d2hab_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('d2h_stream=$v', d['value'], d['ms_per_step'])" >> $OUT/d2hab.txt
done
