#!/bin/bash
# r04i: K7 fml variants (seg_bench), the GPU suite minus the full-size tests, and a writer A/B
# of the pinned transfer arena (KPW_XFER) and the assembly D2H stream (KPW_ASM_D2H_STREAM).
OUT=gpurun_out/r04i
mkdir -p $OUT
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > /dev/null
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin > /dev/null
for b in tests/microbench/build/seg_bench*; do
  for k in 2 4; do timeout -k 10 120 $b /tmp/p$k.bin 3 > $OUT/seg_$(basename $b)_c$k.log 2>&1 || exit $?; done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fullsize" > $OUT/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in base xfer0 asm1; do
    E=""; [ $v = xfer0 ] && E="KPW_XFER=0"; [ $v = asm1 ] && E="KPW_ASM_D2H_STREAM=1"
    env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-resident --per-record-records 0 --secondary-steps 0 > $OUT/ab_${v}_$rep.log 2>&1 || exit $?
    grep -h '"value"' $OUT/ab_${v}_$rep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> $OUT/ab.txt
  done
done
