#!/bin/bash
# r05ac: K7 segment kernel sort as two stable radix passes (SG_RADIX=1) vs the counting sort with
# LDS atomics (seg_bench_cs): dumped C2/C3/C4 pages (byte identity checked by seg_bench), the
# parity suite, then the row-group-sized multi-page jobs on the bulk leg and the C2 line
OUT=gpurun_out/r05ac
mkdir -p $OUT
timeout -k 10 300 python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > $OUT/dump.log 2>&1 || exit $?
timeout -k 10 300 python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin >> $OUT/dump.log 2>&1 || exit $?
timeout -k 10 300 python tests/microbench/dump_any.py 3 100000 /tmp/p3.bin >> $OUT/dump.log 2>&1 || exit $?
for k in 2 3 4; do
  for b in seg_bench seg_bench_cs seg_bench seg_bench_cs; do
    timeout -k 10 120 tests/microbench/build/$b /tmp/p$k.bin 3 >> $OUT/seg_c${k}_$b.log 2>&1 || exit $?
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_multipage.py > $OUT/pytest.log 2>&1 || exit $?
KPW_TRACE=1 timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 1 > $OUT/trace.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python tests/microbench/bulk_mp_leg.py 100000000 2 > $OUT/leg_$r.log 2>&1 || exit $?
done
for w in c2 c4; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --workload $w --steps 4 --warmup 1 > $OUT/$w.json 2> $OUT/$w.err || exit $?
done
