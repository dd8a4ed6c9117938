#!/bin/bash
# r05ad: radix sort (bank-conflict-free counters, bucket starts from LDS) vs counting sort, seg_bench
OUT=gpurun_out/r05ad
mkdir -p $OUT
timeout -k 10 300 python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > $OUT/dump.log 2>&1 || exit $?
timeout -k 10 300 python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin >> $OUT/dump.log 2>&1 || exit $?
for k in 2 4; do
  for b in seg_bench_rx seg_bench; do
    timeout -k 10 120 tests/microbench/build/$b /tmp/p$k.bin 3 >> $OUT/seg_c${k}_$b.log 2>&1 || exit $?
  done
done
