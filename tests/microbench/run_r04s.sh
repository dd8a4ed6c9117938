#!/bin/bash
# r04s: K7 seg with the fragment in LDS (SG_HALF) vs the current kernel, on C2 / C3 / C4 pages.
OUT=gpurun_out/r04s
mkdir -p $OUT
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin > /dev/null
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin > /dev/null
python tests/microbench/dump_any.py 3 100000 /tmp/p3.bin > /dev/null
for k in 2 4 3; do
  for b in seg_bench seg_bench_half; do
    timeout -k 10 120 tests/microbench/build/$b /tmp/p$k.bin 3 > $OUT/${b}_c$k.log 2>&1 || exit $?
  done
done
