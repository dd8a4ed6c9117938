#!/bin/bash
# Test infrastructure: A/B of the K7 segment kernel (build/seg_bench_base = a previous build,
# build/seg_bench = the working tree, build/seg_bench_<v> = -D variants) on dumped C2 / C3 / C4
# pages, from the repo root through gpurun.  seg_bench checks byte identity vs the oracle itself.
set -e
mkdir -p gpurun_out
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
python tests/microbench/dump_any.py 3 100000 /tmp/p3.bin
for k in 2 3 4; do
  for b in tests/microbench/build/seg_bench tests/microbench/build/seg_bench_*; do
    [ -x $b ] || continue
    v=$(basename $b)
    timeout -k 10 120 $b /tmp/p$k.bin 3 > gpurun_out/segab_c${k}_$v.log 2>&1
  done
done
