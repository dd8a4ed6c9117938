#!/bin/bash
# Test infrastructure: k_snappy_v decision-budget sweep for the routed K7 pipeline (through gpurun).
set -e
mkdir -p gpurun_out
python tests/microbench/dump_any.py 1 2200000 /tmp/p2.bin
python tests/microbench/dump_any.py 2 300000 /tmp/p4.bin
for b in 256; do for sb in 32 128 512; do
  KPW_SNAPPY_SBUDGET=$sb KPW_SNAPPY_VBUDGET=$b timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p2.bin 1 8 > gpurun_out/bud_c2_$sb.log 2>&1
  KPW_SNAPPY_SBUDGET=$sb KPW_SNAPPY_VBUDGET=$b timeout -k 10 120 tests/microbench/build/seg_bench /tmp/p4.bin 1 4 > gpurun_out/bud_c4_$sb.log 2>&1
done; done
