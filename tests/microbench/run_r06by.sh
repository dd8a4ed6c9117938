#!/bin/bash
# per-record loop at 64 KiB pages: the tree's library against the previous commit's (KPW_GPU_LIB), alternating
OUT=gpurun_out/r06by
mkdir -p $OUT
for r in 1 2 3; do
  for v in tree head; do
    if [ $v = tree ]; then L=""; else L="KPW_GPU_LIB=tests/microbench/build/libvar/lib_$v.so"; fi
    echo -n "$v " >> $OUT/pr.txt
    env $L timeout -k 10 120 python3 tests/microbench/pr_leg.py 1500000 65536 >> $OUT/pr.txt 2>&1 || exit 1
  done
done
cat $OUT/pr.txt
