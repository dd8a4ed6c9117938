#!/bin/bash
# r05bc: A/B of the multi-page metadata change (build_ab/ = the tree before it) on the bench's
# per-record legs, alternated on one box
OUT=gpurun_out/r05bc
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-resident --secondary-steps 0 --steps 1 --warmup 1"
for r in 1 2; do
  KPW_GPU_LIB=$PWD/build_ab/kafka-parquet-writer_amd/libkpw_gpu.so timeout -k 10 300 $B > $OUT/old_$r.json 2> $OUT/old_$r.err || exit $?
  timeout -k 10 300 $B > $OUT/new_$r.json 2> $OUT/new_$r.err || exit $?
done
