#!/bin/bash
# Test infrastructure: resident-encode A/B of a variant library build (KPW_GPU_LIB) against the
# in-tree one, alternating, on the C2 and C4 workloads.
set -e
mkdir -p gpurun_out
V=${1:-tests/microbench/build/libvar/libkpw_sinkall.so}
for wl in c2 c4; do
  for r in 1 2; do
    timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > gpurun_out/libab_${wl}_base_$r.log 2>&1
    KPW_GPU_LIB=$V timeout -k 10 200 python3 tests/microbench/resident_only.py $wl > gpurun_out/libab_${wl}_var_$r.log 2>&1
  done
done
