#!/bin/bash
set -e
mkdir -p gpurun_out
for mb in 1024 2048 3072; do
  KPW_STAGE_FLUSH_MB=$mb timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/flush_$mb.log 2>&1
done
