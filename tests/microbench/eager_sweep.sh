#!/bin/bash
# Test infrastructure: C2 writer-path bench with eager job sizes (KPW_EAGER_MB) and job sizes
# (KPW_STAGE_FLUSH_MB); one log per setting under gpurun_out/.
set -e
mkdir -p gpurun_out
IFS=, read -ra CFGS <<< "${EAGER_CFGS:--1 1024,512 1024}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  KPW_EAGER_MB=$1 KPW_STAGE_FLUSH_MB=$2 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-resident --per-record-records 0 > gpurun_out/eager_$1_$2.log 2>&1
done
