#!/bin/bash
# Test infrastructure: writer-path bench under several environment settings.
#   ENV_CFGS="tag1:VAR=1 VAR2=2;tag2:VAR=3" WLS="c2 c3" STEPS=6 bash tests/microbench/env_sweep.sh
# one log per (tag, workload) under gpurun_out/env_<tag>_<wl>.log
set -e
mkdir -p gpurun_out
IFS=';' read -ra CFGS <<< "${ENV_CFGS:?}"
for wl in ${WLS:-c2}; do
  for cfg in "${CFGS[@]}"; do
    tag=${cfg%%:*}; vars=${cfg#*:}
    env $vars timeout -k 10 300 python bench.py --workload $wl --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-resident --per-record-records 0 > gpurun_out/env_${tag}_${wl}.log 2>&1
  done
done
