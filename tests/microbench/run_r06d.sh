#!/bin/bash
# r06d: C5 with smaller eager jobs (KPW_EAGER_MB) and 8 / 16 hardware queues: the chip idles
# for the first ~40 ms of a C5 step until every writer holds 384 MiB (r06c busy profile)
OUT=gpurun_out/r06d
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0"
for q in 8 16; do
  for e in 384 256 192 128; do
    GPU_MAX_HW_QUEUES=$q KPW_EAGER_MB=$e timeout -k 10 300 python3 bench.py --workload c5 $A --steps 3 --warmup 1 > $OUT/c5_q${q}_e$e.json 2> $OUT/c5_q${q}_e$e.err || exit $?
  done
done
echo done
