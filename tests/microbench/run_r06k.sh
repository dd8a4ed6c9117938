#!/bin/bash
# r06k: C3 standalone vs as a secondary leg (allocator calls, phases, H2D rate), and one traced
# standalone C3 run (job timeline of the wide schema)
OUT=gpurun_out/r06k
mkdir -p $OUT
A="--no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py $A --workload c3 --secondary-steps 0 --steps 4 --warmup 1 > $OUT/c3_alone_$r.json 2> $OUT/c3_alone_$r.err || exit 1
  KPW_BENCH_LEGS=c3 timeout -k 10 300 python3 bench.py $A --steps 3 --warmup 1 > $OUT/c3_leg_$r.json 2> $OUT/c3_leg_$r.err || exit 1
done
KPW_TRACE=1 timeout -k 10 300 python3 bench.py $A --workload c3 --secondary-steps 0 --steps 2 --warmup 1 > $OUT/c3_tr.json 2> $OUT/c3_tr.err || exit 1
echo done
