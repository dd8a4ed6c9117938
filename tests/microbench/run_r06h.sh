#!/bin/bash
# r06h: C5 variance: stream sets created back to back (this tree), the stream -> hardware queue map
# of a C5 kernel trace, 16 hardware queues, and a shorter look-back spin
OUT=gpurun_out/r06h
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--workload c5 --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 5 --warmup 2"
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py $A > $OUT/c5_$r.json 2> $OUT/c5_$r.err || exit 1
done
for r in 1 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 bench.py $A > $OUT/c5_q16_$r.json 2> $OUT/c5_q16_$r.err || exit 1
  KPW_LB_SPIN=1024 timeout -k 10 300 python3 bench.py $A > $OUT/c5_spin1k_$r.json 2> $OUT/c5_spin1k_$r.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-resident --per-record-records 0 --per-record-64k-records 0 --secondary-steps 0 --steps 1 --warmup 1 > $OUT/tr.log 2>&1 || exit 1
python3 tests/microbench/queue_map.py $(find $OUT/tr -name "*kernel_trace.csv" | head -1) > $OUT/queue_map.txt
python3 tests/microbench/trace_busy.py $(find $OUT/tr -name "*kernel_trace.csv" | head -1) 10 > $OUT/busy.txt
find $OUT/tr -name "*kernel_trace.csv" -delete
echo done
